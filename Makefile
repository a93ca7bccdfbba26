# Build everything in-tree (the .so/.bin travel to the GPU box with the repo snapshot).
#   make            -> keyhuntm1cpu_amd/lib/libkhbsgs.so (HIP, gfx950) + oracle/build/liboracle.so
HIPCC   ?= /opt/rocm/bin/hipcc
ARCH    ?= gfx950
PKG     := keyhuntm1cpu_amd
CSRC    := $(PKG)/csrc
LIBDIR  := $(PKG)/lib
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wno-unused-result -Wno-unused-value

DEV_HDRS := $(wildcard $(CSRC)/device/*.hpp) include/khbsgs.h

all: $(LIBDIR)/libkhbsgs.so oracle

$(LIBDIR):
	mkdir -p $@

$(LIBDIR)/libkhbsgs.so: $(CSRC)/khbsgs.hip $(DEV_HDRS) | $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(CSRC)/khbsgs.hip

oracle:
	$(MAKE) -s -C oracle

clean:
	rm -rf $(LIBDIR) oracle/build

.PHONY: all oracle clean
