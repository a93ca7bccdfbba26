# Build everything in-tree (the .so / binaries travel to the GPU box with the repo snapshot).
#   keyhuntm1cpu_amd/lib/libkhbsgs.so   HIP giant-step library (gfx950), include/khbsgs.h
#   keyhuntm1cpu_amd/lib/libkhhost.so   C++ host engine, include/khhost.h
#   keyhuntm1cpu_amd/bin/keyhunt_amd    keyhunt-compatible CLI (-m bsgs, -m address, -m rmd160)
#   keyhuntm1cpu_amd/bin/bsgsd_amd      bsgsd-compatible TCP daemon
#   oracle/build/liboracle.so           test-only checker (oracle/Makefile)
HIPCC    ?= /opt/rocm/bin/hipcc
CXX      ?= g++
ARCH     ?= gfx950
PKG      := keyhuntm1cpu_amd
CSRC     := $(PKG)/csrc
LIBDIR   := $(PKG)/lib
BINDIR   := $(PKG)/bin
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wno-unused-result -Wno-unused-value
CXXFLAGS ?= -O3 -std=c++17 -fPIC -march=x86-64-v3 -Wall -Wextra -Wno-unused-function -Wno-unused-parameter -Wno-unknown-pragmas -pthread

DEV_HDRS  := $(wildcard $(CSRC)/device/*.hpp) $(CSRC)/scan_kernels.hpp $(CSRC)/check_kernel.hpp include/khbsgs.h
# libkhbsgs: the C ABI (khbsgs.hip) + one translation unit per group of k_giant_scan instances, so
# `make -j` compiles the heavy kernels in parallel
HIP_SRCS  := $(CSRC)/khbsgs.hip $(CSRC)/k_bsgs.hip $(CSRC)/k_addr.hip $(CSRC)/k_addr_e.hip $(CSRC)/k_baby.hip \
             $(CSRC)/k_check.hip
HIP_OBJS  := $(patsubst $(CSRC)/%.hip,build/hip/%.o,$(HIP_SRCS))
HOST_SRCS := $(CSRC)/host/u256.cpp $(CSRC)/host/secp_host.cpp $(CSRC)/host/bloom_host.cpp \
             $(CSRC)/host/bsgs_host.cpp $(CSRC)/host/bsgs_files.cpp $(CSRC)/host/engine.cpp \
             $(CSRC)/host/address_host.cpp
HOST_HDRS := $(wildcard $(CSRC)/host/*.hpp) $(DEV_HDRS) include/khhost.h
HOST_OBJS := $(patsubst $(CSRC)/host/%.cpp,build/host/%.o,$(HOST_SRCS))

all: $(LIBDIR)/libkhbsgs.so $(LIBDIR)/libkhhost.so $(BINDIR)/keyhunt_amd $(BINDIR)/bsgsd_amd oracle

$(LIBDIR) $(BINDIR) build/host build/hip:
	mkdir -p $@

build/hip/%.o: $(CSRC)/%.hip $(DEV_HDRS) | build/hip
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(LIBDIR)/libkhbsgs.so: $(HIP_OBJS) | $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(HIP_OBJS)

build/host/%.o: $(CSRC)/host/%.cpp $(HOST_HDRS) | build/host
	$(CXX) $(CXXFLAGS) -c -o $@ $<

$(LIBDIR)/libkhhost.so: $(HOST_OBJS) build/host/khhost_capi.o $(LIBDIR)/libkhbsgs.so
	$(CXX) $(CXXFLAGS) -shared -o $@ $(HOST_OBJS) build/host/khhost_capi.o -L$(LIBDIR) -lkhbsgs -Wl,-rpath,'$$ORIGIN'

CLI_OBJS := build/host/keyhunt_main.o build/host/keyhunt_address.o
$(BINDIR)/keyhunt_amd: $(HOST_OBJS) $(CLI_OBJS) $(LIBDIR)/libkhbsgs.so | $(BINDIR)
	$(CXX) $(CXXFLAGS) -o $@ $(HOST_OBJS) $(CLI_OBJS) -L$(LIBDIR) -lkhbsgs -Wl,-rpath,'$$ORIGIN/../lib'

$(BINDIR)/bsgsd_amd: $(HOST_OBJS) build/host/bsgsd_main.o $(LIBDIR)/libkhbsgs.so | $(BINDIR)
	$(CXX) $(CXXFLAGS) -o $@ $(HOST_OBJS) build/host/bsgsd_main.o -L$(LIBDIR) -lkhbsgs -Wl,-rpath,'$$ORIGIN/../lib'

oracle:
	$(MAKE) -s -C oracle

clean:
	rm -rf $(LIBDIR) $(BINDIR) build oracle/build

.PHONY: all oracle clean

# Timing-only A/B builds are not the product: tools/build_variant.sh <name> -DKEY=VAL writes
# lib/variants/libkhbsgs_<name>.so for tools/perf_variants.py.  No test loads them.
