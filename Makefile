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

DEV_HDRS  := $(wildcard $(CSRC)/device/*.hpp) $(CSRC)/scan_kernels.hpp include/khbsgs.h
# libkhbsgs: the C ABI (khbsgs.hip) + one translation unit per group of k_giant_scan instances, so
# `make -j` compiles the heavy kernels in parallel
HIP_SRCS  := $(CSRC)/khbsgs.hip $(CSRC)/k_bsgs.hip $(CSRC)/k_addr.hip $(CSRC)/k_baby.hip
HIP_OBJS  := $(patsubst $(CSRC)/%.hip,build/hip/%.o,$(HIP_SRCS))
HOST_SRCS := $(CSRC)/host/u256.cpp $(CSRC)/host/secp_host.cpp $(CSRC)/host/bloom_host.cpp \
             $(CSRC)/host/bsgs_host.cpp $(CSRC)/host/bsgs_files.cpp $(CSRC)/host/engine.cpp \
             $(CSRC)/host/address_host.cpp
HOST_HDRS := $(wildcard $(CSRC)/host/*.hpp) $(DEV_HDRS) include/khhost.h
HOST_OBJS := $(patsubst $(CSRC)/host/%.cpp,build/host/%.o,$(HOST_SRCS))

all: $(LIBDIR)/libkhbsgs.so $(LIBDIR)/libkhbsgs_f9.so $(LIBDIR)/libkhhost.so $(BINDIR)/keyhunt_amd $(BINDIR)/bsgsd_amd oracle

$(LIBDIR) $(BINDIR) build/host build/hip:
	mkdir -p $@

build/hip/%.o: $(CSRC)/%.hip $(DEV_HDRS) | build/hip
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(LIBDIR)/libkhbsgs.so: $(HIP_OBJS) | $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(HIP_OBJS)

# The same library with the gated scan in 9 x 29-bit limbs (KHB_F9WALK=1, device/fe29.hpp): an
# alternative build kept parity-tested (tests/test_gpu_f9walk.py); the product uses the 8 x 32 walk.
build/hip/%_f9.o: $(CSRC)/%.hip $(DEV_HDRS) | build/hip
	$(HIPCC) $(HIPFLAGS) -DKHB_F9WALK=1 -c -o $@ $<
$(LIBDIR)/libkhbsgs_f9.so: build/hip/khbsgs_f9.o build/hip/k_bsgs_f9.o build/hip/k_addr.o build/hip/k_baby.o | $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $^

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

# Kernel variants for A/B timing (tools/perf_variants.py); not used by the product.
VARIANTS := r2
variants: $(patsubst %,$(LIBDIR)/variants/libkhbsgs_%.so,$(VARIANTS))
$(LIBDIR)/variants/libkhbsgs_w%.so: $(HIP_SRCS) $(DEV_HDRS)
	mkdir -p $(LIBDIR)/variants
	$(HIPCC) $(HIPFLAGS) -DKHB_WAVES_PER_SIMD=$* -shared -o $@ $(HIP_SRCS)
$(LIBDIR)/variants/libkhbsgs_r%.so: $(HIP_SRCS) $(DEV_HDRS)
	mkdir -p $(LIBDIR)/variants
	$(HIPCC) $(HIPFLAGS) -DKHB_PROBE_BITS=$* -shared -o $@ $(HIP_SRCS)
$(LIBDIR)/variants/libkhbsgs_g%.so: $(HIP_SRCS) $(DEV_HDRS)
	mkdir -p $(LIBDIR)/variants
	$(HIPCC) $(HIPFLAGS) -DKHB_GSN_SCALAR=$* -shared -o $@ $(HIP_SRCS)
$(LIBDIR)/variants/libkhbsgs_m0s%.so: $(HIP_SRCS) $(DEV_HDRS)
	mkdir -p $(LIBDIR)/variants
	$(HIPCC) $(HIPFLAGS) -DKHB_MUL_IMPL=0 -DKHB_SQR_IMPL=$* -shared -o $@ $(HIP_SRCS)
$(LIBDIR)/variants/libkhbsgs_m1s%.so: $(HIP_SRCS) $(DEV_HDRS)
	mkdir -p $(LIBDIR)/variants
	$(HIPCC) $(HIPFLAGS) -DKHB_MUL_IMPL=1 -DKHB_SQR_IMPL=$* -shared -o $@ $(HIP_SRCS)
$(LIBDIR)/variants/libkhbsgs_m2s%.so: $(HIP_SRCS) $(DEV_HDRS)
	mkdir -p $(LIBDIR)/variants
	$(HIPCC) $(HIPFLAGS) -DKHB_MUL_IMPL=2 -DKHB_SQR_IMPL=$* -shared -o $@ $(HIP_SRCS)
$(LIBDIR)/variants/libkhbsgs_p%.so: $(HIP_SRCS) $(DEV_HDRS)
	mkdir -p $(LIBDIR)/variants
	$(HIPCC) $(HIPFLAGS) -DKHB_PROBE_MODE=$* -shared -o $@ $(HIP_SRCS)
.PHONY: variants
$(LIBDIR)/variants/libkhbsgs_q%.so: $(HIP_SRCS) $(DEV_HDRS)
	mkdir -p $(LIBDIR)/variants
	$(HIPCC) $(HIPFLAGS) -DKHB_PIPE=$* -shared -o $@ $(HIP_SRCS)
$(LIBDIR)/variants/libkhbsgs_b%.so: $(HIP_SRCS) $(DEV_HDRS)
	mkdir -p $(LIBDIR)/variants
	$(HIPCC) $(HIPFLAGS) -DKHB_BATCH=$* -shared -o $@ $(HIP_SRCS)
$(LIBDIR)/variants/libkhbsgs_f%.so: $(HIP_SRCS) $(DEV_HDRS)
	mkdir -p $(LIBDIR)/variants
	$(HIPCC) $(HIPFLAGS) -DKHB_FUSE=$* -shared -o $@ $(HIP_SRCS)
$(LIBDIR)/variants/libkhbsgs_c%.so: $(HIP_SRCS) $(DEV_HDRS)
	mkdir -p $(LIBDIR)/variants
	$(HIPCC) $(HIPFLAGS) -DKHB_LDSCOUNT=$* -shared -o $@ $(HIP_SRCS)
$(LIBDIR)/variants/libkhbsgs_n%.so: $(HIP_SRCS) $(DEV_HDRS)
	mkdir -p $(LIBDIR)/variants
	$(HIPCC) $(HIPFLAGS) -DKHB_NT=$* -shared -o $@ $(HIP_SRCS)
$(LIBDIR)/variants/libkhbsgs_x%.so: $(HIP_SRCS) $(DEV_HDRS)
	mkdir -p $(LIBDIR)/variants
	$(HIPCC) $(HIPFLAGS) -DKHB_RARE=$* -shared -o $@ $(HIP_SRCS)
$(LIBDIR)/variants/libkhbsgs_xf.so: $(HIP_SRCS) $(DEV_HDRS)
	mkdir -p $(LIBDIR)/variants
	$(HIPCC) $(HIPFLAGS) -DKHB_RARE_FORCE=1 -shared -o $@ $(HIP_SRCS)
$(LIBDIR)/variants/libkhbsgs_nonop.so: $(HIP_SRCS) $(DEV_HDRS)
	mkdir -p $(LIBDIR)/variants
	$(HIPCC) $(HIPFLAGS) -DKHB_NONOP=1 -shared -o $@ $(HIP_SRCS)
$(LIBDIR)/variants/libkhbsgs_h%.so: $(HIP_SRCS) $(DEV_HDRS)
	mkdir -p $(LIBDIR)/variants
	$(HIPCC) $(HIPFLAGS) -DKHB_GATE1=$* -shared -o $@ $(HIP_SRCS)
$(LIBDIR)/variants/libkhbsgs_gnt%.so: $(HIP_SRCS) $(DEV_HDRS)
	mkdir -p $(LIBDIR)/variants
	$(HIPCC) $(HIPFLAGS) -DKHB_GATE_NT=$* -shared -o $@ $(HIP_SRCS)
$(LIBDIR)/variants/libkhbsgs_dyn%.so: $(HIP_SRCS) $(DEV_HDRS)
	mkdir -p $(LIBDIR)/variants
	$(HIPCC) $(HIPFLAGS) -DKHB_DYN=$* -shared -o $@ $(HIP_SRCS)
$(LIBDIR)/variants/libkhbsgs_f9w%.so: $(HIP_SRCS) $(DEV_HDRS)
	mkdir -p $(LIBDIR)/variants
	$(HIPCC) $(HIPFLAGS) -DKHB_F9WALK=$* -shared -o $@ $(HIP_SRCS)
$(LIBDIR)/variants/libkhbsgs_cnv%.so: $(HIP_SRCS) $(DEV_HDRS)
	mkdir -p $(LIBDIR)/variants
	$(HIPCC) $(HIPFLAGS) -DKHB_CN_VOLATILE=$* -shared -o $@ $(HIP_SRCS)
$(LIBDIR)/variants/libkhbsgs_gs%.so: $(HIP_SRCS) $(DEV_HDRS)
	mkdir -p $(LIBDIR)/variants
	$(HIPCC) $(HIPFLAGS) -DKHB_GATE_SHR64=$* -shared -o $@ $(HIP_SRCS)
# -m address occupancy A/B: a whole libkhbsgs.so per setting, swapped in with LD_LIBRARY_PATH
$(LIBDIR)/variants/aw%/libkhbsgs.so: $(HIP_SRCS) $(DEV_HDRS)
	mkdir -p $(LIBDIR)/variants/aw$*
	$(HIPCC) $(HIPFLAGS) -DKHB_ADDR_WAVES_PER_SIMD=$* -shared -o $@ $(HIP_SRCS)
$(LIBDIR)/variants/ap%/libkhbsgs.so: $(HIP_SRCS) $(DEV_HDRS)
	mkdir -p $(LIBDIR)/variants/ap$*
	$(HIPCC) $(HIPFLAGS) -DKHB_ADDR_PAIR=1 -DKHB_ADDR_WAVES_PER_SIMD=$* -shared -o $@ $(HIP_SRCS)
$(LIBDIR)/variants/ge%/libkhbsgs.so: $(HIP_SRCS) $(DEV_HDRS)
	mkdir -p $(LIBDIR)/variants/ge$*
	$(HIPCC) $(HIPFLAGS) -DKHB_GATE_EARLY=$* -shared -o $@ $(HIP_SRCS)
