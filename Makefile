# Build of the MI355X approximate counter (gfx950).  `make` builds:
#   approx_counter_amd/lib/libapprox_counter_amd.so   C-ABI + HIP kernel (the hot path)
#   approx_counter_amd/lib/libac_host.so              host stages' C ABI (tests of the CLI's CPU stages)
#   approx_counter_amd/bin/adaptFinder                the drop-in CLI (host C++ + the C-ABI library)
#   oracle/_build/libac_oracle.so                     CPU oracle (tests only)
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 --offload-arch=$(ARCH) -fPIC -Wall
# wm_count: keep the queue-claim atomic a plain returning atomic (the optimizer's wave-aggregated
# form waits for the result at once, exposing the claim latency the kernel hides behind a window)
WM_FLAGS ?= -mllvm -amdgpu-atomic-optimizer-strategy=None
PKG := approx_counter_amd
CSRC := $(PKG)/csrc
LIBDIR := $(PKG)/lib
LIB := $(LIBDIR)/libapprox_counter_amd.so
OBJDIR := build/obj

DEV_SRC := $(CSRC)/wm_count.hip $(CSRC)/exact_count.hip $(CSRC)/capi.cpp $(CSRC)/host_pack.cpp
HDRS := include/approx_counter_amd.h include/approx_counter_amd_testing.h $(CSRC)/wm_count.h $(CSRC)/exact_count.h $(CSRC)/host_pack.h

CXX ?= g++
HOST_CXXFLAGS ?= -O3 -std=c++17 -fPIC -Wall -Wextra
HOSTDIR := $(CSRC)/host
HOST_SRC := $(HOSTDIR)/host_stages.cpp
HOST_HDRS := $(HOSTDIR)/host_stages.h include/approx_counter_host.h include/approx_counter_amd.h
HOSTLIB := $(LIBDIR)/libac_host.so
BINDIR := $(PKG)/bin
CLI := $(BINDIR)/adaptFinder

all: $(LIB) $(HOSTLIB) $(CLI) oracle

$(OBJDIR)/wm_count.o: $(CSRC)/wm_count.hip $(CSRC)/wm_tid_blocks.inc $(CSRC)/wm_window_loop.inc $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) $(WM_FLAGS) -Iinclude -I$(CSRC) -c $< -o $@

$(OBJDIR)/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -Iinclude -I$(CSRC) -c $< -o $@

$(OBJDIR)/capi.o: $(CSRC)/capi.cpp $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -x hip -Iinclude -I$(CSRC) -c $< -o $@

# host staging (worker pool + AVX2 packer): plain host C++, no device code
$(OBJDIR)/host_pack.o: $(CSRC)/host_pack.cpp $(CSRC)/host_pack.h
	@mkdir -p $(OBJDIR)
	$(CXX) $(HOST_CXXFLAGS) -c $< -o $@

$(LIB): $(OBJDIR)/wm_count.o $(OBJDIR)/exact_count.o $(OBJDIR)/capi.o $(OBJDIR)/host_pack.o
	@mkdir -p $(LIBDIR)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^ -pthread

$(HOSTLIB): $(HOST_SRC) $(HOSTDIR)/host_capi.cpp $(HOST_HDRS)
	@mkdir -p $(LIBDIR)
	$(CXX) $(HOST_CXXFLAGS) -Iinclude -I$(HOSTDIR) -shared -o $@ $(HOST_SRC) $(HOSTDIR)/host_capi.cpp

$(CLI): $(HOSTDIR)/adaptfinder.cpp $(HOST_SRC) $(HOST_HDRS) $(LIB)
	@mkdir -p $(BINDIR)
	$(CXX) $(HOST_CXXFLAGS) -Iinclude -I$(HOSTDIR) -o $@ $(HOSTDIR)/adaptfinder.cpp $(HOST_SRC) \
		-L$(LIBDIR) -lapprox_counter_amd -Wl,-rpath,'$$ORIGIN/../lib' -pthread

oracle:
	$(MAKE) -s -C oracle

asm: $(CSRC)/wm_count.hip $(CSRC)/wm_tid_blocks.inc $(CSRC)/wm_window_loop.inc $(HDRS)
	@mkdir -p build/asm
	$(HIPCC) $(HIPFLAGS) $(WM_FLAGS) -Iinclude -I$(CSRC) --cuda-device-only -S $< -o build/asm/wm_count.s

clean:
	rm -rf build $(LIBDIR) $(BINDIR) oracle/_build

.PHONY: all oracle asm clean
