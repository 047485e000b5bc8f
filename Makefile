# Build of the MI355X approximate counter (gfx950).  `make` builds:
#   approx_counter_amd/lib/libapprox_counter_amd.so   C-ABI + HIP kernel
#   oracle/_build/libac_oracle.so                     CPU oracle (tests only)
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 --offload-arch=$(ARCH) -fPIC -Wall
PKG := approx_counter_amd
CSRC := $(PKG)/csrc
LIBDIR := $(PKG)/lib
LIB := $(LIBDIR)/libapprox_counter_amd.so
OBJDIR := build/obj

DEV_SRC := $(CSRC)/wm_count.hip $(CSRC)/capi.cpp
HDRS := include/approx_counter_amd.h $(CSRC)/wm_count.h

all: $(LIB) oracle

$(OBJDIR)/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -Iinclude -I$(CSRC) -c $< -o $@

$(OBJDIR)/capi.o: $(CSRC)/capi.cpp $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -x hip -Iinclude -I$(CSRC) -c $< -o $@

$(LIB): $(OBJDIR)/wm_count.o $(OBJDIR)/capi.o
	@mkdir -p $(LIBDIR)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^

oracle:
	$(MAKE) -s -C oracle

asm: $(CSRC)/wm_count.hip $(HDRS)
	@mkdir -p build/asm
	$(HIPCC) $(HIPFLAGS) -Iinclude -I$(CSRC) --cuda-device-only -S $< -o build/asm/wm_count.s

clean:
	rm -rf build $(LIBDIR) oracle/_build

.PHONY: all oracle asm clean
