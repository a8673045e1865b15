# Builds the product library, the synthetic packet generator and (via
# oracle/Makefile) the test oracle.  Everything is built in-tree so the .so
# files travel to the GPU box with the repo snapshot.
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
CC       ?= gcc
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-function
CFLAGS   ?= -O2 -std=gnu11 -fPIC -Wall -Wextra -Wno-unused-parameter

PRODUCT := onload_amd/liboo_gpu_rx.so
PKTGEN  := onload_amd/liboo_pktgen.so
SRCS    := onload_amd/csrc/oo_rx_kernel.hip onload_amd/csrc/oo_table_kernel.hip \
           onload_amd/csrc/oo_gpu_rx.cpp onload_amd/csrc/oo_rx_csum.cpp
HDRS    := include/oo_gpu_rx.h onload_amd/csrc/oo_rx_device.h

all: $(PRODUCT) $(PKTGEN) oracle tools/hbm_ceiling

$(PRODUCT): $(SRCS) $(HDRS)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(SRCS)

$(PKTGEN): onload_amd/csrc/oo_pktgen.c onload_amd/csrc/oo_pktgen.h include/oo_gpu_rx.h
	$(CC) $(CFLAGS) -shared -o $@ onload_amd/csrc/oo_pktgen.c -lm -lpthread

oracle:
	$(MAKE) -C oracle

asm: $(SRCS) $(HDRS)
	mkdir -p build
	$(HIPCC) $(HIPFLAGS) --offload-device-only -S -o build/oo_rx_kernel.s onload_amd/csrc/oo_rx_kernel.hip \
	  -Rpass-analysis=kernel-resource-usage 2> build/resource-usage.txt

# Tuning variants of the product library (build/var_<name>.so), selected at
# run time with OO_RX_LIB=<path> (tools/sweep.sh); not part of `all`.
VARIANTS ?= sp4:-DOO_RX_SP=4 sp8:-DOO_RX_SP=8
variants: $(SRCS) $(HDRS)
	mkdir -p build
	for v in $(VARIANTS); do n=$${v%%:*}; f=$$(echo "$${v#*:}" | tr ',' ' '); \
	  $(HIPCC) $(HIPFLAGS) $$f -shared -o build/var_$$n.so $(SRCS) || exit 1; done

clean:
	rm -f $(PRODUCT) $(PKTGEN)
	$(MAKE) -C oracle clean

.PHONY: all oracle asm clean variants

tools/hbm_ceiling: tools/hbm_ceiling.hip
	$(HIPCC) -O3 --offload-arch=$(ARCH) -o $@ $<
