# Builds the product library, the synthetic packet generator and (via
# oracle/Makefile) the test oracle.  Everything is built in-tree so the .so
# files travel to the GPU box with the repo snapshot.
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
CC       ?= gcc
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-function \
            -mllvm -amdgpu-atomic-optimizer-strategy=None
CFLAGS   ?= -O2 -std=gnu11 -fPIC -Wall -Wextra -Wno-unused-parameter

PRODUCT := onload_amd/liboo_gpu_rx.so
PKTGEN  := onload_amd/liboo_pktgen.so
SHIM    := onload_amd/liboo_rx_poll.so
SRCS    := onload_amd/csrc/oo_rx_kernel.hip onload_amd/csrc/oo_rx_kernel_short.hip onload_amd/csrc/oo_rx_kernel_poll.hip \
           onload_amd/csrc/oo_table_kernel.hip \
           onload_amd/csrc/oo_gpu_rx.cpp onload_amd/csrc/oo_gpu_rx_group.cpp onload_amd/csrc/oo_rx_csum.cpp
HDRS    := include/oo_gpu_rx.h onload_amd/csrc/oo_rx_device.h

# Builds of the same kernels with other ring / extra-round / wave counts
# (distinct sonames: loaded beside the product in one process).  The kernel's
# static vmcnt waits are written in terms of these constants;
# tests/test_gpu_wait_variants.py runs parity on every build.
CHECK_VARIANTS := r6e4:-DOO_RX_RING=6,-DOO_RX_EXTRA=4 r8e2:-DOO_RX_RING=8,-DOO_RX_EXTRA=2 \
                  w1e0:-DOO_RX_WAVES=1,-DOO_RX_EXTRA=0 rb6:-DOO_RX_BODY_RING=6 \
                  rb12:-DOO_RX_BODY_RING=12
CHECKS := $(foreach v,$(CHECK_VARIANTS),build/check/liboo_gpu_rx_$(firstword $(subst :, ,$(v))).so)

all: $(PRODUCT) $(SHIM) $(PKTGEN) oracle tools/hbm_ceiling tools/ring_probe tools/poll_bench tools/poll_rtt $(CHECKS)

build/check/liboo_gpu_rx_%.so: $(SRCS) $(HDRS)
	@mkdir -p build/check
	$(HIPCC) $(HIPFLAGS) -Wno-pass-failed $(subst $(COMMA), ,$(word 2,$(subst :, ,$(filter $*:%,$(CHECK_VARIANTS))))) \
	  -shared -Wl,-soname,liboo_gpu_rx_$*.so -o $@ $(SRCS)
COMMA := ,

$(PRODUCT): $(SRCS) $(HDRS)
	$(HIPCC) $(HIPFLAGS) -shared -Wl,-soname,liboo_gpu_rx.so -o $@ $(SRCS) -ldl

# The batched ci_netif_poll_evq RX branch (plain C over the C ABI).
$(SHIM): src/shim/oo_rx_poll.c include/oo_rx_poll.h include/oo_gpu_rx.h $(PRODUCT)
	$(CC) $(CFLAGS) -Iinclude -shared -o $@ src/shim/oo_rx_poll.c \
	  -Lonload_amd -l:liboo_gpu_rx.so -Wl,-rpath,'$$ORIGIN'

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
	  $(HIPCC) $(HIPFLAGS) $$f -shared -Wl,-soname,liboo_gpu_rx.so -o build/var_$$n.so $(SRCS) || exit 1; done

clean:
	rm -f $(PRODUCT) $(SHIM) $(PKTGEN)
	$(MAKE) -C oracle clean

# Check-only: the ci_netif_poll_evq integration (integration/netif_event_gpu.c)
# compiled against the reference tree's own sources and headers (this
# container only; never shipped).
REF ?= /root/reference
check-integration: oracle
	mkdir -p build
	$(CC) -c -O2 -Wall -Werror '-DTRANSPORT_CONFIG_OPT_HDR=<ci/internal/transport_config_opt_cloud.h>' \
	  -Ioracle/_ref -I$(REF)/src/include -I$(REF)/src/lib/transport/ip \
	  -I$(REF)/src/lib/transport/common -I$(REF)/src/lib/ciul -I$(REF)/src/lib/citools \
	  -Iinclude -o build/netif_event_gpu.o integration/netif_event_gpu.c

.PHONY: all oracle asm clean variants check-integration

tools/poll_rtt: tools/poll_rtt.hip
	$(HIPCC) -O3 --offload-arch=$(ARCH) -o $@ $<

tools/hbm_ceiling: tools/hbm_ceiling.hip
	$(HIPCC) -O3 --offload-arch=$(ARCH) -o $@ $<

tools/ring_probe: tools/ring_probe.hip
	$(HIPCC) -O3 --offload-arch=$(ARCH) -o $@ $<

# The deployed call shape of the batched RX branch: a C
# caller of the shim, beside the oracle's per-event CPU loop.
tools/poll_bench: tools/poll_bench.c $(SHIM) $(PKTGEN) oracle include/oo_rx_poll.h
	$(CC) $(CFLAGS) -Iinclude -o $@ tools/poll_bench.c -Lonload_amd -l:liboo_rx_poll.so \
	  -l:liboo_gpu_rx.so -l:liboo_pktgen.so -Loracle -l:liboorx_oracle.so \
	  -Wl,-rpath,'$$ORIGIN/../onload_amd' -Wl,-rpath,'$$ORIGIN/../oracle'

