# libpnr.so: the MI355X (gfx950) Point-NeRF hot path behind include/pnr.h.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
SRC_DIR := pointnerf_amd/csrc
SRCS := $(wildcard $(SRC_DIR)/*.hip)
OBJS := $(patsubst $(SRC_DIR)/%.hip,build/%.o,$(SRCS))
LIB := pointnerf_amd/libpnr.so
HIPFLAGS := -O3 --offload-arch=$(ARCH) -fPIC -std=c++17 -Wall -Wno-unused-result \
            -munsafe-fp-atomics -fvisibility=hidden -Iinclude

all: $(LIB) oracle

build/%.o: $(SRC_DIR)/%.hip $(SRC_DIR)/pnr_common.h $(SRC_DIR)/agg_common.h include/pnr.h
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# The query kernels must round exactly like the reference's fp32 ops: no FMA contraction.
build/query.o build/grid.o build/voxelize.o: HIPFLAGS += -ffp-contract=off
# The bf16 pair kernel's gather math (weights, distances, PE) without FMA
# contraction: its render and general instantiations then round every fp32 op
# the same way, so their features agree bit for bit (test_gpu_bf16.py).
build/aggregate_bf16.o: HIPFLAGS += -ffp-contract=off
# Split-MFMA kernels: no SLP packing of scalar f32 math into v_pk_*_f32, which
# issues at a fraction of the rate of scalar VALU beside the MFMA stream
# (MI355X_MICROARCH "price of one filler"; measured 1 % on the aggregate).
build/aggregate_x3.o: HIPFLAGS += -fno-slp-vectorize

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS)

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf build $(LIB)
	$(MAKE) -C oracle clean

.PHONY: all clean oracle
