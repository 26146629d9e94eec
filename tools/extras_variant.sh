#!/bin/bash
# Dev tool: libpnr variants with the x3 backward's block3.0 extras computed in
# k_pairs_bwd<true> (-DPNR_X3_EXTRAS_IN_KERNEL=1) plus extra defines, for the
# co-residency experiment of DESIGN.md section 10:
#   bash tools/extras_variant.sh <name> [-D...]  ->  tools/_var/libpnr_<name>.so
set -e
name=$1; shift
make -s -j8 pointnerf_amd/libpnr.so
mkdir -p tools/_var
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -std=c++17 -munsafe-fp-atomics -fvisibility=hidden -Iinclude \
  -DPNR_X3_EXTRAS_IN_KERNEL=1 "$@" -c pointnerf_amd/csrc/aggregate.hip -o tools/_var/aggregate_$name.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/_var/libpnr_$name.so \
  $(ls build/*.o | grep -v '/aggregate.o') tools/_var/aggregate_$name.o
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -munsafe-fp-atomics -Iinclude --cuda-device-only -S \
  -DPNR_X3_EXTRAS_IN_KERNEL=1 "$@" pointnerf_amd/csrc/aggregate.hip -o tools/_var/aggregate_$name.s
