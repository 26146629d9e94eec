#!/bin/bash
# Dev tool: build libpnr.so into tools/_ablate/$1 with extra hipcc flags $2 (e.g. -DPNR_X3_SCHED=3).
set -e
cd "$(dirname "$0")/.."
d=tools/_ablate/$1; mkdir -p $d; objs=""
for f in pointnerf_amd/csrc/*.hip; do b=$(basename $f .hip); extra=""; if [ "$b" = query ] || [ "$b" = grid ]; then extra="-ffp-contract=off"; fi; if [ "$b" = aggregate_x3 ]; then extra="-fno-slp-vectorize"; fi
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -std=c++17 -munsafe-fp-atomics -Iinclude $extra $2 -c $f -o $d/$b.o & objs="$objs $d/$b.o"; done; wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $d/libpnr.so $objs
