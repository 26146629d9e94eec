#!/bin/bash
# Dev tool: build libpnr.so variants with PNR_ABLATE=N into tools/_ablate/N/.
set -e
cd "$(dirname "$0")/.."
for N in "$@"; do
  mkdir -p tools/_ablate/$N
  objs=""
  for f in pointnerf_amd/csrc/*.hip; do
    b=$(basename $f .hip)
    extra=""
    if [ "$b" = query ] || [ "$b" = grid ]; then extra="-ffp-contract=off"; fi
    if [ "$b" = aggregate_x3 ]; then extra="-fno-slp-vectorize"; fi
    /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -std=c++17 -munsafe-fp-atomics -Iinclude $extra \
      -DPNR_ABLATE=$N -c $f -o tools/_ablate/$N/$b.o &
    objs="$objs tools/_ablate/$N/$b.o"
  done
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/_ablate/$N/libpnr.so $objs
done
