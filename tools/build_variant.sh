#!/bin/bash
# Dev tool: build a libpnr.so variant with extra -D flags into tools/_ablate/<name>/.
#   tools/build_variant.sh <name> "-DFOO=1 -DBAR=2"
set -e
cd "$(dirname "$0")/.."
N=$1; shift
D="$*"
mkdir -p tools/_ablate/$N
objs=""
for f in pointnerf_amd/csrc/*.hip; do
  b=$(basename $f .hip)
  extra=""
  if [ "$b" = query ] || [ "$b" = grid ] || [ "$b" = voxelize ]; then extra="-ffp-contract=off"; fi
  if [ "$b" = aggregate_x3 ]; then extra="-fno-slp-vectorize"; fi
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -std=c++17 -munsafe-fp-atomics -Iinclude $extra $D \
    -c $f -o tools/_ablate/$N/$b.o &
  objs="$objs tools/_ablate/$N/$b.o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/_ablate/$N/libpnr.so $objs
