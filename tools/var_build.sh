#!/bin/bash
# Dev tool: a libpnr variant with one source rebuilt under extra defines:
#   bash tools/var_build.sh <name> <csrc file stem> [-D...]  ->  tools/_var/libpnr_<name>.so
set -e
name=$1; stem=$2; shift 2
make -s -j8 pointnerf_amd/libpnr.so
mkdir -p tools/_var
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -std=c++17 -munsafe-fp-atomics -fvisibility=hidden -Iinclude \
  "$@" -c pointnerf_amd/csrc/$stem.hip -o tools/_var/${stem}_$name.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/_var/libpnr_$name.so \
  $(ls build/*.o | grep -v "/$stem.o") tools/_var/${stem}_$name.o
