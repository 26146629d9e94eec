#!/bin/bash
# Dev tool: libpnr variant with k_pairs_h2s phase stamps (-DPNR_H2S_TRACE) for tools/h2s_trace.py
set -e
make -s -j8
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -std=c++17 -munsafe-fp-atomics -fvisibility=hidden -Iinclude \
  -fno-slp-vectorize -DPNR_H2S_TRACE -c pointnerf_amd/csrc/aggregate_x3.hip -o tools/_var/aggregate_x3_trace.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/_var/libpnr_trace.so \
  $(ls build/*.o | grep -v aggregate_x3.o) tools/_var/aggregate_x3_trace.o
