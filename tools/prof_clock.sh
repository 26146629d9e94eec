#!/bin/bash
# Dev tool: effective clock of the aggregate kernels (GRBM_GUI_ACTIVE per kernel vs its duration)
# for the default lib and each tools/_ablate/<N> variant given.  AGG_ARGS -> agg_bench.py.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/clk
for N in 0 "$@"; do
  if [ "$N" = 0 ]; then unset PNR_LIB; else export PNR_LIB=tools/_ablate/$N/libpnr.so; fi
  timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --kernel-trace --output-format csv \
    -d gpurun_out/clk/$N -o run -- python tools/agg_bench.py --reps 1 $AGG_ARGS > gpurun_out/clk/$N.log 2>&1
done
