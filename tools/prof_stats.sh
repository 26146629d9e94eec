#!/bin/bash
# Dev tool: rocprofv3 kernel-trace stats over tools/agg_bench.py.
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/stats}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python tools/agg_bench.py --reps 2 $AGG_ARGS > $OUT/run.log 2>&1
find $OUT -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
