#!/bin/bash
# Dev tool: rocprofv3 kernel stats of bench.py --mode train (fp32x3 and native fp32
# training paths) into gpurun_out/$1/{x3,fp32}, plus plain timed runs.
export TMPDIR=/tmp
O=gpurun_out/${1:-ptrain}; mkdir -p $O
timeout -k 10 300 python bench.py --mode train --steps 20 --warmup 3 > $O/bench_x3.json 2> $O/bench_x3.err || exit 1
timeout -k 10 300 python bench.py --mode train --steps 20 --warmup 3 --train-precision fp32 > $O/bench_fp32.json 2> $O/bench_fp32.err || exit 1
for p in fp32x3 fp32; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$p -o run -- python bench.py --mode train --steps 20 --warmup 3 --train-precision $p > $O/prof_$p.log 2>&1 || exit 1
done
