#!/bin/bash
# Dev tool: train bench (20 steps) + rocprofv3 kernel stats of the fp32x3 training step.
export TMPDIR=/tmp
O=gpurun_out/r02j; mkdir -p $O
timeout -k 10 300 python bench.py --mode train --steps 20 --warmup 3 > $O/bench_x3.json 2> $O/bench_x3.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/x3 -o run -- python bench.py --mode train --steps 20 --warmup 3 > $O/prof_x3.log 2>&1 || exit 1
tail -1 $O/bench_x3.json
