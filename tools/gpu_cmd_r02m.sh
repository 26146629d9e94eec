#!/bin/bash
# Dev tool: training tests + train bench + rocprof stats of the training step.
export TMPDIR=/tmp
O=gpurun_out/r02m; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_backward.py tests/test_gpu_api.py tests/test_gpu_flagsets.py tests/test_gpu_neural_render.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 300 python bench.py --mode train --steps 20 --warmup 3 > $O/bench_x3.json 2> $O/bench_x3.err || exit 1
tail -1 $O/bench_x3.json | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/x3 -o run -- python bench.py --mode train --steps 20 --warmup 3 > $O/prof_x3.log 2>&1 || exit 1
