#!/bin/bash
# Dev tool: training-path GPU tests + train bench (fp32x3 default and native fp32).
export TMPDIR=/tmp
O=gpurun_out/train; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_backward.py tests/test_gpu_api.py tests/test_gpu_flagsets.py -x -v --timeout 120 --timeout-method thread > $O/t.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --mode train > $O/bench_x3.json 2> $O/bench_x3.err || exit 1
timeout -k 10 300 python bench.py --mode train --train-precision fp32 > $O/bench_fp32.json 2> $O/bench_fp32.err || exit 1
