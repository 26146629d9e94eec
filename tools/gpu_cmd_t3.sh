#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/t3; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_pack.py tests/test_gpu_backward.py tests/test_gpu_query.py tests/test_gpu_flagsets.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || exit 1
bash tools/prof_train.sh t3 || exit 1
timeout -k 10 300 python tools/query_bench.py --reps 5 > $O/query.json || exit 1
