#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/r02k; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_backward.py -x -q --timeout 120 --timeout-method thread -k "gemm" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/nn -o run -- python tools/gemm_nn_bench.py > $O/nn.json 2>&1 || exit 1
grep gemm_nn $O/nn/run_kernel_stats.csv | cut -d, -f1-4
grep -i "Cijk" $O/nn/run_kernel_stats.csv | cut -d, -f2-4
timeout -k 10 300 python bench.py --mode train --steps 20 --warmup 3 > $O/bench_x3.json 2> $O/bench_x3.err || exit 1
tail -1 $O/bench_x3.json | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/x3 -o run -- python bench.py --mode train --steps 20 --warmup 3 > $O/prof_x3.log 2>&1 || exit 1
grep gemm_nn $O/x3/run_kernel_stats.csv | cut -d, -f1-4
