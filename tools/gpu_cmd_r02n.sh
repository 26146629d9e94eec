#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/r02n; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_neural_render.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 300 python tools/nr_bench.py > $O/nr.json 2> $O/nr.err || { tail $O/nr.err; exit 1; }
cat $O/nr.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/nr -o run -- python tools/nr_bench.py > $O/nr_prof.log 2>&1 || exit 1
grep -E "k_conv|k_nr|k_sum|Conv|conv|igemm|MIOpen" $O/nr/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-150
