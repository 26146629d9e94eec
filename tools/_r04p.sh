export TMPDIR=/tmp
O=gpurun_out/r04p; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_query.py tests/test_gpu_edge.py tests/test_gpu_flagsets.py -q -x --timeout 120 --timeout-method thread > $O/tq.log 2>&1 || { tail -30 $O/tq.log; exit 1; }
tail -1 $O/tq.log
timeout -k 10 120 python tools/grid_bench.py > $O/grid.json 2>&1 || exit $?; tail -1 $O/grid.json
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/grid_prof -o run -- python tools/grid_bench.py --reps 5 > $O/grid_prof.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_checkpoint.py -q --timeout 250 --timeout-method thread > $O/t.log 2>&1; tail -2 $O/t.log; grep -E "^(E  .*(Error|outside)|FAILED)" $O/t.log | head -20
