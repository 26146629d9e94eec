export TMPDIR=/tmp
O=gpurun_out/r04u; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_query.py tests/test_gpu_scale.py tests/test_gpu_edge.py -q -x --timeout 250 --timeout-method thread > $O/t.log 2>&1; tail -2 $O/t.log; grep -E "^(E  .*(Error|outside)|FAILED)" $O/t.log | head -20
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5grid_prof -o run -- python tools/grid_bench.py --config c5 --reps 3 --no-oracle > $O/c5grid.log 2>&1 || exit $?; grep build_ms $O/c5grid.log | cut -c1-200
