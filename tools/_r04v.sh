export TMPDIR=/tmp
O=gpurun_out/r04v; mkdir -p $O
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread > $O/t.log 2>&1; rc=$?
tail -3 $O/t.log; grep -E "^(E  .*(Error|outside)|FAILED)" $O/t.log | head -20; ok $rc || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5grid_prof -o run -- python tools/grid_bench.py --config c5 --reps 3 --no-oracle > $O/c5grid.log 2>&1 || exit $?; grep build_ms $O/c5grid.log | cut -c1-200
timeout -k 10 120 python tools/grid_bench.py > $O/grid.json 2>&1 || exit $?; tail -1 $O/grid.json | cut -c1-200
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || exit $?; tail -1 $O/bench.log | cut -c1-200
timeout -k 10 300 python bench.py --mode train > $O/train.json 2>&1 || exit $?; tail -1 $O/train.json | cut -c1-200
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > $O/bench_c5.log 2>&1 || exit $?; tail -1 $O/bench_c5.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/head_prof -o run -- python bench.py --no-cpu-baseline > $O/head_prof.log 2>&1 || exit $?
