export TMPDIR=/tmp
O=gpurun_out/r04e; mkdir -p $O
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 240 python tools/_dbg/bk.py > $O/bk.log 2>&1; rc=$?; tail -8 $O/bk.log; ok $rc || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread > $O/t.log 2>&1; rc=$?
tail -5 $O/t.log; grep -E "^E  .*(Error|outside)" $O/t.log | head -20; ok $rc || exit $rc
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | cut -c1-300
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > $O/bench_c5.log 2>&1 || exit $?
tail -1 $O/bench_c5.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5stats -o run -- python bench.py --config c5 --no-cpu-baseline --steps 8 --warmup 2 > $O/c5stats.log 2>&1 || exit $?
