export TMPDIR=/tmp
O=gpurun_out/r04f; mkdir -p $O
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_flagsets.py -m gpu -q --timeout 300 --timeout-method thread > $O/t.log 2>&1; rc=$?
tail -3 $O/t.log; grep -E "^E  .*(Error|outside)" $O/t.log | head -20; ok $rc || exit $rc
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > $O/bench_c5.log 2>&1 || exit $?
tail -1 $O/bench_c5.log | cut -c1-250
timeout -k 10 300 python tools/_var/run_timed.py > $O/timed.log 2>&1 || exit $?
grep KT= $O/timed.log
