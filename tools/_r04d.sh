export TMPDIR=/tmp
O=gpurun_out/r04d; mkdir -p $O
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 240 python tools/_dbg/bk.py > $O/bk.log 2>&1; rc=$?; tail -8 $O/bk.log; ok $rc || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_train_contract.py tests/test_gpu_bf16.py -m gpu -q --timeout 300 --timeout-method thread > $O/t.log 2>&1; rc=$?
tail -5 $O/t.log; grep -E "^E  .*(Error|outside)" $O/t.log | head -20; ok $rc || exit $rc
CONFIG=c5 STEPS=10 WARMUP=3 timeout -k 10 600 bash tools/prof_bench.sh r04_c5 > $O/prof_c5.log 2>&1; rc=$?; tail -5 $O/prof_c5.log; [ $rc -eq 0 ] || exit $rc
for TP in fp32x3 fp32h2; do timeout -k 10 300 python bench.py --mode train --train-precision $TP > $O/train_$TP.json 2>&1 || exit $?; tail -1 $O/train_$TP.json | cut -c1-300; done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/train_trace -o run -- python bench.py --mode train --train-precision fp32h2 --steps 6 --warmup 3 --no-cpu-baseline > $O/train_trace.log 2>&1 || exit $?

