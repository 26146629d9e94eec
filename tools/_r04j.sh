export TMPDIR=/tmp
O=gpurun_out/r04j; mkdir -p $O
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_backward.py -k "gemm or absmax" -m gpu -q --timeout 120 --timeout-method thread > $O/t0.log 2>&1; rc=$?
tail -3 $O/t0.log; grep -E "^(E  .*(Error|outside)|FAILED)" $O/t0.log | head -20; ok $rc || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_backward.py tests/test_gpu_train_contract.py tests/test_gpu_dist.py -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread > $O/t.log 2>&1; rc=$?
tail -3 $O/t.log; grep -E "^(E  .*(Error|outside)|FAILED)" $O/t.log | head -20; ok $rc || exit $rc
for TP in fp32x3 fp32h2; do timeout -k 10 300 python bench.py --mode train --train-precision $TP > $O/train_$TP.json 2>&1 || exit $?; tail -1 $O/train_$TP.json | cut -c1-200; done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/train_trace -o run -- python bench.py --mode train --train-precision fp32h2 --steps 6 --warmup 3 --no-cpu-baseline > $O/train_trace.log 2>&1 || exit $?
