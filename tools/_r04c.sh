export TMPDIR=/tmp
O=gpurun_out/r04c; mkdir -p $O
timeout -k 10 240 python tools/_dbg/bk.py > $O/bk.log 2>&1; cat $O/bk.log | tail -12
timeout -k 10 600 python -u -m pytest tests/test_gpu_train_contract.py tests/test_gpu_query.py -m gpu -v --timeout 300 --timeout-method thread > $O/t.log 2>&1; tail -5 $O/t.log
grep -E "^E  .*(Error|outside)" $O/t.log | head -20
