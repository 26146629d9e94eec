export TMPDIR=/tmp
O=gpurun_out/r04b; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_train_contract.py tests/test_gpu_bf16.py -m gpu -v --timeout 300 --timeout-method thread > $O/t_contract.log 2>&1; rc=$?
tail -5 $O/t_contract.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --deselect tests/test_gpu_train_contract.py --deselect tests/test_gpu_bf16.py > $O/t_all.log 2>&1; rc2=$?
tail -5 $O/t_all.log
[ $rc2 -gt 1 ] && exit $rc2
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
timeout -k 10 400 python bench.py --config c5 --steps 5 --warmup 2 > $O/bench_c5.json 2> $O/bench_c5.err || { tail -5 $O/bench_c5.err; exit 1; }
cut -c1-300 $O/bench_c5.json
