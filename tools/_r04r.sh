export TMPDIR=/tmp
O=gpurun_out/r04r; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_backward.py tests/test_gpu_train_contract.py tests/test_gpu_api.py -q --timeout 250 --timeout-method thread > $O/t.log 2>&1; tail -2 $O/t.log; grep -E "^(E  .*(Error|outside)|FAILED)" $O/t.log | head -20
timeout -k 10 300 python bench.py --mode train > $O/train.json 2>&1 || exit $?; tail -1 $O/train.json | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/train_prof -o run -- python bench.py --mode train --steps 6 --warmup 3 --no-cpu-baseline > $O/train_prof.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5grid_prof -o run -- python tools/grid_bench.py --config c5 --reps 3 --no-oracle > $O/c5grid.log 2>&1 || exit $?; tail -1 $O/c5grid.log
