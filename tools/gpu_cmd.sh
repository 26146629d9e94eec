export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_x3.py tests/test_gpu_render.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_x3.log 2>&1
REPS=2 bash tools/ab.sh head
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/aggst -o run -- python tools/agg_bench.py --precision fp32h2 > gpurun_out/aggst.log 2>&1
true
