export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_x3.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_x3.log 2>&1
