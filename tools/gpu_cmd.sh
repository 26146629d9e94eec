export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_query.py tests/test_gpu_edge.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_q.log 2>&1
REPS=2 bash tools/ab.sh knn0
true
