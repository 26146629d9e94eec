export TMPDIR=/tmp
O=gpurun_out/q; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_query.py tests/test_gpu_flagsets.py tests/test_gpu_graph.py -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -2 $O/t.log
bash tools/ab_query.sh q qold qnew
