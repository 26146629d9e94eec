export TMPDIR=/tmp
O=gpurun_out/skew; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_x3.py tests/test_gpu_render.py tests/test_gpu_graph.py -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -2 $O/t.log
PNR_SKEW_TRACE=1 PNR_LIB=tools/_ablate/trs/libpnr.so timeout -k 10 200 python tools/x3_trace.py > $O/trs.txt 2>&1 || { tail -5 $O/trs.txt; exit 1; }
cat $O/trs.txt
REPS=2 bash tools/ab.sh skew0
