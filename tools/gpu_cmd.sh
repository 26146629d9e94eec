export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_x3.py tests/test_gpu_edge.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_x3.log 2>&1
REPS=2 bash tools/ab.sh head
PNR_LIB=tools/_ablate/trace/libpnr.so timeout -k 10 200 python tools/x3_trace.py > gpurun_out/trace_dyn.txt 2>&1
true
