export TMPDIR=/tmp
mkdir -p gpurun_out
REPS=2 bash tools/ab.sh sp3
PNR_LIB=tools/_ablate/sp3t/libpnr.so timeout -k 10 300 python tools/x3_trace.py > gpurun_out/trace_sp3.log 2>&1
