export TMPDIR=/tmp
mkdir -p gpurun_out/abl
timeout -k 10 300 python -u -m pytest tests/test_gpu_query.py tests/test_gpu_edge.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_q.log 2>&1
for N in default knnnox; do
  if [ $N = default ]; then L=""; else L=tools/_ablate/$N/libpnr.so; fi
  if [ -n "$L" ]; then export PNR_LIB=$L; else unset PNR_LIB; fi
  rm -rf gpurun_out/abl/$N
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abl/$N -o run -- python tools/agg_bench.py --precision fp32h2 > gpurun_out/abl/$N.log 2>&1
done
true
