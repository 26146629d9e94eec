export TMPDIR=/tmp
mkdir -p gpurun_out/abl
timeout -k 10 300 python -u -m pytest tests/test_gpu_x3.py tests/test_gpu_edge.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_x3.log 2>&1
REPS=2 bash tools/ab.sh noxcd
for N in default noxcd; do
  if [ $N = default ]; then L=""; else L=tools/_ablate/$N/libpnr.so; fi
  if [ -n "$L" ]; then export PNR_LIB=$L; else unset PNR_LIB; fi
  rm -rf gpurun_out/abl/f_$N
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/abl/f_$N -o run -- python tools/agg_bench.py --precision fp32h2 > gpurun_out/abl/f_$N.log 2>&1
done
true
