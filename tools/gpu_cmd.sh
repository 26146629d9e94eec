export TMPDIR=/tmp
mkdir -p gpurun_out/abl
for N in default prev tst; do
  if [ $N = default ]; then L=""; else L=tools/_ablate/$N/libpnr.so; fi
  if [ -n "$L" ]; then export PNR_LIB=$L; else unset PNR_LIB; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abl/$N -o run -- python tools/agg_bench.py --precision fp32h2 > gpurun_out/abl/$N.log 2>&1
done
true
