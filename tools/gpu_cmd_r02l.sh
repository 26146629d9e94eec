#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/r02l; mkdir -p $O
for v in base wm4 wm2; do
  if [ $v = base ]; then L=pointnerf_amd/libpnr.so; else L=tools/_ablate/$v/libpnr.so; fi
  PNR_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python tools/gemm_nn_bench.py > $O/$v.json 2>&1 || exit 1
  echo $v; grep gemm_nn $O/$v/run_kernel_stats.csv | cut -d, -f1-4
done
