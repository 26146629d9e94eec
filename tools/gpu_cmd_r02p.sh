#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/r02p; mkdir -p $O
for v in base cabl1 cabl2 cabl4 cabl7; do
  if [ $v = base ]; then L=pointnerf_amd/libpnr.so; else L=tools/_ablate/$v/libpnr.so; fi
  PNR_LIB=$L timeout -k 10 300 python tools/nr_bench.py > $O/$v.json 2> $O/$v.err || { tail $O/$v.err; exit 1; }
  echo $v; head -1 $O/$v.json
done
