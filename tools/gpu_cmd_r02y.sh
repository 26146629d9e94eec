#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/r02y; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_neural_render.py tests/test_gpu_api.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for v in base nf base nf; do
  if [ $v = base ]; then L=pointnerf_amd/libpnr.so; else L=tools/_ablate/$v/libpnr.so; fi
  PNR_LIB=$L timeout -k 10 300 python tools/nr_bench.py > $O/$v.json 2> $O/$v.err || { tail $O/$v.err; exit 1; }
  echo $v; tail -1 $O/$v.json
done
