#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/r02s; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_backward.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for v in base w8; do
  if [ $v = base ]; then L=pointnerf_amd/libpnr.so; else L=tools/_ablate/$v/libpnr.so; fi
  PNR_LIB=$L timeout -k 10 200 python tools/gemm_bench.py > $O/g_$v.json 2>&1 || exit 1
  echo $v; tail -1 $O/g_$v.json
  PNR_LIB=$L timeout -k 10 300 python bench.py --mode train --steps 20 --warmup 3 > $O/b_$v.json 2> $O/b_$v.err || exit 1
  tail -1 $O/b_$v.json | cut -c150-260
done
