#!/bin/bash
# Dev tool: A/B timing on one box: agg_bench with the in-tree libpnr.so and with
# each tools/_ablate/<name>/libpnr.so given, interleaved ($REPS rounds).
set -e
P=${PREC:-fp32h2}
for r in $(seq 1 ${REPS:-2}); do
  timeout -k 10 200 python tools/agg_bench.py --precision $P > gpurun_out/ab_cur_$r.json
  for N in "$@"; do PNR_LIB=tools/_ablate/$N/libpnr.so timeout -k 10 200 python tools/agg_bench.py --precision $P > gpurun_out/ab_${N}_$r.json; done
done
