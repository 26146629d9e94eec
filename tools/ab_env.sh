#!/bin/bash
# Dev tool: A/B of agg_bench between the in-tree libpnr.so and variants given as
# name=ENV_ASSIGNMENTS (the variant lib tools/_ablate/<name>/libpnr.so run with those env vars).
set -e
P=${PREC:-fp32h2}
for r in $(seq 1 ${REPS:-2}); do
  timeout -k 10 200 python tools/agg_bench.py --precision $P > gpurun_out/ab_cur_$r.json
  for spec in "$@"; do
    N=${spec%%=*}; E=${spec#*=}
    env $E PNR_LIB=tools/_ablate/$N/libpnr.so timeout -k 10 200 python tools/agg_bench.py --precision $P > gpurun_out/ab_${N}_$r.json
  done
done
