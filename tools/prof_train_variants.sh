#!/bin/bash
# Dev tool: k_pairs_bwd / training kernel times per libpnr variant (rocprofv3 stats of bench.py --mode train).
export TMPDIR=/tmp
O=gpurun_out/${1:-ptv}; shift
mkdir -p $O
for v in cur "$@"; do
  L=pointnerf_amd/libpnr.so; [ $v != cur ] && L=tools/_ablate/$v/libpnr.so
  PNR_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python bench.py --mode train --steps 10 --warmup 3 > $O/$v.log 2>&1 || exit 1
done
python - "$O" cur "$@" <<'PY'
import csv, glob, sys
o = sys.argv[1]
for v in sys.argv[2:]:
    f = glob.glob(f"{o}/{v}/**/run_kernel_stats.csv", recursive=True)[0]
    print(v, {r["Name"][:30]: round(float(r["AverageNs"]) / 1e3, 1) for r in csv.DictReader(open(f)) if "k_pairs" in r["Name"]})
PY
