#!/bin/bash
# Dev tool: rocprofv3 kernel stats of tools/agg_bench.py (fp32h2) for the in-tree
# libpnr.so ("cur") and each tools/_ablate/<name>/libpnr.so; prints the average
# duration of the kernels matching $KPAT per variant.
export TMPDIR=/tmp
O=gpurun_out/${1:-pv}; shift
mkdir -p $O
for v in cur "$@"; do
  L=pointnerf_amd/libpnr.so; [ $v != cur ] && L=tools/_ablate/$v/libpnr.so
  PNR_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python tools/agg_bench.py --precision fp32h2 --reps 2 > $O/$v.log 2>&1 || exit 1
done
python - "$O" "${KPAT:-k_color_h2|k_point_pre_h2|k_pairs_h2}" cur "$@" <<'PY'
import csv, glob, re, sys
o, pat = sys.argv[1], re.compile(sys.argv[2])
for v in sys.argv[3:]:
    f = glob.glob(f"{o}/{v}/**/run_kernel_stats.csv", recursive=True)[0]
    print(v, {r["Name"][:40]: round(float(r["AverageNs"]) / 1e6, 3) for r in csv.DictReader(open(f)) if pat.search(r["Name"])})
PY
