#!/bin/bash
# Dev tool: tools/query_bench.py over libpnr variants (tools/_ablate/<name>/libpnr.so), twice each.
export TMPDIR=/tmp
O=gpurun_out/${1:-abq}; shift
mkdir -p $O
for rep in 1 2; do
  for v in "$@"; do
    PNR_LIB=tools/_ablate/$v/libpnr.so timeout -k 10 300 python tools/query_bench.py --reps 5 > $O/$v.$rep.json 2>> $O/err.log || exit 1
  done
done
python - "$O" "$@" <<'PY'
import json, sys
o = sys.argv[1]
for v in sys.argv[2:]:
    r = []
    for rep in (1, 2):
        d = json.load(open(f"{o}/{v}.{rep}.json"))
        r.append([c["query_ms"] for c in d["cams"]])
    print(v, r, [c["pidx_checksum"] for c in d["cams"]][:2])
PY
