#!/bin/bash
# Dev tool: L2 hit/miss of the query kernels for each libpnr variant given
# (tools/_ablate/<name>/libpnr.so) into gpurun_out/$1/<name>.
export TMPDIR=/tmp
O=gpurun_out/${1:-l2}; shift
mkdir -p $O
for v in "$@"; do
  PNR_LIB=tools/_ablate/$v/libpnr.so timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --output-format csv -d $O/$v -o run -- python tools/query_bench.py --reps 2 > $O/$v.log 2>&1 || exit 1
done
