#!/bin/bash
# Dev tool: training tests, x3 GEMM prefetch A/B (pf1 = one chunk in flight), train bench.
export TMPDIR=/tmp
O=gpurun_out/r02i; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_backward.py tests/test_gpu_api.py tests/test_gpu_flagsets.py -x -v --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -2 $O/t.log
timeout -k 10 200 python tools/gemm_bench.py > $O/gemm_pf2.json 2>&1 || exit 1
PNR_LIB=tools/_ablate/pf1/libpnr.so timeout -k 10 200 python tools/gemm_bench.py > $O/gemm_pf1.json 2>&1 || exit 1
cat $O/gemm_pf2.json $O/gemm_pf1.json
timeout -k 10 300 python bench.py --mode train > $O/bench_x3.json 2> $O/bench_x3.err || exit 1
PNR_LIB=tools/_ablate/pf1/libpnr.so timeout -k 10 300 python bench.py --mode train > $O/bench_x3_pf1.json 2> $O/bench_x3_pf1.err || exit 1
python -c "
import json
for f in ('bench_x3','bench_x3_pf1'):
    d=json.loads(open('$O/'+f+'.json').read().strip().splitlines()[-1]); print(f, d['value'], d['ms_per_step'])
"
