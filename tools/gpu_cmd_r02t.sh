#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/r02t; mkdir -p $O
for v in 0 1 0 1; do
  PNR_COMPACT_P1=$v timeout -k 10 300 python bench.py --steps 10 --warmup 2 > $O/b$v.json 2> $O/b$v.err || { tail $O/b$v.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/b$v.json').read().strip().splitlines()[-1])
print('compact=$v', d['value'], d['stages_ms'], d['accuracy']['psnr_vs_oracle_db'], d['accuracy']['max_abs_err_vs_oracle'])"
done
