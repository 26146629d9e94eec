#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/r02u; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python bench.py --steps 3 --warmup 1 > $O/b.log 2>&1 || exit 1
ls -R $O | head
