#!/bin/bash
# Dev tool: bench.py line + rocprofv3 kernel-trace stats + separate PMC passes
# (FETCH_SIZE / WRITE_SIZE / MFMA busy) of the same command, into gpurun_out/$1.
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-benchprof}
mkdir -p $O
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
B="python bench.py --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- $B > $O/stats.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $B > $O/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $B > $O/write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_F32 --output-format csv -d $O/mfma -o run -- $B > $O/mfma.log 2>&1
