#!/bin/bash
# Dev tool: rocprofv3 kernel stats + separate PMC passes of tools/query_bench.py
# (QCONFIG: headline / c4 / c5) into gpurun_out/$1; fold with
#   python tools/pmc_fold.py gpurun_out/$1 k_knn k_march
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-qprof}
C=${QCONFIG:-headline}
mkdir -p $O
B="python tools/query_bench.py --config $C --reps 2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- $B > $O/stats.log 2>&1
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_VALU GRBM_GUI_ACTIVE" \
           "SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_WAVES" \
           "TA_BUSY_avr TA_TA_BUSY_sum" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $set --output-format csv -d $O/p$i -o run -- $B > $O/p$i.log 2>&1 || { echo "pass $i ($set) failed"; tail -5 $O/p$i.log; exit 1; }
done
