#!/bin/bash
# Dev tool: rocprofv3 kernel stats + separate PMC passes of tools/query_bench.py into gpurun_out/$1.
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-qprof}
mkdir -p $O
rocprofv3 -L > $O/counters_list.txt 2>&1 || true
B="python tools/query_bench.py --reps 3"
timeout -k 10 300 python tools/query_bench.py > $O/query.json 2> $O/query.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- $B > $O/stats.log 2>&1
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM GRBM_GUI_ACTIVE" \
           "TA_BUSY_avr TA_TA_BUSY_sum" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $O/p$i -o run -- $B > $O/p$i.log 2>&1 || echo "pass $i ($set) failed" >> $O/fail.txt
done
