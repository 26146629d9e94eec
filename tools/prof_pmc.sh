#!/bin/bash
# Dev tool: PMC counter passes over tools/agg_bench.py (one rocprofv3 run per counter set).
#   PMC_SETS=x3 selects the bf16-MFMA set; AGG_ARGS is passed to agg_bench.py.
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc}
mkdir -p $OUT
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
if [ "${PMC_SETS:-default}" = x3 ]; then
  LIST=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
        "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_VALU"
        "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_INSTS_SALU")
else
  LIST=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
        "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_VALU"
        "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU")
fi
i=0
for set in "${LIST[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o run -- python tools/agg_bench.py --reps 1 $AGG_ARGS > $OUT/p$i.log 2>&1 || echo "pass $i failed" >> $OUT/fail.txt
done
