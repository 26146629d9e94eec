#!/bin/bash
# Dev tool: bench.py line + rocprofv3 kernel-trace stats + separate PMC passes
# (FETCH_SIZE / WRITE_SIZE / MFMA busy) of the same command, into gpurun_out/$1.
#   DTYPE=fp32|fp32x3|bf16 (default: the config's), CONFIG=headline|c4|c5,
#   STEPS / WARMUP (default the bench's); fold with
#   python tools/profile_summary.py gpurun_out/$1 <tag> $DTYPE
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-benchprof}
CONFIG=${CONFIG:-headline}
if [ -z "$DTYPE" ]; then [ "$CONFIG" = c5 ] && DTYPE=bf16 || DTYPE=fp32h2; fi
SW=""
[ -n "$STEPS" ] && SW="$SW --steps $STEPS"
[ -n "$WARMUP" ] && SW="$SW --warmup $WARMUP"
case $DTYPE in
  fp32) MOPS=SQ_INSTS_VALU_MFMA_MOPS_F32 ;;
  fp32h2) MOPS=SQ_INSTS_VALU_MFMA_MOPS_F16 ;;
  *) MOPS=SQ_INSTS_VALU_MFMA_MOPS_BF16 ;;
esac
mkdir -p $O
timeout -k 10 400 python bench.py --config $CONFIG --dtype $DTYPE $SW > $O/bench.json 2> $O/bench.err
B="python bench.py --config $CONFIG --no-cpu-baseline --dtype $DTYPE $SW"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- $B > $O/stats.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $B > $O/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $B > $O/write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE $MOPS --output-format csv -d $O/mfma -o run -- $B > $O/mfma.log 2>&1
