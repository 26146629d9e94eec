export TMPDIR=/tmp
O=gpurun_out/r04h; mkdir -p $O
timeout -k 10 900 bash tools/prof_bench.sh r04_head > $O/prof_head.log 2>&1 || exit $?
CONFIG=c5 STEPS=10 WARMUP=3 timeout -k 10 600 bash tools/prof_bench.sh r04_c5 > $O/prof_c5.log 2>&1 || exit $?
CONFIG=c4 STEPS=10 WARMUP=3 timeout -k 10 600 bash tools/prof_bench.sh r04_c4 > $O/prof_c4.log 2>&1 || exit $?
ls gpurun_out/r04_head gpurun_out/r04_c5 gpurun_out/r04_c4
