export TMPDIR=/tmp
mkdir -p gpurun_out/prec
REPS=2 bash tools/ab.sh pr2 pr1c1
unset PNR_LIB
for D in fp32 fp32x3 bf16; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --dtype $D > gpurun_out/prec/$D.json 2> gpurun_out/prec/$D.err || exit 1
done
