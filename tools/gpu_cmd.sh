export TMPDIR=/tmp
mkdir -p gpurun_out/rt
for T in 0 8 16 4 0 8 16 4; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --ray-tile $T --profile-steps > gpurun_out/rt/t$T.json 2> gpurun_out/rt/t$T.err || exit 1
  cat gpurun_out/rt/t$T.json >> gpurun_out/rt/all.jsonl
done
