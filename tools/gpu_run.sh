# Dev tool: GPU test suite + headline bench on the gpurun box (logs under gpurun_out/$1).
export TMPDIR=/tmp
out=gpurun_out/${1:-run}
mkdir -p $out
shift
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" > $out/t_gpu.log 2>&1 || { tail -30 $out/t_gpu.log; exit 1; }
tail -3 $out/t_gpu.log
timeout -k 10 400 python bench.py > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
