export TMPDIR=/tmp
O=gpurun_out/r02h; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -2 $O/t.log
timeout -k 10 300 python bench.py --dtype bf16 > $O/bf16.json 2> $O/bf16.err || { tail -20 $O/bf16.err; exit 1; }
