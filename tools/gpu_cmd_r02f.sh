export TMPDIR=/tmp
O=gpurun_out/r02f; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -3 $O/t.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/b1.json 2> $O/b1.err || { tail -20 $O/b1.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --emulate-world 8 --shard tiles > $O/b8.json 2> $O/b8.err || { tail -20 $O/b8.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --emulate-world 8 --shard tiles --per-frame-calls > $O/b8pf.json 2> $O/b8pf.err || { tail -20 $O/b8pf.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --emulate-world 2 --shard tiles > $O/b2.json 2> $O/b2.err || { tail -20 $O/b2.err; exit 1; }
