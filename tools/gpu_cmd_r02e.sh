export TMPDIR=/tmp
O=gpurun_out/r02e; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_graph.py -x -v --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -3 $O/t.log
for L in bands tiles16; do
timeout -k 10 300 python bench.py --no-cpu-baseline --emulate-world 8 --shard tiles --tile-layout $L > $O/b8_$L.json 2> $O/b8_$L.err || { tail -20 $O/b8_$L.err; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats8 -o run -- python bench.py --no-cpu-baseline --emulate-world 8 --shard tiles > $O/stats8.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats1 -o run -- python bench.py --no-cpu-baseline > $O/stats1.log 2>&1
