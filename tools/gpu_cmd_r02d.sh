export TMPDIR=/tmp
mkdir -p gpurun_out/r02d
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_render.py tests/test_gpu_x3.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r02d/t.log 2>&1 || { tail -40 gpurun_out/r02d/t.log; exit 1; }
tail -3 gpurun_out/r02d/t.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r02d/b1.json 2> gpurun_out/r02d/b1.err || { tail -20 gpurun_out/r02d/b1.err; exit 1; }
cat gpurun_out/r02d/b1.json | head -c 600; echo
timeout -k 10 300 python bench.py --no-cpu-baseline --emulate-world 8 --shard tiles > gpurun_out/r02d/b8.json 2> gpurun_out/r02d/b8.err || { tail -20 gpurun_out/r02d/b8.err; exit 1; }
cat gpurun_out/r02d/b8.json | head -c 600; echo
