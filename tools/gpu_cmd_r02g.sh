export TMPDIR=/tmp
O=gpurun_out/r02g; mkdir -p $O
timeout -k 10 300 python bench.py --no-cpu-baseline --emulate-world 2 --shard tiles > $O/b2.json 2> $O/b2.err || { tail -20 $O/b2.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --emulate-world 8 --shard tiles > $O/b8.json 2> $O/b8.err || { tail -20 $O/b8.err; exit 1; }
PNR_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 > $O/g2.json 2> $O/g2.err || { tail -30 $O/g2.err; exit 1; }
cat $O/g2.json
