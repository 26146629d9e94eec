set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
PNR_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/bench2f.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/bench1.log 2>&1
