bash tools/prof_train.sh ptrain2 && timeout -k 10 300 python tools/query_bench.py --reps 5 > gpurun_out/ptrain2/query.json
