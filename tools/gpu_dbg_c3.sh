#!/bin/bash
timeout -k 10 300 python -u tools/dbg_bwd_det.py > gpurun_out/det.log 2>&1 || exit 1
T="tests/test_gpu_flagsets.py::test_c3_ship_finetune_batch_grads_vs_oracle"
for i in 1 2; do timeout -k 10 300 python -u -m pytest $T -x -q --timeout 200 --timeout-method thread > gpurun_out/c3_$i.log 2>&1; done
bash tools/prof_train.sh ptrain4
exit 0
