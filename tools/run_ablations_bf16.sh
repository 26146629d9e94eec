set -e
timeout -k 10 200 python tools/agg_bench.py --precision bf16 > gpurun_out/ablb_0.json
for N in "$@"; do PNR_LIB=tools/_ablate/$N/libpnr.so timeout -k 10 200 python tools/agg_bench.py --precision bf16 > gpurun_out/ablb_$N.json; done
