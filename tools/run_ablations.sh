set -e
timeout -k 10 200 python tools/agg_bench.py $ABL_ARGS > gpurun_out/abl_0.json
for N in "$@"; do PNR_LIB=tools/_ablate/$N/libpnr.so timeout -k 10 200 python tools/agg_bench.py $ABL_ARGS > gpurun_out/abl_$N.json; done
