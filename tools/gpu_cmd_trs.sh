export TMPDIR=/tmp
O=gpurun_out/trs; mkdir -p $O
for N in "$@"; do
  PNR_SKEW_TRACE=1 PNR_LIB=tools/_ablate/$N/libpnr.so timeout -k 10 200 python tools/x3_trace.py > $O/$N.txt 2>&1 || { tail -5 $O/$N.txt; exit 1; }
  echo "== $N"; grep -v amdgpu.ids $O/$N.txt
done
