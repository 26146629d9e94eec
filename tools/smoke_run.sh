timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$1/smoke.log 2>&1 || { tail -20 gpurun_out/$1/smoke.log; exit 1; }
tail -2 gpurun_out/$1/smoke.log
