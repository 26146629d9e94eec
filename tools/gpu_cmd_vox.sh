export TMPDIR=/tmp
O=gpurun_out/vox; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_voxelize.py tests/test_abi.py -x -v --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -3 $O/t.log
