# Direct z across processes (IPC-mapped torch buffers of the peer ranks), soak, full fused suite.
set -o pipefail
O=gpurun_out/zdirect2; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 170 --timeout-method thread tests/test_multiprocess.py -m gpu -k "fused" > $O/mp.log 2>&1 || { echo MP_FAIL; tail -40 $O/mp.log; exit 1; }
grep -E "PASS|FAIL" $O/mp.log | tail -15
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused.py -m gpu > $O/fused.log 2>&1 || { echo F_FAIL; tail -30 $O/fused.log; exit 1; }
tail -2 $O/fused.log
