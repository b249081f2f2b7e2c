# Fused-exchange verification: single-process + multi-rank tests (incl. put transport), grid sweep.
set -o pipefail
export IGG_PUT_TIMEOUT=20
O=gpurun_out/fused2; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fused.py tests/test_multiprocess.py -k "fused or put" > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAIL|Error" $O/pytest.log | head; tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python benchmarks/fused_sweep.py --grid --variants 0,14 --reps 10 > $O/grid.log 2>&1 || { echo SWEEP_FAIL; tail -20 $O/grid.log; exit 1; }
grep variant $O/grid.log
