# After the RCCL capture fix + fine-grained arena: full GPU suite, fused cost grid of tilings 40/11.
set -o pipefail
O=gpurun_out/r2c; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 170 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log; grep -E "^FAILED|^ERROR" $O/pytest_gpu.log | head -20
[ $rc -eq 0 ] || { echo PYTEST_FAIL rc=$rc; tail -60 $O/pytest_gpu.log; exit 1; }
timeout -k 10 400 python benchmarks/fused_sweep.py --grid --variants 40,11 > $O/fused_grid.log 2>&1 || { echo GRID_FAIL; tail -20 $O/fused_grid.log; exit 1; }
grep -v amdgpu.ids $O/fused_grid.log
