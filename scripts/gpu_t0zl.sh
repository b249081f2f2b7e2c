# Tiling 0 + lane-distributed z edges (plain 39 / fused 53, 54) vs 40/50: plain sweep, fused tests, fused grid, xyz loopback.
set -o pipefail
O=gpurun_out/t0zl; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_fused.py -m gpu -q -x --timeout 170 --timeout-method thread > $O/pytest_fused.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest_fused.log; exit 1; }
tail -1 $O/pytest_fused.log
timeout -k 10 300 python benchmarks/variant_sweep.py --variants 0,39,40,24,37 --rounds 1,2,3,4 > $O/variant_sweep.log 2>&1 || { echo VS_FAIL; tail -20 $O/variant_sweep.log; exit 1; }
grep -v amdgpu.ids $O/variant_sweep.log | head -24
timeout -k 10 500 python benchmarks/fused_sweep.py --grid --variants 53,54,50 > $O/fused_grid.log 2>&1 || { echo GRID_FAIL; tail -20 $O/fused_grid.log; exit 1; }
grep -v amdgpu.ids $O/fused_grid.log
