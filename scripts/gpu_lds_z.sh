# LDS-staged z edge (fused 41/51/52): fused tests, per-wave timing, loopback bench A/B.
set -o pipefail
O=gpurun_out/ldsz; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_fused.py -m gpu -q -x --timeout 170 --timeout-method thread > $O/pytest_fused.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest_fused.log; exit 1; }
tail -2 $O/pytest_fused.log
timeout -k 10 400 python benchmarks/fused_waves.py --variants 41,40,51,52 --rounds 2 --mode 0 > $O/waves_m0.log 2>&1 || { echo W_FAIL; tail -20 $O/waves_m0.log; exit 1; }
grep -v amdgpu.ids $O/waves_m0.log
timeout -k 10 400 python benchmarks/fused_sweep.py --grid --variants 41,51,52 > $O/fused_grid.log 2>&1 || { echo GRID_FAIL; tail -20 $O/fused_grid.log; exit 1; }
grep -v amdgpu.ids $O/fused_grid.log
