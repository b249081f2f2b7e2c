# Per-wave specialised fused kernel: fused tests, cost grid (40, 0, 50), loopback bench.
set -o pipefail
O=gpurun_out/spec; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_fused.py -m gpu -q -x --timeout 170 --timeout-method thread > $O/pytest_fused.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest_fused.log; exit 1; }
tail -2 $O/pytest_fused.log
timeout -k 10 500 python benchmarks/fused_sweep.py --grid --variants 40,0,50 > $O/fused_grid.log 2>&1 || { echo GRID_FAIL; tail -20 $O/fused_grid.log; exit 1; }
grep -v amdgpu.ids $O/fused_grid.log
timeout -k 10 300 python bench.py --loopback --periodic --steps 100 --warmup 10 > $O/bench_lb.log 2>&1 || { echo LB_FAIL; tail -30 $O/bench_lb.log; exit 1; }
grep -E "fused A/B" $O/bench_lb.log | cut -c1-700
python3 -c "import json; d=json.loads([l for l in open('$O/bench_lb.log') if l.startswith('{')][-1]); c=d['config']; print('lb', d['ms_per_step'], c['fused_kernel'], min(c['stencil_variant_ms'].values()))"
