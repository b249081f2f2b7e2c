# After splitting the fused kernels into per-family TUs: smoke, full GPU suite, driver-shaped bench, loopback xy.
set -o pipefail
O=gpurun_out/r2d; mkdir -p $O
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 170 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -60 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench.log; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$O/bench.log') if l.startswith('{')][-1]); c=d['config']; print('bench', d['ms_per_step'], c['stencil_variant'], c['stencil_grid_rounds'], min(c['stencil_variant_ms'].values()))"
timeout -k 10 300 python bench.py --loopback --periodic-dims xy --steps 100 --warmup 10 > $O/bench_lb_xy.log 2>&1 || { echo LB_FAIL; tail -30 $O/bench_lb_xy.log; exit 1; }
grep -E "fused A/B" $O/bench_lb_xy.log | cut -c1-700
python3 -c "import json; d=json.loads([l for l in open('$O/bench_lb_xy.log') if l.startswith('{')][-1]); c=d['config']; print('lb xy', d['ms_per_step'], c['fused_kernel'], 'plain best', min(c['stencil_variant_ms'].values()))"
