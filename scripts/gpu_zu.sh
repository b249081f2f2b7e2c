# Uniform z-halo loads: fused tests, per-wave timing of 40/41, xyz loopback bench.
set -o pipefail
O=gpurun_out/zu; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_fused.py -m gpu -q -x --timeout 170 --timeout-method thread > $O/pytest_fused.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest_fused.log; exit 1; }
tail -1 $O/pytest_fused.log
timeout -k 10 300 python benchmarks/fused_waves.py --variants 42,55,40 --rounds 2 --mode 0 > $O/waves.log 2>&1 || { echo W_FAIL; tail -20 $O/waves.log; exit 1; }
grep -v amdgpu.ids $O/waves.log | cut -c1-400
timeout -k 10 300 python bench.py --loopback --periodic-dims xyz --steps 100 --warmup 10 > $O/bench_lb_xyz.log 2>&1 || { echo LB_FAIL; tail -30 $O/bench_lb_xyz.log; exit 1; }
grep -E "fused A/B" $O/bench_lb_xyz.log | cut -c1-700
python3 -c "import json; d=json.loads([l for l in open('$O/bench_lb_xyz.log') if l.startswith('{')][-1]); c=d['config']; print('lb', d['ms_per_step'], c['fused_kernel'], 'plain best', min(c['stencil_variant_ms'].values()))"
