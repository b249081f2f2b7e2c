# Variants 40-42 (lane-distributed z edges, one workgroup per CU) and fused variant 40:
# stencil + fused tests, variant sweep, loopback benches (2x1x1 / 2x2x1 / 2x2x2 ranks), 1-GPU bench.
set -o pipefail
export IGG_PUT_TIMEOUT=20
O=gpurun_out/zl2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_stencil.py tests/test_fused.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAIL|Error" $O/pytest.log | head; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python -u benchmarks/variant_sweep.py --variants 24,40,41,42 --rounds 1,2,3,4 > $O/variant_sweep.log 2>&1 || { echo SWEEP_FAIL; tail -20 $O/variant_sweep.log; exit 1; }
grep -v amdgpu.ids $O/variant_sweep.log | head -8
for P in xyz xy x; do
  timeout -k 10 300 python bench.py --loopback --periodic-dims $P > $O/bench_lb_$P.log 2>&1 || { echo BENCH_FAIL $P; tail -20 $O/bench_lb_$P.log; exit 1; }
  grep -E "A/B" $O/bench_lb_$P.log | cut -c1-900
  grep '^{' $O/bench_lb_$P.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('loopback $P', d['ms_per_step'], d['value'], d['config']['fused_kernel'], d['config']['transport'])"
done
timeout -k 10 300 python bench.py > $O/bench_1gpu.log 2>&1 || { echo BENCH_FAIL 1gpu; tail -20 $O/bench_1gpu.log; exit 1; }
grep '^{' $O/bench_1gpu.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('1gpu', d['ms_per_step'], d['value'], d['config']['stencil_variant'], d['config']['stencil_grid_rounds'])"
