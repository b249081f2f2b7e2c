# Fused variant 50 (tiling 0 held at one workgroup per CU): fused tests, loopback benches.
set -o pipefail
export IGG_PUT_TIMEOUT=20
O=gpurun_out/f50; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_fused.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAIL|Error" $O/pytest.log | head; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for P in xyz xy; do
  timeout -k 10 300 python bench.py --loopback --periodic-dims $P > $O/bench_lb_$P.log 2>&1 || { echo BENCH_FAIL $P; tail -20 $O/bench_lb_$P.log; exit 1; }
  grep -E "A/B" $O/bench_lb_$P.log | cut -c1-900
  grep '^{' $O/bench_lb_$P.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('loopback $P', d['ms_per_step'], d['value'], d['config']['fused_kernel'], d['config']['transport'], d['config']['stencil_variant'])"
done
