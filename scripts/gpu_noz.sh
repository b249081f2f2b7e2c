# Fused exchange without a z neighbour (FEAT 195): tests, then loopback benches
# emulating interior ranks of 2x1x1 (x), 2x2x1 (xy) and 2x2x2 (xyz) topologies.
set -o pipefail
export IGG_PUT_TIMEOUT=20
O=gpurun_out/noz; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_fused.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_fused.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAIL|Error" $O/pytest_fused.log | head -20; tail -30 $O/pytest_fused.log; exit 1; }
tail -1 $O/pytest_fused.log
for P in x xy xyz; do
  timeout -k 10 300 python bench.py --loopback --periodic-dims $P > $O/bench_lb_$P.log 2>&1 || { echo BENCH_FAIL $P; tail -20 $O/bench_lb_$P.log; exit 1; }
  grep -E "A/B" $O/bench_lb_$P.log
  grep '^{' $O/bench_lb_$P.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('loopback $P', d['ms_per_step'], d['value'], d['config']['fused_kernel'], d['config']['transport'])"
done
timeout -k 10 300 python bench.py > $O/bench_1gpu.log 2>&1 || { echo BENCH_FAIL 1gpu; tail -20 $O/bench_1gpu.log; exit 1; }
grep '^{' $O/bench_1gpu.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('1gpu', d['ms_per_step'], d['value'], d['config']['stencil_variant'], d['config']['stencil_grid_rounds'])"
