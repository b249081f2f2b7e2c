# Full GPU check: pytest -m gpu, 1-GPU bench (driver default), loopback interior-rank bench.
set -o pipefail
export IGG_PUT_TIMEOUT=20
O=gpurun_out/full; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 175 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAIL|Error" $O/pytest_gpu.log | head -20; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python bench.py > $O/bench_1gpu.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench_1gpu.log; exit 1; }
grep '^{' $O/bench_1gpu.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('1gpu', d['ms_per_step'], d['value'], d['config']['stencil_variant'], d['config']['stencil_grid_rounds'], d['config']['stencil_variant_ms'])"
timeout -k 10 300 python bench.py --loopback --periodic > $O/bench_lb.log 2>&1 || { echo BENCH_LB_FAIL; tail -20 $O/bench_lb.log; exit 1; }
grep -E "A/B" $O/bench_lb.log
grep '^{' $O/bench_lb.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('loopback', d['ms_per_step'], d['value'], d['config']['fused_kernel'], d['config']['transport'])"
