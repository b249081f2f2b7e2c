# Stencil variant 43 (full-row z tiles) in the autotune shortlist: numerics tests, driver-shaped bench x3.
set -o pipefail
O=gpurun_out/v43; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_stencil.py -q -x --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench$i.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench$i.log; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$O/bench$i.log') if l.startswith('{')][-1]); c=d['config']; v=c['stencil_variant_ms']; print('bench', d['ms_per_step'], c['stencil_variant'], c['stencil_grid_rounds'], {k:x for k,x in v.items() if 'pp' in k or k.startswith('43')})"
done
