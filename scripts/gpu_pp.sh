# Ping-pong second autotune stage: driver-shaped bench x3, model GPU tests.
set -o pipefail
O=gpurun_out/pp; mkdir -p $O
for i in 1 2 3; do
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench$i.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench$i.log; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('$O/bench$i.log') if l.startswith('{')][-1]); c=d['config']; t=c['stencil_variant_ms']
pp={k:v for k,v in t.items() if k.endswith('/pp')}; st={k:v for k,v in t.items() if not k.endswith('/pp')}
print('bench', d['ms_per_step'], 'pick', c['stencil_variant'], c['stencil_grid_rounds'], 'stage1 best', min(st.items(), key=lambda kv: kv[1]), 'pp', pp)"
done
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -k "diffusion or model or stencil or example" --timeout 170 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
