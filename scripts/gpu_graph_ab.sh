# Timed loop: graph replays vs eager steps (driver-shaped, alternating).
set -o pipefail
O=gpurun_out/graph_ab; mkdir -p $O
for i in 1 2; do
for g in graph no-graph; do
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --$g > $O/bench_${g}_$i.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench_${g}_$i.log; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('$O/bench_${g}_$i.log') if l.startswith('{')][-1]); c=d['config']; t=c['stencil_variant_ms']
pp={k:v for k,v in t.items() if k.endswith('/pp')}
print('$g', d['ms_per_step'], 'pick', c['stencil_variant'], c['stencil_grid_rounds'], 'pp best', min(pp.values()), 'hip_graph', c['hip_graph'])"
done
done
timeout -k 10 200 python bench.py --gpus 1 --steps 200 --warmup 5 > $O/bench_200.log 2>&1 || { echo BENCH_FAIL; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('$O/bench_200.log') if l.startswith('{')][-1]); c=d['config']; print('graph 200 steps', d['ms_per_step'])"
