# Timed-region bracket cost (1, 2, 4 ranks) and driver-shaped bench with the new bracket.
set -o pipefail
O=gpurun_out/bracket; mkdir -p $O
timeout -k 10 120 python benchmarks/bracket_cost.py > $O/bracket_1.log 2>&1 || { echo BR1_FAIL; tail -20 $O/bracket_1.log; exit 1; }
grep "rank(s)" $O/bracket_1.log
for n in 2 4; do
timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node=$n --master-addr 127.0.0.1 --master-port 2960$n benchmarks/bracket_cost.py --share-gpu > $O/bracket_$n.log 2>&1 || { echo BR_FAIL $n; tail -20 $O/bracket_$n.log; exit 1; }
grep "rank(s)" $O/bracket_$n.log
done
for i in 1 2; do
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench$i.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench$i.log; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('$O/bench$i.log') if l.startswith('{')][-1]); c=d['config']; t=c['stencil_variant_ms']
pp={k:v for k,v in t.items() if k.endswith('/pp')}
print('bench', d['ms_per_step'], 'pick', c['stencil_variant'], c['stencil_grid_rounds'], 'pp', pp, c['timing_bracket'])"
done
timeout -k 10 300 python bench.py --gpus 2 --share-gpu --n 192 --steps 50 --warmup 5 --launch-timeout 250 > $O/b2_self.log 2>&1 || { echo B2_FAIL; tail -30 $O/b2_self.log; exit 1; }
tail -1 $O/b2_self.log | cut -c1-200
