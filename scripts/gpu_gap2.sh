# Same-box comparison: driver-style bench runs vs the loop-gap probe.
set -o pipefail
O=gpurun_out/gap2; mkdir -p $O
for i in 1 2; do
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench$i.log 2>&1 || { echo FAIL; tail -20 $O/bench$i.log; exit 1; }
python3 -c "import json,sys; d=json.loads([l for l in open('$O/bench$i.log') if l.startswith('{')][-1]); c=d['config']; print('bench', d['ms_per_step'], c['stencil_variant'], c['stencil_grid_rounds'], min(c['stencil_variant_ms'].values()))"
done
timeout -k 10 200 python bench.py --gpus 1 --steps 200 --warmup 5 > $O/bench200.log 2>&1 || { echo FAIL; tail -20 $O/bench200.log; exit 1; }
python3 -c "import json,sys; d=json.loads([l for l in open('$O/bench200.log') if l.startswith('{')][-1]); c=d['config']; print('bench200', d['ms_per_step'], c['stencil_variant'], c['stencil_grid_rounds'], min(c['stencil_variant_ms'].values()))"
timeout -k 10 300 python benchmarks/loop_gap.py > $O/auto.log 2>&1 || { echo FAIL; tail -20 $O/auto.log; exit 1; }
tail -1 $O/auto.log
