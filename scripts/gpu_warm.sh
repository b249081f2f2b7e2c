# Driver-style bench after the steady-state warm-up fix (2 runs) + loopback.
set -o pipefail
O=gpurun_out/warm; mkdir -p $O
for i in 1 2; do
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench$i.log 2>&1 || { echo FAIL; tail -20 $O/bench$i.log; exit 1; }
python3 -c "import json,sys; d=json.loads([l for l in open('$O/bench$i.log') if l.startswith('{')][-1]); c=d['config']; print('bench', d['ms_per_step'], c['stencil_variant'], c['stencil_grid_rounds'], min(c['stencil_variant_ms'].values()), c['warmup_steps_run'])"
done
timeout -k 10 300 python bench.py --loopback --periodic --steps 20 --warmup 5 > $O/bench_lb.log 2>&1 || { echo BENCH_LB_FAIL; tail -30 $O/bench_lb.log; exit 1; }
grep -E "A/B" $O/bench_lb.log | cut -c1-600
python3 -c "import json,sys; d=json.loads([l for l in open('$O/bench_lb.log') if l.startswith('{')][-1]); c=d['config']; print('lb', d['ms_per_step'], c['fused_kernel'], min(c['stencil_variant_ms'].values()), c['warmup_steps_run'])"
