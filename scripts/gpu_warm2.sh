# Warm-up length vs the driver-shaped 20-step timed region: IGG_BENCH_WARM_MS 40 (default) vs 300,
# interleaved on one box; ms/step, stage-2 autotune best, warm-up steps run.
set -o pipefail
O=gpurun_out/warm2; mkdir -p $O
for i in 1 2 3; do
for w in 40 300; do
IGG_BENCH_WARM_MS=$w timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b_${w}_$i.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/b_${w}_$i.log; exit 1; }
python3 -c "import json,sys; d=json.loads([l for l in open('$O/b_${w}_$i.log') if l.startswith('{')][-1]); c=d['config']; pp={k:v for k,v in c['stencil_variant_ms'].items() if 'pp' in k}; print('warm', $w, 'run', $i, d['ms_per_step'], c['stencil_variant'], c['stencil_grid_rounds'], min(pp.values()) if pp else None, c.get('warmup_steps_run'))"
done
done
