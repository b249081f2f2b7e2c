# BASELINE config 5: 3-D diffusion 1024^3 f32 with gather_ every 100 steps (1 GPU; interior-rank loopback).
set -o pipefail
export IGG_PUT_TIMEOUT=20
O=gpurun_out/cfg5; mkdir -p $O
timeout -k 10 400 python bench.py --config diffusion3d_f32_gather --steps 200 --warmup 10 > $O/bench.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('1gpu', d['ms_per_step'], d['value'], c['stencil_variant'], c['stencil_grid_rounds'], c['gather_ms'])"
timeout -k 10 400 python bench.py --config diffusion3d_f32_gather --steps 200 --warmup 10 --loopback --periodic --transport put > $O/bench_lb.log 2>&1 || { echo BENCH_LB_FAIL; tail -20 $O/bench_lb.log; exit 1; }
grep -E "A/B" $O/bench_lb.log
grep '^{' $O/bench_lb.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('loopback', d['ms_per_step'], d['value'], c['fused_kernel'], c['gather_ms'])"
