# BASELINE configs 4/5 on the current tree: acoustic 8192^2 f32, diffusion 1024^3 f32 + gather_ every 100.
set -o pipefail
O=gpurun_out/cfgs2; mkdir -p $O
timeout -k 10 300 python bench.py --config acoustic2d --steps 100 --warmup 10 > $O/acoustic.log 2>&1 || { echo AC_FAIL; tail -20 $O/acoustic.log; exit 1; }
tail -1 $O/acoustic.log | cut -c1-260
timeout -k 10 300 python bench.py --config acoustic2d --loopback --periodic --steps 100 --warmup 10 > $O/acoustic_lb.log 2>&1 || { echo AC_LB_FAIL; tail -20 $O/acoustic_lb.log; exit 1; }
grep -E "A/B" $O/acoustic_lb.log | cut -c1-300; tail -1 $O/acoustic_lb.log | cut -c1-260
timeout -k 10 400 python bench.py --config diffusion3d_f32_gather --steps 200 --warmup 10 > $O/f32_gather.log 2>&1 || { echo F32_FAIL; tail -20 $O/f32_gather.log; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$O/f32_gather.log') if l.startswith('{')][-1]); c=d['config']; print('f32 gather', d['ms_per_step'], d['value'], c['stencil_variant'], c['gather_ms'])"
