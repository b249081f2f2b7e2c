# BASELINE configs 4/5 through the self-launched multi-rank bench on one shared GPU (plumbing rehearsal:
# validation, transport/fused A/B, gather_ at N > 1).
set -o pipefail
O=gpurun_out/cfgm; mkdir -p $O
timeout -k 10 400 python bench.py --config acoustic2d --gpus 4 --share-gpu --n 2048 --steps 50 --warmup 5 --launch-timeout 350 > $O/ac4.log 2>&1 || { echo AC4_FAIL; tail -30 $O/ac4.log; exit 1; }
grep -E "A/B|validation" $O/ac4.log | cut -c1-500; tail -1 $O/ac4.log | cut -c1-400
timeout -k 10 400 python bench.py --config diffusion3d_f32_gather --gpus 2 --share-gpu --n 256 --gather-every 10 --steps 40 --warmup 5 --launch-timeout 350 > $O/f32g2.log 2>&1 || { echo F32G_FAIL; tail -30 $O/f32g2.log; exit 1; }
grep -E "A/B|validation" $O/f32g2.log | cut -c1-500; tail -1 $O/f32g2.log | cut -c1-600
