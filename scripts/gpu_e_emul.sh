# Same-box evidence for the fused-exchange overhead: no-exchange 1-GPU step vs loopback interior-rank
# emulation (x, xy, xyz), driver-shaped timed loops, two interleaved passes.
set -o pipefail
O=gpurun_out/e_emul; mkdir -p $O
for pass in 1 2; do
timeout -k 10 200 python bench.py --gpus 1 --steps 100 --warmup 10 > $O/plain_$pass.log 2>&1 || { echo P_FAIL; tail -20 $O/plain_$pass.log; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$O/plain_$pass.log') if l.startswith('{')][-1]); print('pass $pass plain', d['ms_per_step'], d['config']['stencil_variant'], d['config']['stencil_grid_rounds'])"
for p in x xy xyz; do
timeout -k 10 300 python bench.py --loopback --periodic-dims $p --steps 100 --warmup 10 > $O/lb_${p}_$pass.log 2>&1 || { echo LB_FAIL $p; tail -30 $O/lb_${p}_$pass.log; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$O/lb_${p}_$pass.log') if l.startswith('{')][-1]); c=d['config']; print('pass $pass $p', d['ms_per_step'], c['fused_kernel'] or c['transport'])"
done
done
