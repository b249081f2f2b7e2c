# Direct z (fused send mode bit 4): GPU tests, then loopback xyz A/B of direct vs arena forms
# and a same-box plain reference.
set -o pipefail
O=gpurun_out/zdirect; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused.py -m gpu -k "direct or layout" > $O/tests.log 2>&1 || { echo T_FAIL; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python bench.py --gpus 1 --steps 100 --warmup 10 > $O/plain.log 2>&1 || { echo P_FAIL; tail -20 $O/plain.log; exit 1; }
tail -1 $O/plain.log | cut -c1-160
for pass in 1 2; do
IGG_FUSED_CANDIDATES="50/0/2,0/0/3,42/0/2,40/4/2,42/4/2,42/5/2,50/4/2,0/4/3,9/4/3,14/4/3" timeout -k 10 400 python bench.py --loopback --periodic-dims xyz --steps 100 --warmup 10 > $O/lb_xyz_$pass.log 2>&1 || { echo LB_FAIL; tail -30 $O/lb_xyz_$pass.log; exit 1; }
grep -E "fused A/B|fused check" $O/lb_xyz_$pass.log | cut -c1-1200; tail -1 $O/lb_xyz_$pass.log | cut -c1-160
done
