# BASELINE configs 4/5 as interior ranks emulated on one GPU (loopback, every face through the
# remote path) on the current tree: fused A/B for 1024^3 f32, put transport for the 2-D acoustic.
set -o pipefail
O=gpurun_out/cfg_lb; mkdir -p $O
timeout -k 10 400 python -u bench.py --config diffusion3d_f32_gather --loopback --periodic --steps 100 --warmup 10 > $O/f32_lb.log 2>&1 || { echo F32_FAIL; tail -30 $O/f32_lb.log; exit 1; }
grep -E "A/B|validation" $O/f32_lb.log | cut -c1-1500; tail -1 $O/f32_lb.log | cut -c1-400
timeout -k 10 300 python -u bench.py --config diffusion3d_f32_gather --steps 100 --warmup 10 > $O/f32.log 2>&1 || { echo F32P_FAIL; tail -30 $O/f32.log; exit 1; }
tail -1 $O/f32.log | cut -c1-400
IGG_TRANSPORT=put timeout -k 10 300 python -u bench.py --config acoustic2d --loopback --periodic --steps 200 --warmup 10 > $O/ac_lb_put.log 2>&1 || { echo AC_FAIL; tail -30 $O/ac_lb_put.log; exit 1; }
grep -E "A/B|validation" $O/ac_lb_put.log | cut -c1-600; tail -1 $O/ac_lb_put.log | cut -c1-400
timeout -k 10 300 python -u bench.py --config acoustic2d --steps 200 --warmup 10 > $O/ac.log 2>&1 || { echo ACP_FAIL; tail -30 $O/ac.log; exit 1; }
tail -1 $O/ac.log | cut -c1-400
