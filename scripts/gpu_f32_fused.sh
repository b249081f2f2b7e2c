# Fused variants 44/45 (edge-lane z for tilings 14/0): bitwise tests, per-wave class costs in f32,
# and the 1024^3 f32 interior-rank A/B with f32-shaped candidates.
set -o pipefail
O=gpurun_out/f32f; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_fused.py -q -x -k "44 or 45" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u benchmarks/fused_waves.py --n 1024 --dtype float32 --variants 44,14 --rounds 4 --mode 4 > $O/waves_m4.log 2>&1 || { echo WAVES_FAIL; tail -20 $O/waves_m4.log; exit 1; }
grep -v Gloo $O/waves_m4.log | cut -c1-300
IGG_FUSED_CANDIDATES=44/4/4,44/4/3,44/5/4,44/0/4,14/4/4,45/4/4,45/4/3,0/4/4 IGG_TRANSPORT=put timeout -k 10 400 python -u bench.py --config diffusion3d_f32_gather --loopback --periodic --steps 100 --warmup 10 > $O/f32_lb.log 2>&1 || { echo F32_FAIL; tail -30 $O/f32_lb.log; exit 1; }
grep -E "A/B" $O/f32_lb.log | cut -c1-1500; tail -1 $O/f32_lb.log | cut -c1-300
IGG_FUSED_CANDIDATES=45/4/3,45/0/3,45/4/2,0/4/3,0/0/3,42/4/2,40/4/2 timeout -k 10 400 python -u bench.py --loopback --periodic --steps 100 --warmup 10 > $O/f64_lb.log 2>&1 || { echo F64_FAIL; tail -30 $O/f64_lb.log; exit 1; }
grep -E "A/B" $O/f64_lb.log | cut -c1-1500; tail -1 $O/f64_lb.log | cut -c1-300
