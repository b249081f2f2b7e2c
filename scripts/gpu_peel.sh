# Peeled x planes (fused mode bit 8): bitwise tests, per-wave class costs (f32 1024^3 v44, f64 512^3 v40/v42),
# interior-rank A/B with and without peel.
set -o pipefail
O=gpurun_out/peel; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_fused.py -q -x -k "peel or direct_z_matches" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for m in 4 12; do
timeout -k 10 200 python -u benchmarks/fused_waves.py --n 1024 --dtype float32 --variants 44 --rounds 4 --mode $m > $O/waves_f32_m$m.log 2>&1 || { echo WAVES_FAIL; tail -20 $O/waves_f32_m$m.log; exit 1; }
grep -v Gloo $O/waves_f32_m$m.log | grep -E "variant|f6/auto" | cut -c1-260
timeout -k 10 200 python -u benchmarks/fused_waves.py --n 512 --variants 40,42 --rounds 2 --mode $m > $O/waves_f64_m$m.log 2>&1 || { echo WAVES_FAIL; tail -20 $O/waves_f64_m$m.log; exit 1; }
grep -v Gloo $O/waves_f64_m$m.log | grep -E "variant|f6/auto" | cut -c1-260
done
IGG_FUSED_CANDIDATES=40/4/2,40/12/2,42/4/2,42/12/2,0/4/3,0/12/3,40/0/2,40/8/2 timeout -k 10 400 python -u bench.py --loopback --periodic --steps 100 --warmup 10 > $O/f64_lb.log 2>&1 || { echo F64_FAIL; tail -30 $O/f64_lb.log; exit 1; }
grep -E "A/B" $O/f64_lb.log | cut -c1-1500; tail -1 $O/f64_lb.log | cut -c1-200
IGG_FUSED_CANDIDATES=44/4/3,44/12/3,44/4/4,44/12/4 IGG_TRANSPORT=put timeout -k 10 400 python -u bench.py --config diffusion3d_f32_gather --loopback --periodic --steps 100 --warmup 10 > $O/f32_lb.log 2>&1 || { echo F32_FAIL; tail -30 $O/f32_lb.log; exit 1; }
grep -E "A/B" $O/f32_lb.log | cut -c1-1500; tail -1 $O/f32_lb.log | cut -c1-200
