# Batched z sends (fused variants 46/47/48 = 42/44/45 + FEAT 262144): bitwise tests, interior-rank A/B f64/f32.
set -o pipefail
O=gpurun_out/zb; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_fused.py -q -x -k "46 or 47 or 48" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
IGG_FUSED_CANDIDATES=42/12/2,46/12/2,42/4/2,46/4/2,48/12/3,45/12/3,40/12/2 timeout -k 10 400 python -u bench.py --loopback --periodic --steps 100 --warmup 10 > $O/f64_lb.log 2>&1 || { echo F64_FAIL; tail -30 $O/f64_lb.log; exit 1; }
grep -E "A/B" $O/f64_lb.log | cut -c1-1500; tail -1 $O/f64_lb.log | cut -c1-200
IGG_FUSED_CANDIDATES=44/12/3,47/12/3,44/12/4,47/12/4 IGG_TRANSPORT=put timeout -k 10 400 python -u bench.py --config diffusion3d_f32_gather --loopback --periodic --steps 100 --warmup 10 > $O/f32_lb.log 2>&1 || { echo F32_FAIL; tail -30 $O/f32_lb.log; exit 1; }
grep -E "A/B" $O/f32_lb.log | cut -c1-1500; tail -1 $O/f32_lb.log | cut -c1-200
timeout -k 10 200 python -u benchmarks/fused_waves.py --n 512 --variants 42,46 --rounds 2 --mode 12 > $O/waves_f64.log 2>&1 || { echo WAVES_FAIL; tail -20 $O/waves_f64.log; exit 1; }
grep -v Gloo $O/waves_f64.log | grep -E "variant|f6/auto" | cut -c1-330
