# Edge-lane z sends with the LDS read deferred one step (DF modes of variants 42/44/45): bitwise tests, A/B.
set -o pipefail
O=gpurun_out/zdl; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_fused.py -q -x -k "42 or 44 or 45" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
IGG_FUSED_CANDIDATES=42/12/2,42/13/2,42/4/2,42/5/2,40/12/2,45/12/3,45/13/3 timeout -k 10 400 python -u bench.py --loopback --periodic --steps 100 --warmup 10 > $O/f64_lb.log 2>&1 || { echo F64_FAIL; tail -30 $O/f64_lb.log; exit 1; }
grep -E "A/B" $O/f64_lb.log | cut -c1-1500; tail -1 $O/f64_lb.log | cut -c1-200
IGG_FUSED_CANDIDATES=44/12/3,44/13/3,44/12/4,44/13/4 IGG_TRANSPORT=put timeout -k 10 400 python -u bench.py --config diffusion3d_f32_gather --loopback --periodic --steps 100 --warmup 10 > $O/f32_lb.log 2>&1 || { echo F32_FAIL; tail -30 $O/f32_lb.log; exit 1; }
grep -E "A/B" $O/f32_lb.log | cut -c1-1500; tail -1 $O/f32_lb.log | cut -c1-200
