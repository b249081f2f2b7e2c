# Fused halo exchange: GPU tests (single process + multi-rank on one GPU), loopback bench.
set -o pipefail
export IGG_PUT_TIMEOUT=10
O=gpurun_out/fused; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fused.py > $O/pytest_fused.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest_fused.log; exit 1; }
tail -3 $O/pytest_fused.log
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_multiprocess.py -k fused > $O/pytest_mp_fused.log 2>&1 || { echo MP_FAIL; tail -40 $O/pytest_mp_fused.log; exit 1; }
tail -3 $O/pytest_mp_fused.log
timeout -k 10 240 python bench.py --steps 200 --warmup 20 --loopback --periodic --transport put > $O/bench_lb_fused.log 2>&1 || { echo BENCH_FAIL; tail -30 $O/bench_lb_fused.log; exit 1; }
grep -v Gloo $O/bench_lb_fused.log | tail -4
