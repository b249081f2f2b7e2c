# Pack mode (kernel vs hipMemcpy2DAsync) correctness + halo-only timings, 512^3 f64.
set -o pipefail
O=gpurun_out/pack; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_halo.py -k "memcpy2d" > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for pk in kernel memcpy2d; do
  for sf in "--self" ""; do
    IGG_HALO_MODE=sequential IGG_PACK=$pk timeout -k 10 120 python -u benchmarks/halo_only.py --n 512 --reps 50 $sf >> $O/halo.log 2>&1 || { echo HALO_FAIL; tail -20 $O/halo.log; exit 1; }
  done
done
grep halo_us $O/halo.log
