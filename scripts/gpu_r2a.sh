# Round 2, first GPU pass: smoke, full GPU suite (new failure-path / auto-mode
# tests included; the multigpu tier skips on one GPU), driver-style 1-GPU bench,
# loopback bench (measured auto schedule), self-launched 2-rank shared-GPU bench.
set -o pipefail
O=gpurun_out/r2a; mkdir -p $O
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 240 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo BENCH_FAIL; tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-400
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail 8 --timeout 170 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log; grep -E "^FAILED|^ERROR" $O/pytest_gpu.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo PYTEST_ABNORMAL rc=$rc; exit 1; }
timeout -k 10 300 python bench.py --loopback --periodic --steps 100 --warmup 10 > $O/bench_lb.log 2>&1 || { echo BENCH_LB_FAIL; tail -30 $O/bench_lb.log; exit 1; }
grep -E "A/B|validation" $O/bench_lb.log | cut -c1-400; tail -1 $O/bench_lb.log | cut -c1-300
timeout -k 10 300 python bench.py --gpus 2 --share-gpu --n 192 --steps 50 --warmup 5 --launch-timeout 250 > $O/b2_self.log 2>&1 || { echo B2_FAIL; tail -30 $O/b2_self.log; exit 1; }
grep -E "A/B|validation" $O/b2_self.log | cut -c1-400; tail -1 $O/b2_self.log | cut -c1-300
