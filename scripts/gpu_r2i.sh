# Round 2 verification final round-2 tree, rebuilt .so: smoke, driver-style bench x2 (warm-up fix), full
# GPU suite, loopback bench, self-launched 2-rank shared-GPU bench, kernel stats.
set -o pipefail
O=gpurun_out/r2i; mkdir -p $O
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
for i in 1 2; do
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench$i.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench$i.log; exit 1; }
python3 -c "import json,sys; d=json.loads([l for l in open('$O/bench$i.log') if l.startswith('{')][-1]); c=d['config']; print('bench', d['ms_per_step'], c['stencil_variant'], c['stencil_grid_rounds'], min(c['stencil_variant_ms'].values()), c.get('warmup_steps_run'))"
done
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail 8 --timeout 170 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log; grep -E "^FAILED|^ERROR" $O/pytest_gpu.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo PYTEST_ABNORMAL rc=$rc; exit 1; }
timeout -k 10 300 python bench.py --loopback --periodic --steps 100 --warmup 10 > $O/bench_lb.log 2>&1 || { echo BENCH_LB_FAIL; tail -30 $O/bench_lb.log; exit 1; }
grep -E "A/B|validation" $O/bench_lb.log | cut -c1-600; tail -1 $O/bench_lb.log | cut -c1-300
timeout -k 10 300 python bench.py --gpus 2 --share-gpu --n 192 --steps 50 --warmup 5 --launch-timeout 250 > $O/b2_self.log 2>&1 || { echo B2_FAIL; tail -30 $O/b2_self.log; exit 1; }
grep -E "A/B|validation" $O/b2_self.log | cut -c1-600; tail -1 $O/b2_self.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp && R=$GRAFT_REPO_ROOT
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- python3 $R/bench.py --steps 50 --warmup 5 > $R/$O/prof.log 2>&1 || { echo PROF_FAIL; tail -20 $R/$O/prof.log; exit 1; }
find $R/$O/prof -name '*kernel_stats.csv'
