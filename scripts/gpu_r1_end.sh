# Round-end verification of the rebuilt tree: smoke, gpu tests, 1-GPU bench, kernel stats.
set -o pipefail
O=gpurun_out/r1_end; mkdir -p $O
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 240 python bench.py > $O/bench.log 2>&1 || { echo BENCH_FAIL; tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log
cd /tmp && export TMPDIR=/tmp && R=$GRAFT_REPO_ROOT
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- python3 $R/bench.py --steps 50 --warmup 5 > $R/$O/prof.log 2>&1 || { echo PROF_FAIL; tail -20 $R/$O/prof.log; exit 1; }
find $R/$O/prof -name '*kernel_stats.csv' | head -3
