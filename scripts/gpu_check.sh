set -o pipefail
mkdir -p gpurun_out/r12
timeout -k 10 700 python -m pytest tests -m gpu -x -q > gpurun_out/r12/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/r12/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r12/pytest_gpu.log
for t in rccl put; do
  timeout -k 10 180 python bench.py --steps 200 --warmup 20 --loopback --periodic --transport $t > gpurun_out/r12/bench_lb_$t.log 2>&1 || { echo BENCH_FAIL $t; tail -20 gpurun_out/r12/bench_lb_$t.log; exit 1; }
  echo "== $t $(grep -o '"ms_per_step": [0-9.]*\|"phase_ms": {[^}]*}' gpurun_out/r12/bench_lb_$t.log | tr '\n' ' ')"
done
cd /tmp && export TMPDIR=/tmp && R=$GRAFT_REPO_ROOT
IGG_TRACE=1 timeout -k 10 200 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $R/gpurun_out/r12/mtrace -o run -- python3 $R/bench.py --steps 20 --warmup 2 --loopback --periodic --transport put --no-graph > $R/gpurun_out/r12/mtrace.log 2>&1; echo mtrace rc=$?
ls $R/gpurun_out/r12/mtrace
