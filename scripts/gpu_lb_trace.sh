# Loopback (interior-rank emulation) benches + kernel-trace timeline of the put step.
set -o pipefail
O=gpurun_out/lb; mkdir -p $O
for t in put rccl; do
  timeout -k 10 180 python bench.py --steps 200 --warmup 20 --loopback --periodic --transport $t > $O/bench_lb_$t.log 2>&1 || { echo BENCH_FAIL $t; tail -20 $O/bench_lb_$t.log; exit 1; }
  echo "== $t $(tail -1 $O/bench_lb_$t.log | grep -o '"ms_per_step": [0-9.]*')"
done
cd /tmp && export TMPDIR=/tmp && R=$GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$O/ktrace -o run -- python3 $R/bench.py --steps 20 --warmup 2 --loopback --periodic --transport put --no-graph > $R/$O/ktrace.log 2>&1 || { echo TRACE_FAIL; tail -20 $R/$O/ktrace.log; exit 1; }
python3 $R/benchmarks/timeline.py $(find $R/$O/ktrace -name '*kernel_trace.csv' | head -1) --last 24 > $R/$O/timeline_put.txt
cat $R/$O/timeline_put.txt
