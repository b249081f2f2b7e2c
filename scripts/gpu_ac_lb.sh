# Acoustic 2-D loopback (interior-rank emulation): put vs rccl exchange, kernel timeline of the put step.
set -o pipefail
export IGG_PUT_TIMEOUT=20
O=gpurun_out/aclb; mkdir -p $O
R=$GRAFT_REPO_ROOT
for t in put rccl; do
  timeout -k 10 200 python bench.py --config acoustic2d --loopback --periodic --transport $t > $O/bench_$t.log 2>&1 || { echo BENCH_FAIL $t; tail -20 $O/bench_$t.log; exit 1; }
  echo "== $t $(grep '^{' $O/bench_$t.log | cut -c1-260)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$O/prof -o run -- python3 $R/bench.py --config acoustic2d --loopback --periodic --transport put --steps 20 --warmup 2 > $R/$O/prof.log 2>&1 || { echo PROF_FAIL; tail -20 $R/$O/prof.log; exit 1; }
t=$(find $R/$O/prof -name '*kernel_trace.csv' | head -1)
python3 $R/benchmarks/timeline.py $t --last 40 > $R/$O/timeline.txt
head -40 $R/$O/timeline.txt
