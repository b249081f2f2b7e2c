# Kernel trace of the 1-GPU plain step (graph replay): inter-kernel gaps.
set -o pipefail
O=gpurun_out/pprof; mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/prof -o run -- python3 $R/bench.py --steps 20 --warmup 2 > $R/$O/prof.log 2>&1 || { echo PROF_FAIL; tail -20 $R/$O/prof.log; exit 1; }
t=$(find $R/$O/prof -name '*kernel_trace.csv' | head -1)
python3 $R/benchmarks/timeline.py $t --last 8 > $R/$O/timeline.txt && cat $R/$O/timeline.txt
