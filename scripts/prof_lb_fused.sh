# Kernel trace of the loopback fused steady state (graph replays): stencil, sync, gaps.
set -o pipefail
O=gpurun_out/prof_lbf; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && R=$GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- python3 $R/bench.py --loopback --periodic-dims xy --steps 60 --warmup 10 --fused on > $R/$O/prof.log 2>&1 || { echo PROF_FAIL; tail -20 $R/$O/prof.log; exit 1; }
find $R/$O/prof -name '*kernel_trace.csv' | head -2
