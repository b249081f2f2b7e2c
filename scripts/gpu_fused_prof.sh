# Kernel-level cost of the fused halo exchange: sweep + rocprofv3 kernel trace.
set -o pipefail
export IGG_PUT_TIMEOUT=10
O=gpurun_out/fused; mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python benchmarks/fused_sweep.py --variants ${VARIANTS:-0,11} > $O/sweep.log 2>&1 || { echo SWEEP_FAIL; tail -20 $O/sweep.log; exit 1; }
grep -v Gloo $O/sweep.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- python3 $R/benchmarks/fused_sweep.py --variants ${VARIANTS:-0,11} --reps 10 > $R/$O/prof.log 2>&1 || { echo PROF_FAIL; tail -20 $R/$O/prof.log; exit 1; }
f=$(find $R/$O/prof -name '*kernel_stats.csv' | head -1)
python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in rows[:14]:
    print(f\"{float(r['AverageNs'])/1e3:9.1f} us x{r['Calls']:>5}  {r['Name'][:150]}\")
"
