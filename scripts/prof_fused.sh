# rocprofv3 kernel stats + trace of the fused loopback step (interior rank emulation).
set -o pipefail
export IGG_PUT_TIMEOUT=20
O=gpurun_out/fprof; mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- python3 $R/bench.py --steps 40 --warmup 4 --loopback --periodic --fused on ${GRAPH_FLAG:---no-graph} > $R/$O/prof.log 2>&1 || { echo PROF_FAIL; tail -20 $R/$O/prof.log; exit 1; }
f=$(find $R/$O/prof -name '*kernel_stats.csv' | head -1)
cp $f $R/$O/kernel_stats.csv
python3 -c "
import csv
rows=list(csv.DictReader(open('$f')))
for r in rows[:12]:
    print(f\"{float(r['AverageNs'])/1e3:9.1f} us x{r['Calls']:>5} {float(r['Percentage']):5.1f}%  {r['Name'][:110]}\")
"
t=$(find $R/$O/prof -name '*kernel_trace.csv' | head -1)
python3 $R/benchmarks/timeline.py $t --last 12 > $R/$O/timeline.txt && cat $R/$O/timeline.txt
