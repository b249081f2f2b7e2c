# Kernel durations vs wall time of the timed 1-GPU bench (are there gaps between graph-replayed steps?).
set -o pipefail
O=gpurun_out/gaps; mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/trace -o run -- python3 $R/bench.py --steps 200 --warmup 20 > $R/$O/bench.log 2>&1 || { echo FAIL; tail -20 $R/$O/bench.log; exit 1; }
grep '^{' $R/$O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('wall ms/step', d['ms_per_step'], 'variant', d['config']['stencil_variant'], 'rounds', d['config']['stencil_grid_rounds'])"
f=$(find $R/$O/trace -name '*kernel_trace.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if 'diffusion3d' in r['Kernel_Name']]
rows.sort(key=lambda r: int(r['Start_Timestamp']))
last = rows[-200:]  # the timed steps are the last 200 stencil launches
d = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3 for r in last]
gaps = [(int(b['Start_Timestamp']) - int(a['End_Timestamp'])) / 1e3 for a, b in zip(last, last[1:])]
span = (int(last[-1]['End_Timestamp']) - int(last[0]['Start_Timestamp'])) / 1e3
gs = sorted(gaps)
print('kernel us: mean %.1f min %.1f max %.1f' % (sum(d) / len(d), min(d), max(d)))
print('gaps us: mean %.2f median %.2f max %.1f  (count>5us: %d)' % (sum(gaps) / len(gaps), gs[len(gs) // 2], gs[-1], sum(g > 5 for g in gaps)))
print('span per step us: %.1f' % (span / len(last)))
print('kernel name:', last[0]['Kernel_Name'][:90])
PY
