# FETCH_SIZE (x2 calibrated: a 1 GiB copy reports 0.5 GiB) of the plain stencil vs grid rounds (chunk length along x).
set -o pipefail
O=gpurun_out/pmcr; mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O/fetch -o run -- python3 $R/benchmarks/stencil_once.py --variants 24,11 --rounds 1,2,3,-4 --reps 2 > $R/$O/fetch.log 2>&1 || { echo PMC_FAIL; tail -20 $R/$O/fetch.log; exit 1; }
f=$(find $R/$O/fetch -name '*counter_collection.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(dict)
for r in rows:
    n = r['Kernel_Name']
    if 'diffusion3d' not in n:
        continue
    k = int(r['Dispatch_Id'])
    agg[k]['kernel'] = 'hx' if 'hx_kernel' in n else 'vkernel'
    agg[k]['grid'] = r.get('Grid_Size', '?')
    agg[k]['FETCH_GiB_x2'] = agg[k].get('FETCH_GiB_x2', 0.0) + 2 * float(r['Counter_Value']) / 2**20
    agg[k]['us'] = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
for k in sorted(agg):
    c = agg[k]
    print(k, c['kernel'], 'grid', c['grid'], 'fetch %.3f GiB' % c['FETCH_GiB_x2'], '%.1f us' % c['us'])
PY
