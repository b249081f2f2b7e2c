# HBM traffic (FETCH_SIZE, WRITE_SIZE passes) of stencil variants 43 (full-row z tiles), 40 and 24 at 3 rounds, 512^3 f64.
# Expected compulsory traffic per launch: read T + Cp = 2.147 GB, write T2 = 1.073 GB.
set -o pipefail
O=gpurun_out/pmc43; mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O/fetch -o run -- python3 $R/benchmarks/stencil_once.py --variants 43,40,24 --rounds 3 --reps 2 --calib > $R/$O/fetch.log 2>&1 || { echo PMC1_FAIL; tail -20 $R/$O/fetch.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$O/write -o run -- python3 $R/benchmarks/stencil_once.py --variants 43,40,24 --rounds 3 --reps 2 --calib > $R/$O/write.log 2>&1 || { echo PMC2_FAIL; tail -20 $R/$O/write.log; exit 1; }
for d in fetch write; do
f=$(find $R/$O/$d -name '*counter_collection.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(dict)
for r in rows:
    n = r['Kernel_Name']
    if (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) < 100000:
        continue
    k = (int(r['Dispatch_Id']), n[n.find('<'):n.find('>')+1] if 'hx_kernel' in n else ('vkernel' if 'vkernel' in n else 'copy(calib)'))
    agg[k][r['Counter_Name']] = agg[k].get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
    agg[k]['_us'] = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
for k in sorted(agg):
    c = agg[k]
    print(k, {n: (round(v, 0) if 'SIZE' in n else round(v, 1)) for n, v in sorted(c.items())})
PY
done
