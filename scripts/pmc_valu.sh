# One PMC pass over the plain stencil (variant 11) and the fused kernel: VALU activity and FP64 op counts.
set -o pipefail
O=gpurun_out/pmc; mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $R/$O/valu -o run -- python3 $R/benchmarks/stencil_once.py --variants 11,0 --reps 2 > $R/$O/valu.log 2>&1 || { echo PMC_FAIL; tail -20 $R/$O/valu.log; exit 1; }
f=$(find $R/$O/valu -name '*counter_collection.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(dict)
for r in rows:
    if 'stencil' not in r['Kernel_Name'] and 'vkernel' not in r['Kernel_Name']:
        continue
    k = (r['Dispatch_Id'], r['Kernel_Name'][:60])
    agg[k][r['Counter_Name']] = float(r['Counter_Value'])
    agg[k]['_t'] = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
for k, c in agg.items():
    print(k[0], k[1], {n: round(v, 1) for n, v in sorted(c.items())})
PY
