# Kernel trace of fused_sweep: inter-kernel gaps per FusedHalo configuration.
set -o pipefail
export IGG_PUT_TIMEOUT=10
O=gpurun_out/gap; mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/prof -o run -- python3 $R/benchmarks/gap_probe.py $GAP_ARGS > $R/$O/prof.log 2>&1 || { echo PROF_FAIL; tail -20 $R/$O/prof.log; exit 1; }
t=$(find $R/$O/prof -name '*kernel_trace.csv' | head -1)
python3 - "$t" <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
rows = [r for r in rows if 'hx_kernel' in r['Kernel_Name'] or 'put_sync' in r['Kernel_Name'] or 'vkernel' in r['Kernel_Name']]
prev = None
out = []
for r in rows:
    nm = 'hx' if 'hx_kernel' in r['Kernel_Name'] else ('sync' if 'put_sync' in r['Kernel_Name'] else 'plain')
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    if prev:
        out.append(f"{prev[0]:>5}->{nm:<5} gap {(s - prev[2]) / 1e3:7.1f} us   {nm} dur {(e - s) / 1e3:7.1f} us")
    prev = (nm, s, e)
print("\n".join(out))
PY
