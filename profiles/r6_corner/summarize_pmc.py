"""Per-label means of the fused_waves.py counter pass (SQ_* counters, millions
per launch): the launches of each variant come in the script's order - the
plain kernel, then 32 launches per label (none/auto, none/all0, none/all7,
f6/auto, f6/all7). Usage: python summarize_pmc.py pmc/fused_waves_v9_v48_counters.csv"""
import collections
import csv
import sys

LABELS = ["none/auto", "none/all0", "none/all7", "f6/auto", "f6/all7"]
COLS = ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_LDS", "SQ_WAVE_CYCLES")
d = collections.OrderedDict()
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    if "hx_kernel" not in n and "vkernel" not in n:
        continue
    e = d.setdefault(int(r["Dispatch_Id"]), {"name": n[n.find("<"):n.find(">") + 1]})
    e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
seq = []
for e in d.values():
    if not seq or seq[-1][0] != e["name"]:
        seq.append([e["name"], []])
    seq[-1][1].append(e)
print("| kernel | label | " + " | ".join(COLS) + " |")
print("|---" * (len(COLS) + 2) + "|")
for name, v in seq:
    groups = [(LABELS[i], v[i * 32:(i + 1) * 32]) for i in range(5)] if len(v) == 160 else [("plain", v)]
    for label, g in groups:
        print(f"| `{name}` | {label} | " + " | ".join(f"{sum(x[c] for x in g) / len(g) / 1e6:.3f}" for c in COLS) + " |")
