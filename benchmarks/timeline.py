#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel_trace.csv as a per-step timeline.

Usage: python benchmarks/timeline.py <kernel_trace.csv> [--last K]
Prints every dispatch of the last K diffusion steps with start/end relative to
the first dispatch shown, its queue (stream) and duration.
"""
import argparse
import csv


def short(name: str) -> str:
    for key, s in (("diffusion3d_vkernel", "stencil.v"), ("diffusion3d_kernel", "stencil.s"),
                   ("copy2d_batch", "copy2d"), ("nccl", "rccl"), ("Nccl", "rccl")):
        if key in name:
            tmpl = name[name.find("<"):name.find(">") + 1] if "<" in name else ""
            return s + tmpl[:40]
    return name[:50]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--last", type=int, default=40)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[-a.last:]
    t0 = int(rows[0]["Start_Timestamp"])
    for r in rows:
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        print(f"{s / 1e3:10.1f} {e / 1e3:10.1f} {(e - s) / 1e3:8.1f} us  q{r.get('Queue_Id', '?'):>3} "
              f"grid={r.get('Grid_Size_X', r.get('Grid_Size', '?')):>9} wg={r.get('Workgroup_Size_X', '?'):>4} "
              f"vgpr={r.get('VGPR_Count', '?'):>4} {short(r['Kernel_Name'])}")


if __name__ == "__main__":
    main()
