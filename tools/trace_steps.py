#!/usr/bin/env python3
"""Per-step timeline summary of a rocprofv3 kernel trace (CSV).

Takes the last ``--steps`` occurrences of the step's main kernel (a substring
of the kernel name, default the stencil/fused kernels) and reports, per step:
the main kernel's duration, every other kernel between two main kernels
(name, duration) and the idle gaps, as means over the steps. Answers "where
does a time step go besides the stencil" from a trace of the timed loop.

Usage: python tools/trace_steps.py TRACE.csv [--main diffusion3d] [--steps 40]
"""
import argparse
import csv
import re
from collections import defaultdict


def short(name: str) -> str:
    m = re.search(r"(diffusion3d_\w+?kernel|put_\w+kernel|copy2d_batch_kernel|\w*nccl\w*|\w+kernel)", name)
    return m.group(1) if m else name[:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--main", default="diffusion3d")
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--skip-last", type=int, default=0,
                    help="ignore the last K main kernels (e.g. eager phase-timing steps after the timed loop)")
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    mains = [i for i, r in enumerate(rows) if a.main in r[2]]
    if len(mains) < 3:
        raise SystemExit("fewer than 3 main kernels in the trace")
    if a.skip_last:
        mains = mains[:-a.skip_last]
    mains = mains[-(a.steps + 1):]
    dur_main, others, gaps, steps = [], defaultdict(list), [], []
    for i0, i1 in zip(mains[:-1], mains[1:]):
        s0, e0, _ = rows[i0]
        dur_main.append((e0 - s0) / 1e3)
        steps.append((rows[i1][0] - s0) / 1e3)
        t = e0
        gap = 0.0
        for j in range(i0 + 1, i1):
            s, e, n = rows[j]
            gap += max(0, s - t) / 1e3
            others[short(n)].append((e - s) / 1e3)
            t = max(t, e)
        gap += max(0, rows[i1][0] - t) / 1e3
        gaps.append(gap)
    k = len(steps)
    print(f"{k} steps: step {sum(steps) / k:.2f} us = main kernel {sum(dur_main) / k:.2f} us"
          f" + other kernels {sum(sum(v) for v in others.values()) / k:.2f} us + idle gaps {sum(gaps) / k:.2f} us")
    for n, v in sorted(others.items(), key=lambda kv: -sum(kv[1])):
        print(f"  {n}: {len(v) / k:.1f} per step, {sum(v) / len(v):.2f} us each")


if __name__ == "__main__":
    main()
