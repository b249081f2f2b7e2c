#!/usr/bin/env python3
"""Stencil kernel variant sweep on one GPU (correctness + interleaved timing).

1. correctness: every variant vs the C++ host kernel on odd-sized grids and
   random sub-boxes (bitwise for f64 is not required: the host and device
   compile the same expression, max |err| is reported);
2. timing at n^3 (default 512, f64): rounds of all variants interleaved in one
   process (cdna_hip_programming.md §5.4 rule 24), median + min reported,
   T_eff = 3*n^3*sizeof / t;
3. roofline reference: torch copy of a 2 GiB buffer (read+write bytes / t).
"""
import argparse
import json
import statistics
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import igg  # noqa: E402
from igg._native import native  # noqa: E402


def run(v, T2, T, Cp, boxes, rd2, dtlam, stream):
    native.diffusion3d(T2.data_ptr(), T.data_ptr(), Cp.data_ptr(), list(T.shape), rd2, dtlam,
                       T.element_size(), boxes, T.is_cuda, v, stream)


def correctness(dtype):
    g = torch.Generator().manual_seed(0)
    worst = {}
    for shape in [(17, 13, 70), (40, 33, 129), (9, 70, 68), (12, 9, 132), (6, 5, 256), (5, 130, 512)]:
        T = torch.rand(shape, generator=g, dtype=dtype)
        Cp = 1 + torch.rand(shape, generator=g, dtype=dtype)
        boxes_list = [[((1, 1, 1), tuple(s - 1 for s in shape))],
                      [((1, 2, 3), (shape[0] - 2, shape[1] - 1, shape[2] - 4)), ((2, 1, 1), (3, 2, shape[2] - 1))]]
        for boxes in boxes_list:
            ref = T.clone()
            run(0, ref, T, Cp, boxes, [1.1, 0.9, 1.3], 0.05, 0)
            Td, Cd = T.cuda(), Cp.cuda()
            for v in range(len(native.diffusion3d_variants())):
                out = T.clone().cuda()
                run(v, out, Td, Cd, boxes, [1.1, 0.9, 1.3], 0.05, torch.cuda.current_stream().cuda_stream)
                torch.cuda.synchronize()
                err = (out.cpu() - ref).abs().max().item()
                worst[v] = max(worst.get(v, 0.0), err)
    return worst


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--dtype", default="float64")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--grid-rounds", default="1,2,0", help="residency rounds per launch to sweep")
    ap.add_argument("--variants", default="all")
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dtype = getattr(torch, a.dtype)
    names = native.diffusion3d_variants()
    worst = correctness(dtype)
    print(json.dumps({"correctness_max_abs_err": {names[k]: v for k, v in worst.items()}}), flush=True)
    n = a.n
    T = torch.rand((n, n, n), dtype=dtype, device="cuda")
    Cp = 1 + torch.rand((n, n, n), dtype=dtype, device="cuda")
    T2 = T.clone()
    boxes = [((1, 1, 1), (n - 1, n - 1, n - 1))]
    s = torch.cuda.current_stream()
    vs = range(len(names)) if a.variants == "all" else [int(x) for x in a.variants.split(",")]
    grs = [int(x) for x in a.grid_rounds.split(",")]
    times = {(g, v): [] for g in grs for v in vs}
    for g, v in times:
        native.diffusion3d_set_rounds(g)
        run(v, T2, T, Cp, boxes, [1.0, 1.0, 1.0], 0.01, s.cuda_stream)
    ref_out = None
    for r in range(a.rounds):
        for g, v in times:
            native.diffusion3d_set_rounds(g)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(a.reps):
                run(v, T2, T, Cp, boxes, [1.0, 1.0, 1.0], 0.01, s.cuda_stream)
            e1.record(s)
            e1.synchronize()
            times[(g, v)].append(e0.elapsed_time(e1) / a.reps)
            if r == 0:
                if ref_out is None:
                    ref_out = T2.clone()
                elif not torch.equal(T2, ref_out):
                    print(f"variant {names[v]} differs from variant 0: {(T2-ref_out).abs().max().item()}")
    abytes = 3 * n ** 3 * T.element_size()
    res = {}
    for (g, v), ts in sorted(times.items(), key=lambda kv: statistics.median(kv[1])):
        med, mn = statistics.median(ts), min(ts)
        res[f"{names[v]}@r{g}"] = {"ms_median": round(med, 4), "ms_min": round(mn, 4), "T_eff_GBs": round(abytes / (med * 1e-3) / 1e9, 1)}
    # roofline: device copy
    x = torch.empty(2 ** 31 // 8, dtype=torch.float64, device="cuda")
    y = torch.empty_like(x)
    y.copy_(x)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(10):
        y.copy_(x)
    e1.record(s)
    e1.synchronize()
    tc = e0.elapsed_time(e1) / 10
    res["torch_copy_2GiB"] = {"ms": round(tc, 4), "GBs_rw": round(2 * x.numel() * 8 / (tc * 1e-3) / 1e9, 1)}
    print(json.dumps({"n": n, "dtype": a.dtype, "results": res}), flush=True)


if __name__ == "__main__":
    main()
