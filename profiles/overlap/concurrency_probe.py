#!/usr/bin/env python3
"""How long does a small communication-like op take while the big interior
stencil kernel runs on another stream?  (Decides how to overlap halo exchange.)

For each small op X (RCCL self send/recv 2x2 MiB, copy2d kernel 2 MiB strided,
hipMemcpyAsync D2D 4 MiB) and each placement (alone; concurrent on a
high-priority stream; concurrent with CU-masked streams reserving R CUs) we
time X with events on its own stream, plus the big kernel's duration.

Usage: python profiles/overlap/concurrency_probe.py [--n 512] [--reps 5]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--delay-us", type=float, default=100.0, help="host delay before launching the small op")
    ap.add_argument("--reserve", default="0,8,16,32")
    a = ap.parse_args()
    import torch

    import igg
    from igg._native import native
    from igg.ops import stencil
    from igg.utils.streams import cu_partition

    igg.init_global_grid(a.n, a.n, a.n, quiet=True)
    dev = torch.device("cuda", 0)
    n = a.n
    T = torch.rand(n, n, n, dtype=torch.float64, device=dev)
    Cp = 1 + torch.rand(n, n, n, dtype=torch.float64, device=dev)
    T2 = T.clone()
    kw = dict(lam=1.0, dt=1e-4, dx=0.1, dy=0.1, dz=0.1)
    inner = [stencil.inner_box(T.shape)]
    comm = native.RcclComm(native.RcclComm.unique_id(), 1, 0)
    src = torch.rand(2 * n * n, dtype=torch.float64, device=dev)
    dst = torch.empty_like(src)
    nbytes = n * n * 8

    def op_rccl(s):
        comm.p2p([(dst.data_ptr(), nbytes, 0), (dst.data_ptr() + nbytes, nbytes, 0)],
                 [(src.data_ptr(), nbytes, 0), (src.data_ptr() + nbytes, nbytes, 0)], s.cuda_stream)

    def op_copy2d(s):  # z-face-like strided pack of one plane of T (n*n rows, 1 element each)
        native.copy2d([(T.data_ptr() + 8, dst.data_ptr(), n * n, 1, n, 1, 1, 1)], 8, True, s.cuda_stream)

    def op_memcpy(s):
        with torch.cuda.stream(s):
            dst.copy_(src, non_blocking=True)

    ops = {"rccl_2x2MiB": op_rccl, "copy2d_zplane": op_copy2d, "memcpy_4MiB": op_memcpy}

    def run_big(s):
        stencil.diffusion3d_(T2, T, Cp, boxes=inner, variant=0, stream=s.cuda_stream, **kw)

    def measure(op, big_stream, small_stream, concurrent):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        ts, tb = [], []
        for _ in range(a.reps):
            torch.cuda.synchronize()
            if concurrent:
                e[2].record(big_stream)
                run_big(big_stream)
                e[3].record(big_stream)
                t0 = time.perf_counter()
                while (time.perf_counter() - t0) * 1e6 < a.delay_us:
                    pass
            e[0].record(small_stream)
            op(small_stream)
            e[1].record(small_stream)
            torch.cuda.synchronize()
            ts.append(e[0].elapsed_time(e[1]) * 1e3)
            if concurrent:
                tb.append(e[2].elapsed_time(e[3]) * 1e3)
        med = lambda v: sorted(v)[len(v) // 2] if v else None  # noqa: E731
        return med(ts), med(tb)

    main_s = torch.cuda.current_stream()
    _lo, hi = torch.cuda.Stream.priority_range()
    prio = torch.cuda.Stream(device=dev, priority=hi)
    for name, op in ops.items():  # warm up
        op(prio)
    run_big(main_s)
    torch.cuda.synchronize()
    out = {}
    for name, op in ops.items():
        out[f"{name}/alone"] = measure(op, main_s, prio, False)[0]
        out[f"{name}/prio"] = measure(op, main_s, prio, True)
    out["big/alone"] = measure(lambda s: None, main_s, prio, True)[1]
    for r in [int(x) for x in a.reserve.split(",") if int(x) > 0]:
        cs, hs = cu_partition(r)
        for name, op in ops.items():
            out[f"{name}/cu{r}"] = measure(op, cs, hs, True)
    for k, v in out.items():
        print(f"{k:28s} {v}", flush=True)
    print(json.dumps(out))
    comm.abort()
    igg.finalize_global_grid()


if __name__ == "__main__":
    main()
