#!/usr/bin/env python3
"""Cost of the z-unpack copy of the fused corner step (FusedHalo::unpack_z) in
isolation: one z side of an n^3 field, the received face [x][y] (row pitch
zp) copied into the halo column z = n-1 of rows x, y in [1, n-2] (one 8-B
element per 4 KiB row). Source in torch (coarse-grained) or native
fine-grained memory (the put arena's kind), destination likewise; alone and
right after a 1 GiB streaming copy (the stencil's write stream before it in a
step). CUDA-event timing, median of 5 x reps.

Usage: python benchmarks/unpack_probe.py [--n 512] [--reps 50]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import igg  # noqa: E402,F401
from igg._native import native  # noqa: E402
from igg.models.diffusion3d import native_buffer  # noqa: E402


def timed(fn, reps, pre=None):
    """us per call: ``reps`` back-to-back calls in one event bracket, or (with
    ``pre``) each call bracketed alone right behind ``pre`` on the stream."""
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        if pre is None:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) / reps * 1e3)
            continue
        ev = []
        for _ in range(reps):
            pre()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            ev.append((e0, e1))
        torch.cuda.synchronize()
        ts.append(sum(a.elapsed_time(b) for a, b in ev) / reps * 1e3)
    return sorted(ts)[2]


def buf(nbytes, kind):
    if kind == "torch":
        return torch.zeros(nbytes, dtype=torch.uint8, device="cuda")
    return native_buffer(nbytes, 1, torch.device("cuda"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--reps", type=int, default=30)
    a = ap.parse_args()
    n, eb = a.n, 8
    zp = -(-(n - 2) // 16) * 16
    s = torch.cuda.current_stream().cuda_stream
    big_a = torch.rand(n, n, n, dtype=torch.float64, device="cuda")
    big_b = torch.empty_like(big_a)
    for skind in ("torch", "fine"):
        for dkind in ("torch", "fine"):
            src = buf(n * zp * eb, skind).view(torch.float64).view(n, zp)
            src.copy_(torch.rand(n, zp, dtype=torch.float64, device="cuda"))
            T = buf(n * n * n * eb, dkind).view(torch.float64).view(n, n, n)
            one = [(src.data_ptr() + 1 * zp * eb, T.data_ptr() + ((1 * n + 1) * n + n - 1) * eb,
                    n - 2, n - 2, zp, 1, n * n, n)]
            both = one + [(src.data_ptr() + 1 * zp * eb, T.data_ptr() + ((1 * n + 1) * n) * eb,
                           n - 2, n - 2, zp, 1, n * n, n)]
            t1 = timed(lambda: native.copy2d(one, eb, True, s), a.reps)
            t2 = timed(lambda: native.copy2d(both, eb, True, s), a.reps)
            t1p = timed(lambda: native.copy2d(one, eb, True, s), a.reps, pre=lambda: big_b.copy_(big_a))
            col = T[1:n - 1, 1:n - 1, n - 1]
            tf = timed(lambda: col.fill_(1.0), a.reps)  # the scattered stores alone
            tt = timed(lambda: col.copy_(src[1:n - 1, :n - 2]), a.reps)  # torch's strided copy
            print(f"src {skind:5s} dst {dkind:5s}: one side {t1:6.2f} us, both sides {t2:6.2f} us, "
                  f"one side after a 1 GiB copy {t1p:6.2f} us | torch fill of the column {tf:6.2f} us, "
                  f"torch copy {tt:6.2f} us", flush=True)
            ref = T.clone()
            native.copy2d(one, eb, True, s)
            torch.cuda.synchronize()
            ref[1:n - 1, 1:n - 1, n - 1] = src[1:n - 1, :n - 2]
            assert torch.equal(ref, T), "unpack mismatch"
            del T, src, ref
    print("unpack check: bitwise OK")


if __name__ == "__main__":
    main()
