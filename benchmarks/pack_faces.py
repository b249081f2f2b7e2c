#!/usr/bin/env python3
"""Per-face pack/unpack cost of the batched copy kernel (1 GPU, no transport).

For each dim of an n^3 field: pack both send planes into a contiguous buffer
(what update_halo_ launches before a send) and unpack a buffer into both halo
planes, timed alone with CUDA events (median of 5 x reps). Reports us per call
and the effective GB/s on the payload bytes.

Usage: python benchmarks/pack_faces.py [--n 512] [--reps 50] [--dtype float64]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import igg  # noqa: E402,F401
from igg._native import native  # noqa: E402


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) / reps * 1e3)
    return sorted(ts)[2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--dtype", default="float64")
    a = ap.parse_args()
    n = a.n
    dt = getattr(torch, a.dtype)
    T = torch.rand(n, n, n, dtype=dt, device="cuda") if dt.is_floating_point else \
        torch.randint(0, 100, (n, n, n), dtype=dt, device="cuda")
    eb = T.element_size()
    buf = torch.empty(2 * n * n, dtype=dt, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    st = T.stride()
    base = T.data_ptr()
    out = {}
    for d in range(3):
        o = [k for k in range(3) if k != d]
        inner, outer = (o[1], o[0]) if st[o[1]] < st[o[0]] else (o[0], o[1])
        planes = [(1, 0), (n - 2, n * n)]  # (send index, buffer offset)
        pack = [(base + i * st[d] * eb, buf.data_ptr() + off * eb, n, n, st[outer], st[inner], n, 1)
                for i, off in planes]
        unpack = [(buf.data_ptr() + off * eb, base + i * st[d] * eb, n, n, n, 1, st[outer], st[inner])
                  for i, off in ((0, 0), (n - 1, n * n))]
        tp = timed(lambda: native.copy2d(pack, eb, True, s), a.reps)
        tu = timed(lambda: native.copy2d(unpack, eb, True, s), a.reps)
        payload = 2 * n * n * eb * 2  # read + write
        out[d] = (tp, tu)
        print(f"dim {d} (inner stride {st[inner]}): pack {tp:7.2f} us ({payload / tp / 1e3:7.1f} GB/s)  "
              f"unpack {tu:7.2f} us ({payload / tu / 1e3:7.1f} GB/s)", flush=True)
    # Paired form of the strided dim: ONE copy whose inner extent is the 2 sides
    # (z=1 and z=n-2 of the same row are read by adjacent lanes: same 4 KiB
    # page, possibly the same DRAM row) and whose outer index runs over all
    # n*n rows (x and y strides collapse: st[0] = n * st[1]).
    d = 2
    pair_pack = [(base + 1 * eb, buf.data_ptr(), n * n, 2, st[1], (n - 3), 1, n * n)]
    pair_unpack = [(buf.data_ptr(), base, n * n, 2, 1, n * n, st[1], (n - 1))]
    tp = timed(lambda: native.copy2d(pair_pack, eb, True, s), a.reps)
    tu = timed(lambda: native.copy2d(pair_unpack, eb, True, s), a.reps)
    payload = 2 * n * n * eb * 2
    print(f"dim 2 paired sides: pack {tp:7.2f} us ({payload / tp / 1e3:7.1f} GB/s)  "
          f"unpack {tu:7.2f} us ({payload / tu / 1e3:7.1f} GB/s)", flush=True)
    ref = T.clone()
    native.copy2d(pair_pack, eb, True, s)
    native.copy2d(pair_unpack, eb, True, s)
    torch.cuda.synchronize()
    ref.select(2, 0).copy_(ref.select(2, 1))
    ref.select(2, n - 1).copy_(ref.select(2, n - 2))
    assert torch.equal(ref, T), "paired round trip mismatch"
    del ref
    # check: pack/unpack round trip of every dim reproduces the planes
    for d in range(3):
        ref = T.clone()
        o = [k for k in range(3) if k != d]
        inner, outer = (o[1], o[0]) if st[o[1]] < st[o[0]] else (o[0], o[1])
        pack = [(base + i * st[d] * eb, buf.data_ptr() + off * eb, n, n, st[outer], st[inner], n, 1)
                for i, off in ((1, 0), (n - 2, n * n))]
        unpack = [(buf.data_ptr() + off * eb, base + i * st[d] * eb, n, n, n, 1, st[outer], st[inner])
                  for i, off in ((0, 0), (n - 1, n * n))]
        native.copy2d(pack, eb, True, s)
        native.copy2d(unpack, eb, True, s)
        torch.cuda.synchronize()
        ref.select(d, 0).copy_(ref.select(d, 1))
        ref.select(d, n - 1).copy_(ref.select(d, n - 2))
        assert torch.equal(ref, T), f"dim {d}: round trip mismatch"
        del ref
    print("round trip: bitwise OK")


if __name__ == "__main__":
    main()
