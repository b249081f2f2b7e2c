#!/usr/bin/env python3
"""Where the fused kernel's time goes, per wave (1 GPU, self as peer).

The fused kernel dispatches every wave to a sweep specialised to the exchange
features its tile touches (class bits: 1 = x chunk, 2 = y edge rows, 4 = z edge
tile). With native.fused_debug(stamps) each wave records {class, start, end,
hw id} (wall_clock64 ticks, 100 MHz). For each configuration this prints the
kernel time (CUDA events, median), and per class: wave count, mean/max wave
duration and the latest end relative to the kernel's first start.

force_sel runs every wave with one class (timing only: 0 on an exchanging
grid skips its exchange): 'auto' vs 'all0' separates the cost of the boundary
waves' work from the cost of merely having the exchange code in the kernel.

Usage: python benchmarks/fused_waves.py [--n 512] [--variants 40,0] [--rounds 2] [--mode 0] [--dtype float64]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import igg  # noqa: E402
from igg._native import native  # noqa: E402

PLAIN_OF = {50: 0, 55: 0, 41: 40, 42: 40, 44: 14, 45: 0, 48: 9}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--variants", default="40,0")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--mode", type=int, default=0)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--dtype", default="float64", choices=["float64", "float32"])
    ap.add_argument("--shape", default="xyz",
                    help="neighbour sides of the exchanging halo (rank_shapes.py names: xyz = 6 faces, "
                         "xyz+ = a 2x2x2 corner rank with coords 0, ...)")
    a = ap.parse_args()
    n = a.n
    igg.init_global_grid(n, n, n, periodx=1, periody=1, periodz=1, quiet=True)
    dt = getattr(torch, a.dtype)
    T = torch.rand(n, n, n, dtype=dt, device="cuda")
    T2 = T.clone()
    Cp = torch.rand(n, n, n, dtype=dt, device="cuda") + 1
    rd2 = [1.0, 1.0, 1.0]
    eb = T.element_size()
    s = torch.cuda.current_stream().cuda_stream
    inner = [([1, 1, 1], [n - 1, n - 1, n - 1])]
    mesh = native.PeerMesh(0, 1, lambda b: [bytes(b)])
    dims = a.shape.rstrip("+-")
    side = a.shape[len(dims):] or "+-"
    nb = [[0 if (d in dims and "-" in side) else -1, 0 if (d in dims and "+" in side) else -1] for d in "xyz"]
    fh6 = native.FusedHalo(mesh, [n, n, n], eb, nb)
    # its own mesh: a neighbourless halo advances EPOCH without publishing
    # ARRIVED, which would stall fh6's in-kernel step sync on a shared flag block
    fh0 = native.FusedHalo(native.PeerMesh(0, 1, lambda b: [bytes(b)]), [n, n, n], eb,
                           [[-1, -1], [-1, -1], [-1, -1]])
    if a.mode & 4:  # direct z: the z sends land in the halo column of the other buffer
        fh6.set_fields(T.data_ptr(), T2.data_ptr())
    stamps = torch.zeros(1 << 22, dtype=torch.int64, device="cuda")
    k = [0]

    def fused(fh, v):
        fh.step(T2.data_ptr(), T.data_ptr(), Cp.data_ptr(), rd2, 1e-4, v, k[0], True, s, a.rounds, a.mode)
        k[0] += 1

    def ev_time(fn):
        fn()
        ts = []
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) / a.reps)
        return sorted(ts)[1]

    print(f"n={n}^3 {a.dtype} rounds={a.rounds} mode={a.mode} shape={a.shape} (nb {nb}): ms per step (stencil + "
          f"sync), per-class wave stats in us")
    for v in (int(x) for x in a.variants.split(",")):
        pv = PLAIN_OF.get(v, v)
        tp = ev_time(lambda: native.diffusion3d(T2.data_ptr(), T.data_ptr(), Cp.data_ptr(), [n, n, n], rd2, 1e-4,
                                                eb, inner, True, pv, s, a.rounds))
        print(f"variant {v}: plain {tp:.4f}")
        for label, fh, force in (("none/auto", fh0, -1), ("none/all0", fh0, 0), ("none/all7", fh0, 7),
                                 ("f6/auto", fh6, -1), ("f6/all7", fh6, 7)):
            native.fused_debug(0, force)
            t = ev_time(lambda: fused(fh, v))
            stamps.zero_()
            native.fused_debug(stamps.data_ptr(), force)
            fused(fh, v)
            torch.cuda.synchronize()
            native.fused_debug(0, -1)
            st = stamps.view(-1, 4).cpu()
            st = st[st[:, 1] != 0]
            t0 = int(st[:, 1].min())
            row = []
            for c in sorted(set(st[:, 0].tolist())):
                m = st[st[:, 0] == c]
                d = (m[:, 2] - m[:, 1]).double() / 100.0
                row.append(f"c{c}: {m.shape[0]} waves {d.mean():.1f}/{d.max():.1f} us end {(int(m[:, 2].max()) - t0) / 100:.1f}")
            span = (int(st[:, 2].max()) - t0) / 100.0
            print(f"  {label:10s} {t:.4f} ms  span {span:.1f} us | " + " | ".join(row), flush=True)
    mesh.check_error()
    igg.finalize_global_grid()


if __name__ == "__main__":
    main()
