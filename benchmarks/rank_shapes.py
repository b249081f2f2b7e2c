#!/usr/bin/env python3
"""Fused-exchange cost per RANK SHAPE of a real node (1 GPU, self as peer).

The round-3 ratios (1.05x) were measured on an emulated INTERIOR rank (six
faces). An 8-GPU node runs 2x1x1 / 2x2x1 / 2x2x2 decompositions without
periodicity, where every rank has ONE neighbour per split dimension, on the
high side (coordinate 0) or the low side (coordinate 1). This script times,
for each such one-sided shape (and the six-face interior for reference):

  plain   the best plain stencil (variants x grid rounds), no exchange;
  fused   each fused candidate of the bench's A/B (variant / send mode /
          rounds, incl. direct z and peeled x planes), stencil + sync kernel,

all in the time loop's ping-pong shape (T2 = f(T), T = f(T2)), interleaved,
median of rounds. The exchange partner is this rank itself (a one-sided
shape stores into its own arena / fields and reads halos nobody wrote:
timing only, the values are not checked here - tests/test_fused.py checks
them). ratio = best fused / best plain.

Usage: python benchmarks/rank_shapes.py [--n 512] [--dtype float64]
       [--shapes x+,x-,xy+,xy-,xyz+,xyz-,xyz] [--steps 20] [--rounds 5]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import igg  # noqa: E402
from igg._native import native  # noqa: E402

PLAIN = (2, 11, 14, 21, 24, 26, 40, 43, 44)  # ops/stencil.py SHORTLIST
ROUNDS = (1, 2, 3)
# bench.py FUSED_CANDIDATES / FUSED_DIRECT / FUSED_DIRECT_F32 (+ peel bit 8)
FUSED = ((0, 0, 3), (0, 1, 3), (0, 0, 1), (9, 0, 3), (14, 0, 3), (40, 0, 2), (42, 0, 2), (42, 1, 2), (50, 0, 2),
         (11, 0, 2), (11, 2, 2), (11, 8, 2), (11, 10, 2), (14, 0, 2), (9, 0, 2))
DIRECT = ((40, 4, 2), (42, 4, 2), (42, 5, 2), (50, 4, 2), (0, 4, 3))
DIRECT_F32 = ((44, 4, 3), (44, 4, 4), (14, 4, 4))
# z unpack (send mode bit 64, FusedHalo::Z_UNPACK): arena z sends, no z receive
# in the sweep, a copy kernel writes the received z faces after the step sync
ZUNPACK = ((9, 64, 3), (42, 64, 2), (40, 64, 2), (0, 64, 3))
ZUNPACK_F32 = ((44, 64, 4), (14, 64, 3))


def neighbours(shape: str):
    """nb[d] = [low, high] (0 = this rank, -1 = none) of a named shape."""
    dims = shape.rstrip("+-")
    side = shape[len(dims):] or "+-"
    nb = []
    for d in "xyz":
        if d in dims:
            nb.append([0 if "-" in side else -1, 0 if "+" in side else -1])
        else:
            nb.append([-1, -1])
    return nb


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--dtype", default="float64", choices=["float64", "float32"])
    ap.add_argument("--shapes", default="x+,x-,xy+,xy-,xyz+,xyz-,xyz")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--candidates", default=None, help="v/mode/rounds,... (default: the bench's lists)")
    ap.add_argument("--json", default=None, help="write the results here")
    ap.add_argument("--order", type=int, default=3,
                    help="re-time the N fastest forms per z shape with z-edge tiles first (send mode bit 32)")
    ap.add_argument("--inkernel", type=int, default=3,
                    help="re-time the N fastest forms per shape with the in-kernel step sync (send mode bit 16)")
    ap.add_argument("--update-halo", action="store_true",
                    help="also time the generic path per shape: best plain stencil + update_halo_(T2) through the "
                         "loopback emulation of exactly that shape's sides (RCCL sequential / one-phase, put)")
    ap.add_argument("--fused", type=int, default=1, help="0: skip the fused candidates (update_halo_ column only)")
    ap.add_argument("--graph", action="store_true",
                    help="time hipGraph replays of --steps captured steps (the bench's timed form) instead of eager "
                         "launches (--steps must be even)")
    ap.add_argument("--halo-z", type=int, default=1,
                    help="whole-line z-edge stores (DiffusionArgs::halo_z, the model's default) in plain and fused")
    a = ap.parse_args()
    if a.graph and a.steps % 2:
        raise SystemExit("--graph: --steps must be even (the ping-pong buffers return to their roles)")
    n = a.n
    hz = bool(a.halo_z)
    dt = getattr(torch, a.dtype)
    igg.init_global_grid(n, n, n, periodx=1, periody=1, periodz=1, quiet=True)
    from igg.models import diffusion3d as D
    from igg.parallel import grid as _grid
    from igg.utils import placement as PL

    # fine-grained fields in one allocation, as the model allocates them, on
    # the fastest of the placement probe's candidates (utils/placement.py;
    # IGG_FIELD_PLACEMENT=1: whatever the allocator gives)
    nbytes = n * n * n * dt.itemsize

    def views(b):
        return [b[k * (nbytes + 266240):k * (nbytes + 266240) + nbytes].view(dt).view(n, n, n) for k in range(3)]

    cnt = PL.candidate_count(_grid.global_grid(), nbytes, 3 * nbytes, torch.device("cuda", 0))
    buf, placement = PL.placed(lambda: D.native_buffer(3 * nbytes + 2 * 266240, 1, torch.device("cuda", 0)), cnt,
                               lambda cands: D._time_placements([(v[0], v[2], v[1]) for v in map(views, cands)], dt))
    if placement:
        print(f"field placement: {placement['candidates']} candidates, chosen {placement['chosen']} "
              f"({min(placement['ms']):.5f} vs max {max(placement['ms']):.5f} ms)", flush=True)
    T, T2, Cp = views(buf)
    g = torch.Generator(device="cpu").manual_seed(0)
    T.copy_(torch.rand(n, n, n, generator=g, dtype=torch.float64).to(dt))
    T2.copy_(T)
    Cp.copy_(torch.rand(n, n, n, generator=g, dtype=torch.float64).to(dt) + 1)
    rd2 = [1.0, 1.0, 1.0]
    eb = T.element_size()
    if a.graph:  # captures need a non-default stream; every launch below goes to it
        torch.cuda.set_stream(torch.cuda.Stream())
    s = torch.cuda.current_stream()
    inner = [([1, 1, 1], [n - 1, n - 1, n - 1])]
    mesh = native.PeerMesh(0, 1, lambda b: [bytes(b)])
    bufs = [T, T2]

    def plain(v, r, hz_=False):
        k = [0]

        def f():
            src, dst = bufs[k[0] & 1], bufs[(k[0] + 1) & 1]
            native.diffusion3d(dst.data_ptr(), src.data_ptr(), Cp.data_ptr(), [n, n, n], rd2, 1e-4, eb, inner, True,
                               v, s.cuda_stream, r, hz_)
            k[0] += 1
        return f

    def fused(fh, v, mode, r):
        k = [0]

        def f():
            src, dst = bufs[k[0] & 1], bufs[(k[0] + 1) & 1]
            fh.step(dst.data_ptr(), src.data_ptr(), Cp.data_ptr(), rd2, 1e-4, v, k[0], True, s.cuda_stream, r, mode,
                    False, hz)
            k[0] += 1
        return f

    def bench(fns: dict) -> dict:
        for f in fns.values():
            for _ in range(2):
                f()
        runs = dict(fns)
        if a.graph:
            # the steps as the bench's timed region runs them: hipGraph
            # replays (launch gaps of the sync / unpack kernels as in a run)
            runs = {}
            for c, f in fns.items():
                g = torch.cuda.CUDAGraph()
                torch.cuda.synchronize()
                with torch.cuda.graph(g, stream=s):
                    for _ in range(a.steps):
                        f()
                torch.cuda.synchronize()
                runs[c] = g
        times = {c: [] for c in fns}
        for _ in range(a.rounds):
            for c, f in runs.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                if a.graph:
                    f.replay()
                else:
                    for _ in range(a.steps):
                        f()
                e1.record(s)
                e1.synchronize()
                times[c].append(e0.elapsed_time(e1) / a.steps)
        return {c: sorted(t)[len(t) // 2] for c, t in times.items()}

    compiled = set(v for v in range(len(native.diffusion3d_variants())) if native.diffusion3d_variant_compiled(v))
    forms = (False, True) if hz else (False,)
    pl = bench({f"plain v{v}/r{r}" + ("/hz" if f else ""): plain(v, r, f)
                for v in PLAIN if v in compiled for r in ROUNDS for f in forms})
    best_plain = min(pl, key=pl.get)
    print(f"n={n}^3 {a.dtype}: best plain {best_plain} {pl[best_plain]:.4f} ms "
          f"({3 * n ** 3 * eb / pl[best_plain] / 1e6:.0f} GB/s)", flush=True)
    out = {"n": n, "dtype": a.dtype, "placement": placement, "plain": pl, "best_plain": best_plain, "shapes": {}}
    if a.candidates:
        base = [tuple(int(x) for x in c.split("/")) for c in a.candidates.split(",")]
    else:
        base = list(FUSED)
    # IGG_TRANSPORT=put|rccl: that loopback transport (run the script once per
    # kind); auto (the default): update_halo_ chooses between both loopback
    # transports itself on the first exchange of each shape (the library's own
    # default path, parallel/transport_select.py auto_select)
    from igg.utils import config as _cfg

    choice = _cfg.transport_choice()
    uh_forms = ((("put", "auto"),) if choice == "put"
                else ((("auto", "auto"),) if choice == "auto" else (("rccl", "sequential"), ("rccl", "onephase"))))
    for shape in a.shapes.split(","):
        nb = neighbours(shape)
        if a.update_halo:
            # generic update_halo_ of T2 after the plain stencil, through the
            # loopback emulation of exactly these sides (one rank plays both
            # ends of every face: the full pack -> transport -> unpack path)
            from igg.parallel import halo as H
            from igg.parallel.grid import global_grid

            bp = best_plain.split()[1].split("/")
            v0, r0, hz0 = int(bp[0][1:]), int(bp[1][1:]), len(bp) > 2
            sides = [(nb[d][0] >= 0, nb[d][1] >= 0) for d in range(3)]
            uh = {"plain": plain(v0, r0, hz0)}
            for tr, mode in uh_forms:
                def f_uh(tr=tr, mode=mode, k=[0]):
                    src, dst = bufs[k[0] & 1], bufs[(k[0] + 1) & 1]
                    native.diffusion3d(dst.data_ptr(), src.data_ptr(), Cp.data_ptr(), [n, n, n], rd2, 1e-4, eb,
                                       inner, True, v0, s.cuda_stream, r0, hz0)
                    H.update_halo_(dst)
                    k[0] += 1
                uh[f"{tr}/{mode}"] = f_uh
            t_uh = {}
            for tr, mode in uh_forms:
                if mode == "onephase" and any(sd[0] != sd[1] for sd in sides):
                    continue  # one-sided over one self-peer: only the sequential schedule pairs (halo.py)
                H.set_halo_mode("sequential")  # (enable_loopback refuses a one-sided RCCL loopback in one-phase mode)
                global_grid().neighbors[:, :] = -1
                H.enable_loopback(sides)
                H.set_halo_mode(mode)
                r_ = bench({"plain": uh["plain"], f"{tr}/{mode}": uh[f"{tr}/{mode}"]})
                t_uh["plain"] = min(t_uh.get("plain", float("inf")), r_.pop("plain"))
                t_uh.update(r_)
            tpu = t_uh.pop("plain")
            chosen = H.tuned_transports()[-1]["chosen"] if choice == "auto" and H.tuned_transports() else None
            out.setdefault("update_halo", {})[shape] = {"plain_ms": tpu, "ms": t_uh,
                                                       "ratio": {k: v / tpu for k, v in t_uh.items()},
                                                       "auto_chose": chosen}
            print(f"{shape:5s} update_halo_: plain {tpu:.4f} | " +
                  ", ".join(f"{k}={v:.4f} ({v / tpu:.4f}x)" for k, v in t_uh.items()) +
                  (f" [auto chose {chosen}]" if chosen else ""), flush=True)
        if not a.fused:
            continue
        fh = native.FusedHalo(mesh, [n, n, n], eb, nb)
        fh.set_fields(T.data_ptr(), T2.data_ptr())
        cands = list(base)
        if not a.candidates and any(nb[2][s_] >= 0 for s_ in range(2)):
            cands += list(DIRECT) + (list(DIRECT_F32) if eb == 4 else [])
            cands += list(ZUNPACK) + (list(ZUNPACK_F32) if eb == 4 else [])
        if not a.candidates:
            cands += [(v, m | 8, r) for v, m, r in cands]
        has_z = any(nb[2][s_] >= 0 for s_ in range(2))
        # mode bit 2 compiles the z exchange out: only without a z neighbour
        cands = [c for c in cands if native.diffusion3d_fused_variant_ok(c[0]) and not (has_z and c[1] & 2)]
        fns = {f"v{v}/m{m}/r{r}": fused(fh, v, m, r) for v, m, r in cands}
        bp = best_plain.split()[1].split("/")
        fns["plain"] = plain(int(bp[0][1:]), int(bp[1][1:]), len(bp) > 2)
        t = bench(fns)
        if has_z and a.order > 0:
            # z-edge tiles dispatched first (send mode bit 32) at 2..4 residency rounds:
            # longest work first, so more rounds spread the z-edge waves' extra time
            front = sorted((c for c in t if c != "plain"), key=t.get)[:a.order]
            fo = {}
            for c in front:
                v, m, r = (int(x[1:]) for x in c.split("/"))
                for rr in (2, 3, 4):
                    fo[f"v{v}/m{m | 32}/r{rr}"] = fused(fh, v, m | 32, rr)
                    if rr != r:
                        fo[f"v{v}/m{m}/r{rr}"] = fused(fh, v, m, rr)
            fo["plain"] = fns["plain"]
            to = bench(fo)
            t["plain"] = min(t["plain"], to.pop("plain"))
            for k, v_ in to.items():
                t[k] = min(t.get(k, float("inf")), v_)
        if a.inkernel > 0:  # the fastest forms again with the step sync inside the kernel
            front = sorted((c for c in t if c != "plain"), key=t.get)[:a.inkernel]
            fk = {}
            for c in front:
                v, m, r = (int(x[1:]) for x in c.split("/"))
                fk[f"v{v}/m{m | 16}/r{r}"] = fused(fh, v, m | 16, r)
            fk["plain"] = fns["plain"]
            tk = bench(fk)
            t["plain"] = min(t["plain"], tk.pop("plain"))
            t.update(tk)
        tp = t.pop("plain")
        best = min(t, key=t.get)
        ratio = t[best] / tp
        out["shapes"][shape] = {"neighbours": nb, "plain_ms": tp, "fused_ms": t, "best": best, "ratio": ratio}
        top = sorted(t.items(), key=lambda kv: kv[1])[:4]
        print(f"{shape:5s} nb={nb}: plain {tp:.4f} | best fused {best} {t[best]:.4f} -> {ratio:.4f}x | "
              + ", ".join(f"{k}={v:.4f}" for k, v in top[1:]), flush=True)
        mesh.check_error()
        del fh
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)
    igg.finalize_global_grid()
    return 0


if __name__ == "__main__":
    sys.exit(main())
