#!/usr/bin/env python3
"""Single-GPU study of the multi-GPU time step (halo exchange + overlap).

Loopback mode (igg.parallel.halo.enable_loopback) sends every face through the
real remote path (pack -> RCCL group -> unpack) to this same GPU, i.e. the
workload of an interior rank with 6 neighbours. Measured (CUDA-event timing,
median of interleaved rounds):
  plain      : stencil only, no neighbours (the 1-GPU bench step)
  halo_only  : update_halo_ of T in loopback mode (3 dims, 6 faces)
  serial     : stencil (whole interior) then update_halo_ (no overlap)
  overlap    : slabs + halo on the high-priority stream || interior
Efficiency proxy E = plain / overlap.
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import igg  # noqa: E402
from igg.models.diffusion3d import Diffusion3D  # noqa: E402
from igg.parallel import halo as H  # noqa: E402


def timeit(fn, reps, stream):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--dtype", default="float64")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--loopback-dims", default="111", help="dims with loopback neighbours, e.g. 110 = x,y only")
    ap.add_argument("--combos", default="0:11:0:0,0:11:0:8,0:11:0:16,0:11:0:32,0:0:0:16",
                    help="interior_rounds:halo_variant:halo_rounds:reserved_cus list")
    a = ap.parse_args()
    dtype = getattr(torch, a.dtype)
    n = a.n
    s = torch.cuda.current_stream()
    igg.init_global_grid(n, n, n, quiet=True)
    m = Diffusion3D(dtype=dtype)
    plain = [timeit(m.step, a.reps, s) for _ in range(a.rounds)]
    del m
    torch.cuda.empty_cache()
    H.enable_loopback(tuple(c == "1" for c in a.loopback_dims))
    ms = Diffusion3D(dtype=dtype, overlap=False)
    combos = [tuple(int(x) for x in c.split(":")) for c in a.combos.split(",")]
    models = {}
    for c in combos:
        if c[3] not in models:
            models[c[3]] = Diffusion3D(dtype=dtype, overlap=True, reserve_cus=c[3])
            models[c[3]].Cp = ms.Cp  # share inputs (memory)
            models[c[3]].T, models[c[3]].T2 = ms.T.clone(), ms.T.clone()
    mo = models[combos[0][3]]
    res = {"plain": plain, "halo_only": [], "serial": []}
    for c in combos:
        res[f"overlap_ir{c[0]}_hv{c[1]}_hr{c[2]}_cu{c[3]}"] = []
        res[f"slabs_hv{c[1]}_hr{c[2]}"] = []

    def slabs():
        from igg.ops import stencil as st
        st.diffusion3d_(mo.T2, mo.T, mo.Cp, boxes=mo.slabs, **mo._kw(mo.halo_variant, mo.halo_rounds))

    for _ in range(a.rounds):
        res["halo_only"].append(timeit(lambda: igg.update_halo_(mo.T), a.reps, s))
        res["serial"].append(timeit(ms.step, a.reps, s))
        for c in combos:
            mo = models[c[3]]
            mo.interior_rounds, mo.halo_variant, mo.halo_rounds = c[:3]
            res[f"slabs_hv{c[1]}_hr{c[2]}"].append(timeit(slabs, a.reps, s))
            res[f"overlap_ir{c[0]}_hv{c[1]}_hr{c[2]}_cu{c[3]}"].append(timeit(mo.step, a.reps, s))
    out = {k: round(statistics.median(v), 4) for k, v in res.items()}
    best = min((k for k in out if k.startswith("overlap")), key=lambda k: out[k])
    out["best_overlap"] = best
    out["E_proxy_best_overlap"] = round(out["plain"] / out[best], 4)
    out["E_proxy_serial"] = round(out["plain"] / out["serial"], 4)
    out["faces"] = H.halo_plan_summary(mo.T)
    print(json.dumps({"n": n, "dtype": a.dtype, "ms": out}), flush=True)
    # correctness: loopback overlap == loopback serial after a few steps
    for mm in (mo, ms):
        mm.T.copy_(ms.Cp * 0 + torch.arange(n, device=mm.T.device, dtype=dtype).view(1, 1, -1))
        mm.T2.copy_(mm.T)
    for _ in range(3):
        mo.step()
        ms.step()
    torch.cuda.synchronize()
    print(json.dumps({"overlap_equals_serial": bool(torch.equal(mo.T, ms.T))}), flush=True)
    igg.finalize_global_grid()


if __name__ == "__main__":
    main()
