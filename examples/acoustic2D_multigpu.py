#!/usr/bin/env python3
"""2-D acoustic waves on a staggered grid, multiple MI355X GPUs (2-D topology).

Pressure at cell centres, velocities on faces (Vx: nx+1 by ny, Vy: nx by ny+1):
update_halo_(Vx, Vy) exchanges fields with different halo overlaps in one call.
Optional in-situ visualisation of P via gather_ every --vis-every steps.

    torchrun --standalone --local-addr 127.0.0.1 --nproc-per-node 4 \\
        examples/acoustic2D_multigpu.py --nx 1024 --nt 2000 --vis-every 200
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import igg  # noqa: E402
from igg.models.acoustic2d import Acoustic2D  # noqa: E402
from igg.utils.vis import Animation  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nx", type=int, default=1024)
    ap.add_argument("--nt", type=int, default=2000)
    ap.add_argument("--vis-every", type=int, default=0)
    ap.add_argument("--out", default="acoustic2D.gif")
    ap.add_argument("--dtype", default="float32", choices=["float64", "float32"])
    ap.add_argument("--cpu", action="store_true")
    a = ap.parse_args()
    import torch

    nx = a.nx
    me, dims, nprocs, coords, comm = igg.init_global_grid(nx, nx, 1, device_type="none" if a.cpu else "auto")
    model = Acoustic2D(dtype=getattr(torch, a.dtype), device="cpu" if a.cpu else None)
    P_v = None
    if a.vis_every and me == 0:
        P_v = torch.zeros(nx * int(dims[0]), nx * int(dims[1]), dtype=model.P.dtype, device=model.P.device)
    anim = Animation()
    igg.tic()
    for it in range(a.nt):
        if a.vis_every and it % a.vis_every == 0:
            igg.gather_(model.P, P_v)
            if me == 0:
                anim.frame(P_v.T.float(), vmin=-0.1, vmax=0.1)
        model.step()
    t = igg.toc()
    if me == 0:
        t_it = t / a.nt
        print(f"{nprocs} process(es) {dims.tolist()}: {t_it * 1e3:.4f} ms/step, "
              f"T_eff = {model.a_eff_bytes / t_it / 1e9:.1f} GB/s per process")
        if a.vis_every:
            anim.save_gif(a.out)
            print(f"wrote {a.out}")
    igg.finalize_global_grid()


if __name__ == "__main__":
    main()
