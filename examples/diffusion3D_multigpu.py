#!/usr/bin/env python3
"""3-D heat diffusion on multiple MI355X GPUs with in-situ visualisation.

Counterpart of the reference's examples/diffusion3D_multigpu_CuArrays.jl: every
``--vis-every`` steps the halo-free interior of T is gathered on rank 0
(gather_, device to device: on one node the root's copy engines pull every
block over IPC straight into its place, parallel/gather.py; RCCL receives +
HIP reorder kernel across nodes or with IGG_GATHER_PULL=0) and a y-mid slice is appended to an animated GIF (utils/vis.py). Pass
``--cpu`` for the multicpu variant (examples/diffusion3D_multicpu.jl).

    torchrun --standalone --local-addr 127.0.0.1 --nproc-per-node 8 \\
        examples/diffusion3D_multigpu.py --nx 128 --nt 2000 --vis-every 100
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import igg  # noqa: E402
from igg.models.diffusion3d import Diffusion3D  # noqa: E402
from igg.utils.vis import Animation  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nx", type=int, default=128)
    ap.add_argument("--nt", type=int, default=2000)
    ap.add_argument("--vis-every", type=int, default=100)
    ap.add_argument("--out", default="diffusion3D.gif")
    ap.add_argument("--cpu", action="store_true")
    a = ap.parse_args()
    import torch

    nx = a.nx
    me, dims, nprocs, coords, comm = igg.init_global_grid(nx, nx, nx, device_type="none" if a.cpu else "auto")
    model = Diffusion3D(dtype=torch.float64, device="cpu" if a.cpu else None)
    dev = model.T.device
    nx_v, ny_v, nz_v = ((nx - 2) * int(d) for d in dims)
    T_v = torch.zeros(nx_v, ny_v, nz_v, dtype=torch.float64, device=dev) if me == 0 else None
    anim = Animation()
    for it in range(a.nt):
        if it % a.vis_every == 0:
            T_nohalo = model.T[1:-1, 1:-1, 1:-1].contiguous()   # remove the halo
            igg.gather_(T_nohalo, T_v)                          # gather on process 0
            if me == 0:
                anim.frame(T_v[:, ny_v // 2, :].T, scale=max(1, 256 // nx_v))
        model.step()
    if me == 0:
        anim.save_gif(a.out, fps=15)
        print(f"wrote {a.out} ({len(anim.frames)} frames of the {nx_v}x{ny_v}x{nz_v} gathered interior)")
    igg.finalize_global_grid()


if __name__ == "__main__":
    main()
