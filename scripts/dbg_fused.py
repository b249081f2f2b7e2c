"""Locate mismatches of the fused diffusion step vs stencil + update_halo_."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import igg
from igg.models.diffusion3d import Diffusion3D

n = tuple(int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (34, 29, 136)))
v = int(sys.argv[4]) if len(sys.argv) > 4 else 0
mode = int(sys.argv[5]) if len(sys.argv) > 5 else 0
igg.init_global_grid(*n, periodx=1, periody=1, periodz=1, quiet=True)
a = Diffusion3D(dtype=torch.float64, variant=v)
b = Diffusion3D(dtype=torch.float64, variant=v)
b.fused_variant, b.fused_mode = v, mode
assert b.set_fused(True)
for k in range(3):
    a.step()
    b.step()
    torch.cuda.synchronize()
    I = (slice(1, -1),) * 3
    d = (a.T[I] != b.T[I])
    idx = d.nonzero() + 1
    print(f"step {k}: {int(d.sum())} interior mismatches of {d.numel()}")
    if len(idx):
        for ax, nm in enumerate("xyz"):
            vals, cnt = torch.unique(idx[:, ax], return_counts=True)
            print(f"  {nm}: " + " ".join(f"{int(q)}:{int(c)}" for q, c in list(zip(vals.tolist(), cnt.tolist()))[:20]))
        break
igg.finalize_global_grid()
