#!/usr/bin/env python3
"""Back-to-back launches of the fused step (stencil + sync) and of the plain
stencil for several (variant, grid rounds), for kernel-trace gap analysis
(scripts/prof_gap.sh). Also rehearses the Diffusion3D model's own step."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

import igg  # noqa: E402
from igg._native import native  # noqa: E402

n = 512
igg.init_global_grid(n, n, n, periodx=1, periody=1, periodz=1, quiet=True)
if "--rccl" in sys.argv:  # a live 1-rank RCCL communicator (as in the loopback bench)
    comm = native.RcclComm(native.RcclComm.unique_id(), 1, 0)
if "--loopback" in sys.argv:
    from igg.parallel import halo as H

    H.enable_loopback()
T = torch.rand(n, n, n, dtype=torch.float64, device="cuda")
T2, Cp = T.clone(), T.clone() + 1
s = torch.cuda.current_stream().cuda_stream
mesh = native.PeerMesh(0, 1, lambda b: [bytes(b)])
fh = native.FusedHalo(mesh, [n, n, n], 8, [[0, -1], [0, -1], [0, -1]])
inner = [([1, 1, 1], [n - 1, n - 1, n - 1])]
k = 0
for v, r in ((0, 1), (0, 3), (14, 3)):
    for _ in range(6):
        fh.step(T2.data_ptr(), T.data_ptr(), Cp.data_ptr(), [1.0] * 3, 1e-4, v, k, True, s, r, 0)
        k += 1
    torch.cuda.synchronize()
    for _ in range(6):
        native.diffusion3d(T2.data_ptr(), T.data_ptr(), Cp.data_ptr(), [n] * 3, [1.0] * 3, 1e-4, 8, inner, True, v, s, r)
    torch.cuda.synchronize()
# the model (carved allocation), eager fused steps
from igg.models.diffusion3d import Diffusion3D  # noqa: E402

m = Diffusion3D(dtype=torch.float64, variant=0)
m.fused_variant, m.fused_rounds = 0, 3
m.set_fused(True)
for _ in range(6):
    m.step()
torch.cuda.synchronize()
print("done")
igg.finalize_global_grid()
