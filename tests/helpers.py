"""Shared test helpers: the coordinate-encoding oracle of the reference suite
(test/test_update_halo.jl:748-1053)."""
import torch

import igg


def encode(A: torch.Tensor, dx=1.0, dy=1.0, dz=1.0, complex_factor=None) -> torch.Tensor:
    """Fill A with z_g*1e2 + y_g*1e1 + x_g (only the dims A has)."""
    nd = A.dim()
    kw = dict(dtype=torch.float64, device="cpu")
    v = igg.coords_g(0, dx, A, **kw).view([-1] + [1] * (nd - 1))
    if nd >= 2:
        v = v + igg.coords_g(1, dy, A, **kw).view([1, -1] + [1] * (nd - 2)) * 1e1
    if nd >= 3:
        v = v + igg.coords_g(2, dz, A, **kw).view(1, 1, -1) * 1e2
    v = v.expand(A.shape)
    if complex_factor is not None:
        v = v.to(torch.complex128) * complex_factor
    A.copy_(v.to(A.dtype).to(A.device))
    return A


def zero_boundaries(A: torch.Tensor) -> torch.Tensor:
    for d in range(A.dim()):
        idx = [slice(None)] * A.dim()
        idx[d] = [0, A.shape[d] - 1]
        A[tuple(idx)] = 0
    return A
