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


def expected_after_halo(ref: torch.Tensor, fields_dim_has_halo, neighbors) -> torch.Tensor:
    """Exact oracle of update_halo after zeroing every boundary plane.

    An entry keeps its reference value iff, for every dim in which it lies on a
    boundary plane (index 0 or n-1), the field has a halo in that dim and a
    neighbour exists on that side; otherwise it stays 0 (x->y->z sequential
    exchange carries corners only through existing neighbours).
    ``fields_dim_has_halo[d]``: ol(d,A) >= 2; ``neighbors[s][d]``: rank or -1.
    """
    keep = torch.ones(ref.shape, dtype=torch.bool)
    for d in range(ref.dim()):
        n = ref.shape[d]
        for side, idx in ((0, 0), (1, n - 1)):
            ok = fields_dim_has_halo[d] and neighbors[side][d] != -1
            if not ok:
                sl = [slice(None)] * ref.dim()
                sl[d] = idx
                keep[tuple(sl)] = False
    out = torch.zeros_like(ref)
    out[keep] = ref[keep]
    return out


def has_halo(A, gg) -> list:
    return [int(gg.overlaps[d]) + (A.shape[d] if A.dim() > d else 1) - int(gg.nxyz[d]) >= 2 for d in range(3)]
