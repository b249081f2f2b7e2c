"""HIP streams with CU masks (MI355X-specific resource partitioning).

``cu_partition(reserved)`` returns two torch ExternalStreams: a compute stream
that excludes ``reserved`` CUs and a (high-priority-by-placement) halo stream
that may only use those CUs. Communication kernels (RCCL's p2p kernels keep all
their workgroups spinning on each other) then never wait behind a compute
kernel that occupies every CU, at the price of the reserved CUs for compute.
Reserved CUs are spread evenly over the mask (every k-th bit) so each XCD
keeps the same share.
"""
from __future__ import annotations

import torch

from .._native import native

_owned: list[int] = []


def _mask_words(bits: list[bool]) -> list[int]:
    words = [0] * ((len(bits) + 31) // 32)
    for i, b in enumerate(bits):
        if b:
            words[i // 32] |= 1 << (i % 32)
    return words


def cu_partition(reserved: int):
    """(compute_stream, halo_stream) with ``reserved`` CUs for the halo stream."""
    n = native.cu_count()
    reserved = max(1, min(reserved, n - 1))
    step = n / reserved
    halo = [False] * n
    for k in range(reserved):
        halo[int(k * step)] = True
    comp = [not b for b in halo]
    hc = native.stream_create_cu_mask(_mask_words(comp), 0)
    hh = native.stream_create_cu_mask(_mask_words(halo), 0)
    _owned.extend([hc, hh])
    dev = torch.cuda.current_device()
    return (torch.cuda.ExternalStream(hc, device=dev), torch.cuda.ExternalStream(hh, device=dev))


def release_streams() -> None:
    torch.cuda.synchronize()
    while _owned:
        native.stream_destroy(_owned.pop())
