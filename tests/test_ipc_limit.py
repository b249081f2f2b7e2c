"""The IPC size limit (csrc/include/igg/ipc.hpp IPC_MAX_BYTES): on this ROCm
runtime hipIpcOpenMemHandle of an allocation above 2 GiB never returns
(profiles/r3_ipc/), so the framework refuses to export one and keeps every
allocation a peer maps below the limit."""
import pytest
import torch

from igg.models.diffusion3d import _carve


def test_carve_splits_at_the_limit():
    ts = [torch.full((4, 5, 6), float(k)) for k in range(3)]
    one = _carve(ts, gap=64, kind=None)
    assert len({t.untyped_storage().data_ptr() for t in one}) == 1  # one buffer
    split = _carve(ts, gap=64, kind=None, split_at=3 * 4 * 5 * 6 * 4)
    assert len({t.untyped_storage().data_ptr() for t in split}) == 3  # one per array
    for k, (a, b) in enumerate(zip(one, split)):
        assert torch.equal(a, ts[k]) and torch.equal(b, ts[k])
    big_enough = _carve(ts, gap=64, kind=None, split_at=1 << 30)
    assert len({t.untyped_storage().data_ptr() for t in big_enough}) == 1


@pytest.mark.gpu
def test_ipc_export_refuses_allocations_of_2_gib(gpu):
    from torch.utils import dlpack

    from igg._native import IGGError, native

    limit = int(native.IPC_MAX_BYTES)
    assert limit == 1 << 31
    small = dlpack.from_dlpack(native.alloc_dlpack(64 << 20, 1))
    assert native.alloc_bytes(small.data_ptr()) >= 64 << 20
    assert len(native.ipc_get_handle(small.data_ptr())) > 0
    big = dlpack.from_dlpack(native.alloc_dlpack(limit, 0))
    assert native.alloc_bytes(big.data_ptr() + 4096) >= limit
    with pytest.raises(IGGError, match="2 GiB"):
        native.ipc_get_handle(big.data_ptr())
    del big, small
    torch.cuda.synchronize()
