"""Port of test/test_select_device.jl."""
import pytest
import torch

import igg
from igg import IGGError


def test_select_device_without_gpu_errors():
    igg.init_global_grid(4, 4, 4, quiet=True, init_MPI=False, device_type="CUDA")  # no CUDA backend here
    with pytest.raises(IGGError, match="Cannot select a device"):
        igg.select_device()
    igg.finalize_global_grid(finalize_MPI=False)


@pytest.mark.gpu
def test_select_device_returns_valid_id():
    igg.init_global_grid(4, 4, 4, quiet=True, init_MPI=False, device_type="AMDGPU")
    dev = igg.select_device()
    assert 0 <= dev < torch.cuda.device_count()
    assert torch.cuda.current_device() == dev
    assert igg.native.get_device() == dev
    igg.finalize_global_grid(finalize_MPI=False)
