"""Per-rank checkpoint / restart (utils/checkpoint.py): restart reproduces the
uninterrupted run bitwise; topology and field mismatches are refused."""
import json
import os

import pytest
import torch

import igg
from igg.models.diffusion3d import Diffusion3D
from tests._mp import run_ranks


@pytest.mark.parametrize("nprocs,model", [(1, "diffusion"), (4, "diffusion"), (4, "acoustic")])
def test_restart_matches_uninterrupted_run_cpu(tmp_path, nprocs, model):
    run_ranks(nprocs, "checkpoint", "cpu", model, str(tmp_path))


def test_roundtrip_and_manifest(tmp_path):
    igg.init_global_grid(10, 8, 6, periodz=1, quiet=True, init_MPI=False, device_type="none")
    A = torch.arange(480, dtype=torch.float32).view(10, 8, 6)
    B = torch.ones(3, 4, dtype=torch.complex64)
    prefix = str(tmp_path / "sub" / "c")
    path = igg.save_checkpoint(prefix, step=7, A=A, B=B)
    assert os.path.exists(path) and path.endswith(".rank00000.safetensors")
    meta = json.load(open(prefix + ".json"))
    assert meta["step"] == 7 and meta["nxyz"] == [10, 8, 6] and meta["periods"] == [0, 0, 1]
    meta, f = igg.load_checkpoint(prefix)
    assert torch.equal(f["A"], A) and torch.equal(f["B"], B)
    igg.finalize_global_grid(finalize_MPI=False)


def test_mismatched_grid_is_refused(tmp_path):
    prefix = str(tmp_path / "c")
    igg.init_global_grid(10, 8, 6, quiet=True, init_MPI=False, device_type="none")
    igg.save_checkpoint(prefix, A=torch.zeros(10, 8, 6))
    igg.finalize_global_grid(finalize_MPI=False)
    igg.init_global_grid(12, 8, 6, quiet=True, init_MPI=False, device_type="none")
    with pytest.raises(igg.IGGError, match="nxyz"):
        igg.load_checkpoint(prefix)
    with pytest.raises(igg.IGGError, match="no manifest"):
        igg.load_checkpoint(str(tmp_path / "missing"))
    igg.finalize_global_grid(finalize_MPI=False)


def test_stale_block_from_another_save_is_refused(tmp_path):
    """A block file left from an earlier save (e.g. a rank crashed before
    rewriting it) must not be mixed with a manifest naming a later step."""
    from safetensors.torch import save_file

    prefix = str(tmp_path / "c")
    igg.init_global_grid(10, 8, 6, quiet=True, init_MPI=False, device_type="none")
    A = torch.zeros(10, 8, 6)
    path = igg.save_checkpoint(prefix, step=3, A=A)
    save_file({"A": A}, path, metadata={"coords": "[0, 0, 0]", "step": "2"})  # the stale block
    with pytest.raises(igg.IGGError, match="step 2"):
        igg.load_checkpoint(prefix)
    igg.finalize_global_grid(finalize_MPI=False)


def test_model_restore_checks_shapes(tmp_path):
    prefix = str(tmp_path / "c")
    igg.init_global_grid(10, 8, 6, quiet=True, init_MPI=False, device_type="none")
    m = Diffusion3D(dtype=torch.float64, device="cpu")
    m.run(2)
    m.save(prefix, step=2)
    m32 = Diffusion3D(dtype=torch.float32, device="cpu")
    with pytest.raises(ValueError, match="restore"):
        m32.restore(prefix)
    igg.finalize_global_grid(finalize_MPI=False)


@pytest.mark.gpu
@pytest.mark.parametrize("fused", [False, True])
def test_gpu_restart_diffusion(gpu, tmp_path, fused):
    igg.init_global_grid(20, 18, 32, periodx=1, periody=1, periodz=1, quiet=True, init_MPI=False)
    a, b = Diffusion3D(dtype=torch.float64), Diffusion3D(dtype=torch.float64)
    if fused:
        assert a.set_fused(True) and b.set_fused(True)
    a.run(7)
    a.save(str(tmp_path / "c"), step=7)
    a.run(6)
    assert b.restore(str(tmp_path / "c")) == 7
    b.run(6)
    a.sync_halo()
    b.sync_halo()
    torch.cuda.synchronize()
    assert torch.equal(a.T, b.T)
    a.close()
    b.close()
    igg.finalize_global_grid(finalize_MPI=False)
