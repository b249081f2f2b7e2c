"""Field placement probe of Diffusion3D (models/diffusion3d.py _placed_fields):
the same T/Cp/T2 carve sweeps at one of two speeds depending on where the
allocator put it (profiles/r6_placement/), so the model times a few candidate
allocations and keeps the fastest."""
import gc
import weakref

import pytest
import torch

import igg
from igg.models import diffusion3d as D


class _Grid:
    nprocs = 1
    comm = None


def test_placed_fields_keeps_the_fastest_and_frees_the_rest(monkeypatch):
    made = []

    def carve():
        c = [torch.zeros(4), torch.ones(4), torch.zeros(4)]
        made.append([weakref.ref(t) for t in c])
        return c

    monkeypatch.setattr(D, "_placement_count", lambda gg, meta, device: 3)
    monkeypatch.setattr(D, "_time_placements", lambda cands, dtype: [0.61, 0.58, 0.60])
    fields, rec = D._placed_fields(carve, _Grid(), torch.empty(4, device="meta"), torch.device("cpu"))
    gc.collect()
    assert rec == {"candidates": 3, "ms": [0.61, 0.58, 0.6], "chosen": 1}
    assert all(r() is not None for r in made[1])
    assert all(r() is None for k in (0, 2) for r in made[k])
    assert fields[0] is made[1][0]()


def test_placement_count_off_cases(monkeypatch):
    big = torch.empty((1024, 1024, 64), dtype=torch.float64, device="meta")  # 512 MiB
    small = torch.empty((64, 64, 64), dtype=torch.float64, device="meta")
    monkeypatch.delenv("IGG_FIELD_PLACEMENT", raising=False)
    assert D._placement_count(_Grid(), big, torch.device("cpu")) == 1  # host fields
    assert D._placement_count(_Grid(), small, torch.device("cuda", 0)) == 1  # below PLACEMENT_MIN_BYTES
    monkeypatch.setenv("IGG_FIELD_PLACEMENT", "1")
    assert D._placement_count(_Grid(), big, torch.device("cuda", 0)) == 1  # switched off


def test_cpu_model_has_no_placement_record():
    igg.init_global_grid(8, 8, 8, quiet=True, init_MPI=False, device_type="none")
    try:
        m = D.Diffusion3D()
        assert m.placement is None
    finally:
        igg.finalize_global_grid(finalize_MPI=False)


@pytest.mark.gpu
def test_placement_probe_on_the_headline_size(monkeypatch):
    """512^3 f64 (the bench's shape): four candidate carves timed, the fastest
    kept; the chosen fields hold the initial conditions (the probe's scribbles
    are overwritten) and step bitwise like a model without the probe."""
    monkeypatch.delenv("IGG_FIELD_PLACEMENT", raising=False)
    igg.init_global_grid(512, 512, 512, quiet=True, init_MPI=False)
    try:
        m = D.Diffusion3D(variant=43)
        rec = m.placement
        assert rec is not None and rec["candidates"] == D.PLACEMENT_CANDIDATES, rec
        assert rec["ms"][rec["chosen"]] == min(rec["ms"])
        print(f"placement: {rec}")
        monkeypatch.setenv("IGG_FIELD_PLACEMENT", "1")
        ref = D.Diffusion3D(variant=43)
        assert ref.placement is None
        assert torch.equal(m.T, ref.T) and torch.equal(m.Cp, ref.Cp) and torch.equal(m.T2, ref.T2)
        m.run(6)
        ref.run(6)
        torch.cuda.synchronize()
        assert torch.equal(m.T, ref.T)
    finally:
        igg.finalize_global_grid(finalize_MPI=False)
