"""Field placement probe (utils/placement.py): the same carve of fields sweeps
at one of two speeds depending on where the allocator put it
(profiles/r6_placement/), so the models time a few candidate allocations and
keep the fastest."""
import gc
import weakref

import pytest
import torch

import igg
from igg.models import diffusion3d as D
from igg.utils import placement as PL


class _Grid:
    nprocs = 1
    comm = None


def test_placed_keeps_the_fastest_and_frees_the_rest():
    made = []

    def carve():
        c = [torch.zeros(4), torch.ones(4), torch.zeros(4)]
        made.append([weakref.ref(t) for t in c])
        return c

    fields, rec = PL.placed(carve, 3, lambda cands: [0.61, 0.58, 0.60])
    gc.collect()
    assert rec == {"candidates": 3, "batches": 1, "ms": [0.61, 0.58, 0.6], "chosen": 1}
    assert all(r() is not None for r in made[1])
    assert all(r() is None for k in (0, 2) for r in made[k])
    assert fields[0] is made[1][0]()
    one, rec1 = PL.placed(carve, 1, lambda cands: pytest.fail("no probe with one candidate"))
    assert rec1 is None and len(made) == 4


def test_placed_escalates_while_all_candidates_are_alike():
    """All of a batch within SPREAD: another batch, timed with the best so far;
    a batch with two speeds ends the search."""
    calls = []
    speeds = iter([0.62, 0.621, 0.622, 0.6215, 0.62, 0.619, 0.595, 0.62, 0.621])

    def timer(cands):
        calls.append(len(cands))
        return [c[0] for c in cands]

    def carve():
        return [next(speeds)]

    fields, rec = PL.placed(carve, (3, 10), lambda cands: timer(cands))
    assert calls == [3, 4, 4]  # batch 1; the best + batch 2; the best + batch 3 (0.595: two speeds)
    assert fields == [0.595] and rec["candidates"] == 9 and rec["batches"] == 3
    speeds2 = iter([0.62] * 5)
    f2, rec2 = PL.placed(lambda: [next(speeds2)], (2, 5), lambda cands: [c[0] for c in cands])
    assert rec2["candidates"] == 5 and rec2["batches"] == 3  # stopped at the limit


def test_candidate_count_off_cases(monkeypatch):
    big, small = 512 << 20, 2 << 20
    monkeypatch.delenv("IGG_FIELD_PLACEMENT", raising=False)
    assert PL.candidate_count(_Grid(), big, 3 * big, torch.device("cpu")) == (1, 1)  # host fields
    assert PL.candidate_count(_Grid(), small, 3 * small, torch.device("cuda", 0)) == (1, 1)  # below MIN_FIELD_BYTES
    monkeypatch.setenv("IGG_FIELD_PLACEMENT", "1")
    assert PL.candidate_count(_Grid(), big, 3 * big, torch.device("cuda", 0)) == (1, 1)  # switched off


class _Comm:
    def __init__(self, devs):
        self.devs = devs

    def all_gather_object(self, obj):
        return self.devs


def test_candidate_count_is_off_when_ranks_share_a_gpu(monkeypatch):
    """Multi-rank: a shared device turns the probe off on every rank (the probes
    would time each other); distinct devices keep it, sized by free memory."""
    monkeypatch.delenv("IGG_FIELD_PLACEMENT", raising=False)
    monkeypatch.setattr(torch.cuda, "current_device", lambda: 0)
    monkeypatch.setattr(torch.cuda, "mem_get_info", lambda device=None: (288 << 30, 288 << 30))
    g = _Grid()
    g.nprocs = 2
    import socket

    host = socket.gethostname()
    g.comm = _Comm([(host, 0), (host, 0)])
    big = 1 << 30
    assert PL.candidate_count(g, big, 3 * big, torch.device("cuda", 0)) == (1, 1)
    g.comm = _Comm([(host, 0), (host, 1)])
    assert PL.candidate_count(g, big, 3 * big, torch.device("cuda", 0)) == (PL.CANDIDATES, PL.MAX_CANDIDATES)
    g.comm = _Comm([(host, 0), (host, 1)])
    assert PL.candidate_count(g, 4 * big, 12 * big, torch.device("cuda", 0)) == (PL.CANDIDATES, 18)  # 216 / 12 GiB
    monkeypatch.setenv("IGG_FIELD_PLACEMENT", "5")
    assert PL.candidate_count(g, big, 3 * big, torch.device("cuda", 0)) == (5, 5)  # an explicit count: no escalation


def test_cpu_model_has_no_placement_record():
    igg.init_global_grid(8, 8, 8, quiet=True, init_MPI=False, device_type="none")
    try:
        m = D.Diffusion3D()
        assert m.placement is None
    finally:
        igg.finalize_global_grid(finalize_MPI=False)


@pytest.mark.gpu
def test_placement_probe_diffusion_headline_size(monkeypatch):
    """512^3 f64 (the bench's shape): CANDIDATES carves timed, the fastest
    kept; the chosen fields hold the initial conditions (the probe's scribbles
    are overwritten) and step bitwise like a model without the probe."""
    monkeypatch.delenv("IGG_FIELD_PLACEMENT", raising=False)
    igg.init_global_grid(512, 512, 512, quiet=True, init_MPI=False)
    try:
        m = D.Diffusion3D(variant=43)
        rec = m.placement
        assert rec is not None and rec["candidates"] >= PL.CANDIDATES, rec
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


@pytest.mark.gpu
def test_placement_probe_acoustic(monkeypatch):
    """8192^2 f32 acoustic: the probe steps the candidates with the model's own
    kernel; the chosen carve is reset to the initial state and steps bitwise
    like a model without the probe."""
    from igg.models.acoustic2d import Acoustic2D

    monkeypatch.delenv("IGG_FIELD_PLACEMENT", raising=False)
    igg.init_global_grid(8192, 8192, 1, quiet=True, init_MPI=False)
    try:
        m = Acoustic2D()
        rec = m.placement
        assert rec is not None and rec["candidates"] >= PL.CANDIDATES, rec
        assert rec["ms"][rec["chosen"]] == min(rec["ms"])
        print(f"placement: {rec}")
        monkeypatch.setenv("IGG_FIELD_PLACEMENT", "1")
        ref = Acoustic2D()
        assert ref.placement is None
        for a, b in ((m.P, ref.P), (m.Vx, ref.Vx), (m.Vy, ref.Vy), (m.P2, ref.P2), (m.Vx2, ref.Vx2), (m.Vy2, ref.Vy2)):
            assert torch.equal(a, b)
        m.run(6)
        ref.run(6)
        torch.cuda.synchronize()
        assert torch.equal(m.P, ref.P) and torch.equal(m.Vx, ref.Vx) and torch.equal(m.Vy, ref.Vy)
    finally:
        igg.finalize_global_grid(finalize_MPI=False)
