"""Fused halo exchange of the diffusion model (csrc/include/igg/fused.hpp).

The stencil kernel stores its send planes into the neighbours' arenas and reads
its own face halos from its arena; results must equal stencil + update_halo_
bitwise (the reference's step, examples/diffusion3D_multigpu_CuArrays_novis.jl:
42-47). Single process here: periodic grids (every neighbour is this rank) and
the loopback emulation; multi-rank runs are in test_multiprocess.py.
"""
import pytest
import torch

import igg
from igg.models.diffusion3d import Diffusion3D
from igg.ops import stencil as _stencil

FUSED = _stencil.compiled_fused_variants()  # 2, 11, 41, 45 only in a --probes build


def test_fused_unavailable_on_cpu():
    igg.init_global_grid(12, 10, 16, periodx=1, quiet=True, init_MPI=False, device_type="none")
    m = Diffusion3D(dtype=torch.float64, device="cpu")
    assert not m.can_fuse
    assert m.set_fused(True) is False
    m.run(2)
    igg.finalize_global_grid(finalize_MPI=False)


@pytest.mark.gpu
def test_fused_unavailable_without_neighbours(gpu):
    igg.init_global_grid(12, 10, 16, quiet=True, init_MPI=False)
    m = Diffusion3D(dtype=torch.float64)
    assert not m.can_fuse and m.set_fused(True) is False
    igg.finalize_global_grid(finalize_MPI=False)


def _pair(n, periods, dtype, variant, loopback=False, mode=0):
    from igg.parallel import halo as H

    igg.init_global_grid(*n, periodx=periods[0], periody=periods[1], periodz=periods[2], quiet=True,
                         init_MPI=False)
    if loopback:
        H.enable_loopback()
    from igg.ops import stencil

    # fused ids reuse the plain index space; fused-only / measurement-only ids
    # (e.g. 50: a tiling 0 form) run the plain step with variant 0
    plain = variant if variant in stencil.compiled_variants() else 0
    a = Diffusion3D(dtype=dtype, variant=plain)
    b = Diffusion3D(dtype=dtype, variant=plain)
    b.fused_variant, b.fused_mode = variant, mode
    assert b.set_fused(True)
    assert b.fused_variant == variant, f"fused variant {variant} is not compiled in this build"
    return a, b


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("variant", FUSED)
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_fused_periodic_matches_update_halo(gpu, variant, dtype, mode):
    a, b = _pair((34, 29, 136), (1, 1, 1), dtype, variant, mode=mode)
    a.run(9)
    b.run(9)
    b.sync_halo()
    torch.cuda.synchronize()
    b.check()
    assert torch.equal(a.T, b.T)
    igg.finalize_global_grid(finalize_MPI=False)


@pytest.mark.gpu
@pytest.mark.parametrize("periods", [(1, 0, 0), (0, 1, 0), (0, 0, 1), (1, 1, 0), (0, 1, 1)])
def test_fused_partial_periodic(gpu, periods):
    """Only some sides have a neighbour; the others keep their boundary values."""
    a, b = _pair((21, 19, 64), periods, torch.float64, 40, mode=int(sum(periods) == 1))
    a.run(6)
    b.run(6)
    b.sync_halo()
    torch.cuda.synchronize()
    assert torch.equal(a.T, b.T)
    igg.finalize_global_grid(finalize_MPI=False)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [2, 3])
@pytest.mark.parametrize("variant", FUSED)
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("periods", [(1, 1, 0), (1, 1, 1)])
def test_fused_no_z_exchange_matches_update_halo(gpu, variant, dtype, mode, periods):
    """Modes 2/3: with x/y neighbours only (a 2x2x1 rank) the kernel form without
    the z-edge exchange (FEAT 195 in fused_kernels.hip) runs, for every tiling,
    send mode and dtype; with a z neighbour they fall back to the full form."""
    a, b = _pair((34, 29, 136), periods, dtype, variant, mode=mode)
    a.run(7)
    b.run(7)
    b.sync_halo()
    torch.cuda.synchronize()
    b.check()
    assert torch.equal(a.T, b.T)
    igg.finalize_global_grid(finalize_MPI=False)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [4, 5])
@pytest.mark.parametrize("variant", FUSED)
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("periods", [(1, 1, 1), (0, 0, 1), (1, 0, 1)])
def test_fused_direct_z_matches_update_halo(gpu, variant, dtype, mode, periods):
    """Modes 4/5 (direct z): the z faces are stored into the halo column of the
    neighbour's next field (here: this rank's own, periodic) and no z receive
    code runs; same results as update_halo_, halos included after sync_halo."""
    a, b = _pair((34, 29, 136), periods, dtype, variant, mode=mode)
    assert b.fused_mode == mode
    a.run(9)
    b.run(9)
    b.sync_halo()
    torch.cuda.synchronize()
    b.check()
    assert torch.equal(a.T, b.T)
    igg.finalize_global_grid(finalize_MPI=False)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [8, 9, 12, 13, 40, 44, 45])  # + 32: z-edge tiles dispatched first
@pytest.mark.parametrize("variant", [0, 14, 40, 42, 44])
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("periods", [(1, 1, 1), (1, 0, 1)])
def test_fused_peel_matches_update_halo(gpu, variant, dtype, mode, periods):
    """Mode bit 8 (peel): x-chunk waves sweep x = 1 / n0-2 with the x exchange
    and the planes between without it (multi-plane chunks on this grid, so
    first, middle and last parts all run); same results as update_halo_."""
    a, b = _pair((48, 130, 264), periods, dtype, variant, mode=mode)
    assert b.fused_mode == mode
    a.run(7)
    b.run(7)
    b.sync_halo()
    torch.cuda.synchronize()
    b.check()
    assert torch.equal(a.T, b.T)
    igg.finalize_global_grid(finalize_MPI=False)


@pytest.mark.gpu
def test_fused_direct_z_graph(gpu):
    """Direct z under hipGraph replays (both buffer parities captured) and the
    loopback emulation's remote path."""
    a, b = _pair((40, 36, 72), (1, 1, 1), torch.float64, 42, loopback=True, mode=4)
    a.run(3)
    b.run(3)
    b.capture(steps=4)
    a.run(11)
    b.run(11)
    b.sync_halo()
    torch.cuda.synchronize()
    b.check()
    assert torch.equal(a.T, b.T)
    igg.finalize_global_grid(finalize_MPI=False)


@pytest.mark.gpu
def test_fused_loopback_graph_and_mode_switches(gpu):
    """Loopback grid, hipGraph replays with odd/even step counts, sync_halo in
    between (re-primes from the field) and switching back to update_halo_."""
    a, b = _pair((40, 36, 72), (1, 1, 1), torch.float64, 9, loopback=True, mode=1)
    a.run(3)
    b.run(3)
    b.capture(steps=4)  # counter odd: the graph bakes in that parity
    a.run(8)
    b.run(8)
    b.sync_halo()
    torch.cuda.synchronize()
    assert torch.equal(a.T, b.T)
    a.run(5)
    b.run(5)  # unprimed after sync_halo: an eager step first, then replays
    b.set_fused(False)
    a.run(2)
    b.run(2)
    torch.cuda.synchronize()
    assert torch.equal(a.T, b.T)
    assert b.set_fused(True)
    a.run(4)
    b.run(4)
    b.sync_halo()
    torch.cuda.synchronize()
    b.check()
    assert torch.equal(a.T, b.T)
    igg.finalize_global_grid(finalize_MPI=False)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1, 8, 64, 72, 16, 88])
@pytest.mark.parametrize("n2", [320, 512])
@pytest.mark.parametrize("periods", [(1, 1, 1), (1, 0, 1), (0, 0, 1)])
def test_fused_dpp_z_matches_update_halo(gpu, mode, n2, periods):
    """Fused variant 48 (tiling 9, z-edge lane moves as DPP row shifts,
    ZDPP): n2 = 320 / 512 put the high edge's rows inside the edge lane's
    16-lane row (zh = 15 / 63), so the DPP form runs; bitwise equal to
    stencil + update_halo_ in every send form (incl. z unpack and the
    in-kernel step sync)."""
    a, b = _pair((20, 26, n2), periods, torch.float64, 48, mode=mode)
    a.run(7)
    b.run(7)
    b.sync_halo()
    torch.cuda.synchronize()
    b.check()
    assert torch.equal(a.T, b.T)
    igg.finalize_global_grid(finalize_MPI=False)


@pytest.mark.gpu
@pytest.mark.parametrize("graph", [False, True])
def test_fused_receive_form_switch_reprimes(gpu, graph):
    """Switching the send mode's receive form mid-run (arena z 8 -> z unpack
    72 -> direct z 12 -> in-kernel sync 88 -> 8) re-primes from the field: a
    primed z-unpack step would otherwise read a z halo column no unpack wrote
    (ADVICE r5). Bitwise against stencil + update_halo_ after every switch,
    eager and with a capture after each switch."""
    a, b = _pair((40, 36, 72), (1, 1, 1), torch.float64, 9, mode=8)
    a.run(3)
    b.run(3)
    for mode in (72, 12, 88, 8):
        b.fused_mode = mode
        if graph:
            k0 = b._fstep
            b.capture(steps=2)  # re-primes with one eager step of the new form
            a.run(b._fstep - k0 - 2)  # (recording the 2 captured steps advanced the counter too)
        a.run(5)
        b.run(5)
        b.sync_halo()
        torch.cuda.synchronize()
        b.check()
        assert torch.equal(a.T, b.T), mode
    igg.finalize_global_grid(finalize_MPI=False)


@pytest.mark.gpu
def test_fused_arena_layout(gpu):
    """Region offsets are 256 B aligned and the z-face pitch covers n1-2 rows."""
    a, b = _pair((20, 37, 64), (1, 1, 1), torch.float64, 0)
    fh = b._fh
    assert fh.zpitch >= 35 and fh.zpitch % 16 == 0
    for d in range(3):
        for s in range(2):
            assert (fh.region_offset(d, s) * 8) % 256 == 0
    ins, outs, zp, zr = fh.io(0, False)
    assert all(p == 0 for pair in ins for p in pair)  # unprimed: halos from the field
    ins, outs, zp, zr = fh.io(1, True)
    assert all(p != 0 for pair in ins for p in pair) and all(p != 0 for pair in outs for p in pair)
    assert fh.n_peers == 1
    # direct z: the z sends target the halo columns of the buffer matching t2
    assert fh.has_fields
    n1, n2, eb = 37, 64, 8
    for t2 in (b.T2, b.T):
        ins, outs, zp, zr = fh.io(1, True, t2.data_ptr(), True)
        assert ins[2] == (0, 0) and ins[0][0] != 0
        assert zp == n1 * n2 and zr == n2
        assert outs[2][0] == t2.data_ptr() + (n2 - 1 + n2) * eb  # self-periodic: my own next field
        assert outs[2][1] == t2.data_ptr() + n2 * eb
    with pytest.raises(Exception, match="registered"):
        fh.io(1, True, b.Cp.data_ptr(), True)
    igg.finalize_global_grid(finalize_MPI=False)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [(4, 4, 8), (5, 40, 8), (9, 4, 132)])
def test_fused_tiny_extents(gpu, n):
    """Tiny extents: the two send planes are neighbours (n=4), a wave holds
    both y send rows, a single z tile / wave holds both z edges."""
    for mode in (0, 1):
        a, b = _pair(n, (1, 1, 1), torch.float64, 0, mode=mode)
        a.run(5)
        b.run(5)
        b.sync_halo()
        torch.cuda.synchronize()
        assert torch.equal(a.T, b.T), (n, mode)
        igg.finalize_global_grid(finalize_MPI=False)


@pytest.mark.gpu
def test_fused_default_graph_steps(gpu):
    """Default capture (GRAPH_STEPS per replay) with step counts that are not
    multiples of it, fused and plain."""
    from igg.models.diffusion3d import GRAPH_STEPS

    a, b = _pair((24, 22, 64), (1, 1, 1), torch.float64, 0)
    c = Diffusion3D(dtype=torch.float64, variant=0)
    a.run(2 * GRAPH_STEPS + 7)
    b.capture()
    c.capture()
    assert b.graph_steps == GRAPH_STEPS and c.graph_steps == GRAPH_STEPS
    b.run(2 * GRAPH_STEPS + 6)  # capture() ran one (priming) step
    c.run(2 * GRAPH_STEPS + 6)
    b.sync_halo()
    torch.cuda.synchronize()
    assert torch.equal(a.T, b.T) and torch.equal(a.T, c.T)
    igg.finalize_global_grid(finalize_MPI=False)


@pytest.mark.gpu
def test_graph_after_odd_step_counts(gpu):
    """run() after odd step counts (the graph reads the capture's T first),
    plain and fused, and after a restore-like write with mark_modified."""
    a, b = _pair((24, 22, 64), (1, 1, 1), torch.float64, 0)
    c = Diffusion3D(dtype=torch.float64, variant=0)
    b.capture(steps=4)  # one priming step each
    c.capture(steps=4)
    a.run(1)
    for k in (5, 3, 8, 7):
        for m in (a, b, c):
            m.run(k)
    b.sync_halo()
    torch.cuda.synchronize()
    assert torch.equal(a.T, b.T) and torch.equal(a.T, c.T)
    for m in (b, c):
        m.T.copy_(a.T)
        m.T2.copy_(a.T2)
        m.mark_modified()
    for m in (a, b, c):
        m.run(9)
    b.sync_halo()
    torch.cuda.synchronize()
    b.check()
    assert torch.equal(a.T, b.T) and torch.equal(a.T, c.T)
    igg.finalize_global_grid(finalize_MPI=False)


@pytest.mark.gpu
@pytest.mark.parametrize("variant,mode", [(0, 0), (0, 1), (40, 8), (42, 4), (42, 12), (50, 1), (40, 72)])
@pytest.mark.parametrize("periods", [(1, 1, 1), (0, 1, 0), (1, 0, 1)])
def test_in_kernel_step_sync_counts_every_step(gpu, variant, mode, periods):
    """The in-kernel step synchronisation advances EPOCH exactly once per step
    and leaves COUNT at 0: the host's count of exchanging waves equals the
    neighbour). Eager steps and graph replays. The in-kernel form is send mode
    bit 16 (the default is the sync kernel after the stencil)."""
    a, b = _pair((26, 37, 136), periods, torch.float64, variant, mode=mode | 16)
    assert not b._fh.in_kernel_sync  # default send modes: the sync kernel
    assert b._fh.in_kernel_sync_for(b.fused_mode)
    e0 = b._fh.flag(0)
    b.run(3)
    torch.cuda.synchronize()
    # + the entry barrier and run()'s exit barrier (drain)
    assert b._fh.flag(0) == e0 + 5 and b._fh.flag(2) == 0
    b.capture(steps=4)
    b.run(9)
    b.sync_halo()
    a.run(12)
    torch.cuda.synchronize()
    b.check()
    assert b._fh.flag(0) == e0 + 5 + 9 + 1 and b._fh.flag(2) == 0
    assert torch.equal(a.T, b.T)
    igg.finalize_global_grid(finalize_MPI=False)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [64, 72, 73])  # z unpack (+ 8 peel, + 1 deferred sends)
@pytest.mark.parametrize("variant", [0, 9, 40, 42, 44])
@pytest.mark.parametrize("periods", [(1, 1, 1), (1, 0, 1), (0, 0, 1)])
def test_fused_z_unpack_matches_update_halo(gpu, variant, mode, periods):
    """Send mode bit 64 (z unpack): the z faces go into the neighbours' arenas
    (coalesced), the sweep has no z receive code and reads the z halo from the
    field, which a copy kernel fills after the step synchronisation; bitwise
    the same as stencil + update_halo_ (halos included after sync_halo)."""
    a, b = _pair((34, 29, 136), periods, torch.float64, variant, mode=mode)
    assert b.fused_mode == mode
    a.run(9)
    b.run(9)
    b.sync_halo()
    torch.cuda.synchronize()
    b.check()
    assert torch.equal(a.T, b.T)
    igg.finalize_global_grid(finalize_MPI=False)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [80, 88])  # z unpack + in-kernel step sync (+ 8 peel)
@pytest.mark.parametrize("variant", [0, 9, 40, 42])
@pytest.mark.parametrize("periods", [(1, 1, 1), (0, 0, 1)])
def test_fused_z_unpack_in_kernel_sync_matches_update_halo(gpu, variant, mode, periods):
    """z unpack with the step synchronisation inside the fused kernel: no sync
    kernel runs, the unpack kernel waits for the z senders' ARRIVED flags
    itself (CopyWait); eager steps and graph replays, bitwise."""
    a, b = _pair((34, 29, 136), periods, torch.float64, variant, mode=mode)
    assert b._fh.in_kernel_sync_for(b.fused_mode)
    a.run(3)
    b.run(3)
    b.capture(steps=4)
    a.run(8)
    b.run(8)
    b.sync_halo()
    torch.cuda.synchronize()
    b.check()
    assert torch.equal(a.T, b.T)
    igg.finalize_global_grid(finalize_MPI=False)


@pytest.mark.gpu
@pytest.mark.parametrize("variant,mode", [(44, 72), (14, 64), (42, 73)])
def test_fused_z_unpack_f32_graph_loopback(gpu, variant, mode):
    """z unpack in f32, under hipGraph replays with odd step counts and through
    the loopback emulation's remote path."""
    a, b = _pair((40, 36, 264), (1, 1, 1), torch.float32, variant, loopback=True, mode=mode)
    a.run(3)
    b.run(3)
    b.capture(steps=4)
    a.run(11)
    b.run(11)
    b.sync_halo()
    torch.cuda.synchronize()
    b.check()
    assert torch.equal(a.T, b.T)
    igg.finalize_global_grid(finalize_MPI=False)


@pytest.mark.gpu
def test_fused_z_unpack_rejects_direct_z(gpu):
    a, b = _pair((24, 22, 64), (1, 1, 1), torch.float64, 0, mode=64 | 4)
    with pytest.raises(Exception, match="exclusive"):
        b.step()
    igg.finalize_global_grid(finalize_MPI=False)
