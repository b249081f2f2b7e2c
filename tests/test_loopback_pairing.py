"""Plans of the one-sided loopback emulation (halo.enable_loopback with
(low, high) sides: a node's edge/corner rank on one GPU) checked on the CPU:
one process plays every neighbour through ONE self-peer, so a transport
pairs the k-th receive with the k-th send. The sequential schedule pairs
messages of equal size for every shape; the one-phase schedule does not on
one-sided shapes (its receives are issued by receiver-side direction), which
over RCCL read past a send buffer and faulted the GPU in round 5 - hence the
guard in parallel/halo.py. Host fields and a host loopback transport here:
the same copy/message plans the device path launches."""
import ctypes

import numpy as np
import pytest
import torch

import igg
from igg._native import native
from igg.parallel import halo as H
from igg.parallel.grid import global_grid


def _loop(log):
    def f(recvs, sends, device, stream):
        assert not device
        log.append([(rn, sn) for (_rp, rn, _a, _b), (_sp, sn, _c, _d) in zip(recvs, sends)] +
                   ([("count", len(recvs), len(sends))] if len(recvs) != len(sends) else []))
        for (rp, rn, _a, _b), (sp, sn, _c, _d) in zip(recvs, sends):
            n = min(rn, sn)
            ctypes.memmove(rp, sp, n)
    return f


def _setup(shape, n=12):
    igg.init_global_grid(n, n - 1, n + 2, periodx=1, periody=1, periodz=1, quiet=True, init_MPI=False,
                         device_type="none")
    gg = global_grid()
    dims = shape.rstrip("+-")
    side = shape[len(dims):] or "+-"
    sides = [(d in dims and "-" in side, d in dims and "+" in side) for d in "xyz"]
    gg.neighbors[:, :] = -1
    for d in range(3):
        for s in range(2):
            if sides[d][s]:
                gg.neighbors[s, d] = 0
    peers = [0 if all(c == 1 or sides[d][c // 2] for d, c in enumerate((k // 9, (k // 3) % 3, k % 3))) else -1
             for k in range(27)]
    peers[13] = 1
    H._engine.set_grid(native.GridInfo(1, 2, gg.nxyz.tolist(), gg.overlaps.tolist(), gg.neighbors.tolist(),
                                       peers))
    log = []
    H._engine.set_transport(native.PyTransport(_loop(log), True, False, "loop"), False)
    H._plans.clear()
    H._sig_modes.clear()
    return log


def _pairs_ok(log):
    return all(all(p[0] == p[1] for p in phase if p[0] != "count") and not any(p[0] == "count" for p in phase)
               for phase in log)


@pytest.mark.parametrize("shape", ["x+", "x-", "xy+", "xy-", "xyz+", "xyz-", "xyz"])
def test_sequential_pairs_equal_sizes(shape):
    log = _setup(shape)
    try:
        H.set_halo_mode("sequential")
        for shp in [(12, 11, 14), (13, 11, 14), (12, 11, 15)]:
            A = torch.arange(float(np.prod(shp)), dtype=torch.float64).view(shp)
            H.update_halo_(A)
        assert log and _pairs_ok(log), log
    finally:
        igg.finalize_global_grid(finalize_MPI=False)


def test_onephase_one_sided_mispairs_and_is_refused_over_rccl():
    log = _setup("xy+")
    try:
        H.set_halo_mode("onephase")
        A = torch.zeros((12, 11, 14), dtype=torch.float64)
        H.update_halo_(A)
        assert not _pairs_ok(log)  # the hazard the guard exists for
        # the guard: a one-sided RCCL loopback refuses the one-phase mode
        H._loopback_one_sided = True

        class _R:
            name = "rccl"

        H._loopback_comm = H._loopback_comms["rccl"] = _R()
        with pytest.raises(igg.IGGError, match="one-sided"):
            H.set_halo_mode("onephase")
    finally:
        H._loopback_one_sided = False
        H._loopback_comm = None
        H._loopback_comms.clear()
        igg.finalize_global_grid(finalize_MPI=False)
