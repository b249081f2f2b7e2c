"""Multi-rank tests on CPU (gloo, world sizes 2..8) — the reference suite's
"any number of processes" mode, with an exact per-entry oracle."""
import pytest

from tests._mp import run_ranks


@pytest.mark.parametrize("mode", ["sequential", "onephase"])
@pytest.mark.parametrize("nprocs,cfg", [
    (2, (7, 5, 6, 0, 0, 0)),
    (2, (7, 5, 6, 1, 1, 1)),   # dims 2x1x1 periodic: left == right neighbour
    (4, (7, 5, 6, 1, 0, 1)),
    (8, (7, 5, 6, 0, 0, 0)),   # 2x2x2
    (3, (7, 5, 6, 1, 1, 1)),
    (8, (7, 5, 6, 1, 1, 1)),   # 2x2x2 periodic: every direction is a neighbour
])
def test_halo_cpu_multirank(nprocs, cfg, mode):
    run_ranks(nprocs, "halo", "cpu", *cfg, "f64", env_extra={"IGG_HALO_MODE": mode})


@pytest.mark.parametrize("nprocs,cfg,dims", [
    (2, (7, 1, 1, 1, 0, 0), (0, 1, 1)),   # 1-D
    (4, (7, 5, 1, 1, 1, 0), (0, 0, 1)),   # 2-D 2x2 periodic
    (4, (7, 5, 6, 0, 1, 0), (1, 4, 1)),   # 4 ranks along y
])
def test_halo_cpu_lowdim(nprocs, cfg, dims):
    run_ranks(nprocs, "halo", "cpu", *cfg, "f32", *dims)
    run_ranks(nprocs, "halo", "cpu", *cfg, "f32", *dims, env_extra={"IGG_HALO_MODE": "sequential"})


def test_halo_cpu_complex():
    run_ranks(2, "halo", "cpu", 7, 5, 6, 1, 1, 1, "c128")


@pytest.mark.parametrize("nprocs", [2, 4])
def test_gather_cpu_multirank(nprocs):
    run_ranks(nprocs, "gather", "cpu", "f64")


def test_gather_cpu_int16():
    run_ranks(2, "gather", "cpu", "i16")


@pytest.mark.parametrize("nprocs,overlap", [(2, 0), (8, 0)])
def test_diffusion_cpu_multirank_matches_global(nprocs, overlap):
    run_ranks(nprocs, "diffusion", "cpu", 10, 9, 8, 4, overlap)


def test_ring_cpu():
    run_ranks(3, "ring", "cpu")


# --- order-only matching (the default host matching, IGG_HOST_MATCHING=ordered):
# one tag-0 message per peer and phase, paired with the peer's receives by issue
# position only - RCCL's rule, and MPI's with the reference's all-zero tags
# (update_halo.jl:713-735). A tagged transport would mask an ordering bug
# between two distinct ranks; these runs would not.
@pytest.mark.parametrize("nprocs", [2, 3])
def test_ring_cpu_order_only(nprocs):
    run_ranks(nprocs, "ring", "cpu", env_extra={"IGG_HOST_MATCHING": "ordered"})


@pytest.mark.parametrize("matching", ["ordered", "tagged"])
def test_halo_cpu_matching_forms_agree(matching):
    run_ranks(2, "halo", "cpu", 7, 5, 6, 1, 1, 1, "f64",
              env_extra={"IGG_HOST_MATCHING": matching, "IGG_HALO_MODE": "sequential"})


@pytest.mark.parametrize("scenario,args,mode", [
    ("halo", (7, 5, 6, 1, 1, 1, "f64"), "sequential"),  # dims=2 periodic: both x faces go to ONE peer
    ("halo", (7, 5, 6, 1, 1, 1, "f64"), "onephase"),
    ("ring", (), None),
])
def test_order_only_matching_catches_a_swapped_send_order(scenario, args, mode):
    """The same runs with every peer's sends issued in reverse order
    (IGG_DEBUG_SWAP_SENDS=1) must fail: nothing but the order pairs them."""
    env = {"IGG_HOST_MATCHING": "ordered", "IGG_DEBUG_SWAP_SENDS": "1"}
    if mode:
        env["IGG_HALO_MODE"] = mode
    with pytest.raises(AssertionError):
        run_ranks(2, scenario, "cpu", *args, env_extra=env, timeout=60)


# --- same scenarios with GPU fields, several ranks sharing the one GPU via the
# host-staged transport (exercises the HIP pack/unpack kernels across ranks).
GPU_ENV = {"IGG_TRANSPORT": "staged"}


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["sequential", "onephase"])
@pytest.mark.parametrize("nprocs,cfg", [(2, (7, 5, 6, 1, 1, 1)), (8, (7, 5, 6, 0, 0, 0)), (4, (9, 6, 5, 1, 0, 1))])
def test_halo_gpu_multirank_staged(nprocs, cfg, mode):
    run_ranks(nprocs, "halo", "gpu", *cfg, "f64", env_extra={**GPU_ENV, "IGG_HALO_MODE": mode})


@pytest.mark.gpu
def test_diffusion_gpu_multirank_staged_overlap():
    run_ranks(8, "diffusion", "gpu", 24, 20, 18, 5, 1, env_extra=GPU_ENV)


@pytest.mark.gpu
def test_gather_gpu_multirank_staged():
    run_ranks(4, "gather", "gpu", "f64", env_extra=GPU_ENV)


# --- the one-sided 'put' transport (IPC-mapped arenas + stream flag ops); on
# the one-GPU box every rank maps the same device, which exercises the whole
# protocol (layout agreement, epochs, parity reuse, arena growth) bitwise.
PUT_ENV = {"IGG_TRANSPORT": "put"}


@pytest.mark.gpu
@pytest.mark.parametrize("nprocs,cfg", [(2, (7, 5, 6, 1, 1, 1)), (8, (7, 5, 6, 0, 0, 0)), (4, (9, 6, 5, 1, 0, 1)),
                                        (3, (6, 5, 4, 1, 1, 0))])
def test_halo_gpu_multirank_put(nprocs, cfg):
    run_ranks(nprocs, "halo", "gpu", *cfg, "f64", env_extra=PUT_ENV)


@pytest.mark.gpu
@pytest.mark.parametrize("overlap", [0, 1])
def test_diffusion_gpu_multirank_put(overlap):
    run_ranks(8, "diffusion", "gpu", 24, 20, 18, 7, overlap, env_extra=PUT_ENV)


@pytest.mark.gpu
@pytest.mark.parametrize("queues", ["1", "2", "4"])
def test_diffusion_overlap_graph_two_split_dims(queues):
    """The boundary/interior overlapped step captured in a hipGraph and
    replayed on a 2x2x1 decomposition (the N = 4 shape of a node): round 3's
    SIGSEGV in the replay (profiles/r3_overlap_crash/, root cause in
    profiles/r4_overlap_crash/: one hardware queue per process). Checked
    against the global single-array solution."""
    run_ranks(4, "diffusion", "gpu", 24, 20, 18, 7, 1,
              env_extra={**PUT_ENV, "IGG_TEST_DIMS": "2,2,1", "IGG_TEST_GRAPH": "4", "GPU_MAX_HW_QUEUES": queues},
              timeout=160)


@pytest.mark.gpu
@pytest.mark.parametrize("queues", ["1", "4"])
def test_diffusion_overlap_graph_two_side_streams(queues):
    """The overlapped put step with a CU-masked compute stream forks TWO side
    streams per step: the graph-fork cell that crashes the HIP runtime's
    replay with one hardware queue (profiles/r4_overlap_crash/NOTES.md table:
    2 side streams at GPU_MAX_HW_QUEUES=1 crash, every 4-queue cell replays).
    With 4 queues the forked graph is captured and replayed; with 1 the model
    runs the parts in stream order (models/diffusion3d.py _serial_overlap).
    Checked against the global single-array solution."""
    run_ranks(2, "diffusion", "gpu", 24, 20, 18, 7, 1,
              env_extra={**PUT_ENV, "IGG_TEST_DIMS": "2,1,1", "IGG_TEST_GRAPH": "4", "GPU_MAX_HW_QUEUES": queues,
                         "IGG_TEST_RESERVE_CUS": "8"},
              timeout=160)


@pytest.mark.gpu
@pytest.mark.parametrize("late", [False, True])
def test_rccl_bootstrap_is_bounded_and_collective(late):
    """Two ranks on one GPU: RCCL refuses the duplicate device (an asynchronous
    error of the non-blocking bootstrap); with rank 1 arriving 7 s late, rank
    0's bootstrap times out after IGG_FIRST_CONTACT_TIMEOUT = 3 s and is
    aborted. Either way every rank raises the same error, none hangs."""
    env = {"IGG_FIRST_CONTACT_TIMEOUT": "3"}
    if late:
        env["IGG_INJECT_HANG"] = "rccl_init@1:7"
    run_ranks(2, "rccl_init_bounded", 40 if late else 30, env_extra=env, timeout=120)


@pytest.mark.gpu
def test_put_transport_timeout_reports_and_never_hangs():
    run_ranks(2, "put_timeout", env_extra={**PUT_ENV, "IGG_PUT_TIMEOUT": "2"}, timeout=120)


@pytest.mark.gpu
def test_put_transport_arena_regrowth():
    """Receive arenas that grow several times (collective re-export of IPC
    memory) keep every exchange exact on 4 ranks."""
    run_ranks(4, "put_regrow", env_extra={"IGG_TRANSPORT": "staged", "IGG_PUT_TIMEOUT": "20",
                                          "IGG_PUT_ARENA_FLOOR_MB": "1", "GPU_MAX_HW_QUEUES": "1"}, timeout=150)


@pytest.mark.gpu
def test_put_transport_absorbs_rank_skew():
    run_ranks(4, "put_skew", 12, env_extra=PUT_ENV, timeout=170)


@pytest.mark.gpu
@pytest.mark.parametrize("nprocs", [2, 4])
def test_gather_async_gpu(nprocs):
    run_ranks(nprocs, "gather_async", env_extra=PUT_ENV)


@pytest.mark.gpu
@pytest.mark.parametrize("nprocs", [pytest.param(2, marks=pytest.mark.slow), 4])
def test_gather_pull_staged_chunks_gpu(nprocs):
    """Blocks too large to export whole (above 2 GiB on the real runtime,
    above 100 / 400 bytes here) are staged in chunks of whole x-planes and
    pulled chunk by chunk: gather_async_ (ordering, reuse) and gather_."""
    run_ranks(nprocs, "gather_async", env_extra=dict(PUT_ENV, IGG_GATHER_CHUNK_BYTES="400"))
    run_ranks(nprocs, "gather", "gpu", "f64", env_extra=dict(PUT_ENV, IGG_GATHER_CHUNK_BYTES="100"))


@pytest.mark.gpu
def test_gather_pull_chunk_regrowth_gpu():
    """Staged chunks of MiB size (dedicated allocations) that grow between
    gathers are retired, not freed: every gathered block stays right."""
    run_ranks(3, "gather_regrow", env_extra=dict(PUT_ENV, IGG_GATHER_CHUNK_BYTES=str(1 << 20)), timeout=160)


@pytest.mark.gpu
@pytest.mark.parametrize("inject,expect", [("gather_export@1", "could not export"),
                                           ("gather_open@0", "could not map or pull")])
def test_gather_pull_failure_is_collective_gpu(inject, expect):
    """A rank whose export fails (or a root whose mapping fails) does not leave
    the others blocked in the gather's collective: every rank raises."""
    run_ranks(3, "gather_fail", expect, env_extra=dict(PUT_ENV, IGG_INJECT_FAIL=inject), timeout=120)


@pytest.mark.parametrize("dev", ["cpu", pytest.param("gpu", marks=pytest.mark.gpu)])
def test_select_transport(dev):
    """igg.select_transport: every candidate checked bitwise against the
    host-staged exchange, the fastest checked one kept (GPU ranks sharing a
    device: 'put'; RCCL skipped); a CPU grid has nothing to choose."""
    run_ranks(2, "select_transport", dev, timeout=150)


@pytest.mark.gpu
@pytest.mark.parametrize("inject,expect", [("", "put"), ("peer_map@1", "staged")])
def test_auto_transport_shared_gpu(inject, expect):
    """IGG_TRANSPORT=auto (default) on ranks sharing one GPU: the first
    exchange per field set checks put against the host-staged exchange (RCCL
    refuses shared devices: skipped) and keeps it; with put's peer mapping
    failing on one rank, every rank falls back to the staged transport
    together. Halos bitwise exact in both."""
    env = {"IGG_TRANSPORT": "auto", "IGG_PUT_TIMEOUT": "20"}
    if inject:
        env["IGG_INJECT_FAIL"] = inject
    run_ranks(2, "auto_transport", "gpu", expect, env_extra=env, timeout=150)


# --- fused halo exchange (stencil kernel stores into the neighbours' arenas)
SLOW = pytest.mark.slow  # redundant cases: IGG_TEST_SLOW=1 (conftest.py)


@pytest.mark.gpu
@pytest.mark.parametrize("nprocs,cfg,kernel", [(2, (24, 20, 64, 6, 0, 0), ("0", "0")),
                                               (4, (20, 22, 32, 5, 1, 1), ("9", "1")),
                                               pytest.param(8, (18, 20, 40, 7, 0, 0), ("0", "1"), marks=SLOW),
                                               pytest.param(8, (16, 18, 24, 6, 1, 1), ("50", "0"), marks=SLOW),
                                               # per-side wave classes of variant 40 and the edge-lane z
                                               # form of 42 (n2 > 64*VZ+VZ) on one-sided (non-periodic) ranks
                                               (4, (20, 22, 136, 5, 0, 0), ("40", "0")),
                                               (8, (18, 20, 136, 5, 0, 1), ("42", "0")),
                                               # direct z (mode bit 4): z faces into the neighbours' T2
                                               pytest.param(2, (24, 20, 64, 6, 1, 0), ("40", "4"), marks=SLOW),
                                               (8, (18, 20, 136, 5, 0, 1), ("42", "4")),
                                               pytest.param(8, (16, 18, 24, 6, 1, 1), ("0", "5"), marks=SLOW),
                                               # peeled x planes (mode bit 8) with remote x neighbours
                                               (2, (40, 66, 136, 6, 1, 0), ("42", "12")),
                                               (8, (34, 66, 136, 5, 1, 1), ("40", "8")),
                                               # z-edge tiles first (mode bit 32) on one-sided corner ranks
                                               (8, (34, 66, 136, 5, 0, 0), ("42", "44")),
                                               # tiling 9 with 2 grid rounds on 2x2x2 corner ranks (the
                                               # corner's best form, the bench's first candidate)
                                               (8, (18, 20, 136, 5, 0, 0), ("9", "8", "2")),
                                               # z unpack (mode bit 64) on 2x2x2 corner ranks and periodic
                                               (8, (18, 20, 136, 5, 0, 0), ("9", "72")),
                                               (8, (16, 18, 24, 6, 1, 1), ("42", "73")),
                                               (2, (24, 20, 64, 6, 0, 1), ("0", "64"))])
def test_diffusion_gpu_multirank_fused(nprocs, cfg, kernel):
    # ranks share one GPU on the test box: RCCL cannot, so sync_halo uses 'put'
    env = {**PUT_ENV, "IGG_PUT_TIMEOUT": "20", "IGG_TEST_VARIANT": kernel[0], "IGG_TEST_FUSED_MODE": kernel[1]}
    if len(kernel) > 2:
        env["IGG_TEST_FUSED_ROUNDS"] = kernel[2]
    if nprocs > 2:
        env["GPU_MAX_HW_QUEUES"] = "1"  # ranks share one GPU: no queue oversubscription (profiles/r2_reh8/)
    run_ranks(nprocs, "diffusion_fused", *cfg, env_extra=env, timeout=170)


@pytest.mark.gpu
@pytest.mark.parametrize("nprocs,cfg,kernel", [(2, (24, 20, 64, 6, 1, 0), ("0", "0")),
                                               (4, (20, 22, 32, 5, 1, 1), ("0", "1")),
                                               (8, (18, 20, 40, 7, 1, 0), ("0", "5")),
                                               # z unpack: the unpack kernel waits for the z senders itself
                                               (8, (18, 20, 136, 5, 0, 0), ("0", "72")),
                                               (2, (24, 20, 64, 6, 0, 1), ("0", "64"))])
def test_diffusion_gpu_multirank_fused_in_kernel_sync(nprocs, cfg, kernel):
    """The step synchronisation inside the fused kernel across processes
    (forced: ranks sharing one GPU default to the sync kernel, because waiting
    waves could hold the compute units another rank's kernel needs; tiling 0
    leaves room). Bitwise vs stencil + update_halo_."""
    env = {**PUT_ENV, "IGG_PUT_TIMEOUT": "20", "IGG_TEST_VARIANT": kernel[0], "IGG_TEST_FUSED_MODE": kernel[1],
           "IGG_FUSED_SYNC_KERNEL": "0"}
    if nprocs > 2:
        env["GPU_MAX_HW_QUEUES"] = "1"
    run_ranks(nprocs, "diffusion_fused", *cfg, env_extra=env, timeout=170)


@pytest.mark.gpu
@pytest.mark.parametrize("nprocs,kernel", [pytest.param(4, ("0", "0"), marks=pytest.mark.slow), (8, ("0", "1")),
                                            pytest.param(8, ("40", "4"), marks=pytest.mark.slow)])
def test_fused_soak_with_rank_skew(nprocs, kernel):
    """Thousands of graph-replayed fused steps with random host skew between
    ranks stay bitwise equal to stencil + update_halo_."""
    env = {**PUT_ENV, "IGG_PUT_TIMEOUT": "30", "IGG_TEST_VARIANT": kernel[0], "IGG_TEST_FUSED_MODE": kernel[1]}
    if nprocs > 2:
        # N processes x 4 hardware queues on ONE device are time-sliced by the
        # command processor (8 ranks: 95 s per soak, GPU_MAX_HW_QUEUES=1: a
        # few s; profiles/r2_reh8/); one rank per GPU never shares queues
        env["GPU_MAX_HW_QUEUES"] = "1"
    rounds = 30 if nprocs > 4 else 60
    run_ranks(nprocs, "fused_soak", 20, 18, 32, rounds, 40, env_extra=env, timeout=170)


# --- failure path and comm_cart interop ------------------------------------
def test_barrier_timeout_raises_instead_of_hanging():
    run_ranks(2, "barrier_timeout", env_extra={"IGG_COMM_TIMEOUT": "3"}, timeout=60)


@pytest.mark.parametrize("nprocs", [2, 4])
def test_tensor_collectives_cpu(nprocs):
    run_ranks(nprocs, "collectives", "cpu")


def test_suite_chains_scenarios_cpu():
    """The multigpu tier's chained suite (several scenarios per launch, the
    grid re-initialised on one process group) works; CPU/gloo ranks here."""
    outs = run_ranks(2, "suite", "halo:cpu:7:5:6:1:1:1:f64", "gather:cpu:f64", "ring:cpu",
                     "collectives:cpu", "diffusion:cpu:24:20:18:3:0|IGG_HALO_MODE=sequential", timeout=120)
    for o in outs:
        assert "suite OK (5 items" in o, o[-2000:]


@pytest.mark.gpu
def test_suite_chains_scenarios_shared_gpu():
    """The multigpu tier's suite mechanism on GPU ranks sharing device 0 (put
    transport; RCCL refuses ranks on one device): direct-z soak, fused forms,
    halo oracle, pull gather, gather_async in one launch."""
    dev = "IGG_TEST_DEV=gpu;IGG_TRANSPORT=put;IGG_PUT_TIMEOUT=20"
    outs = run_ranks(2, "suite",
                     f"fused_soak:20:18:32:10:20|{dev};IGG_TEST_VARIANT=40;IGG_TEST_FUSED_MODE=4",
                     f"diffusion_fused:24:20:64:6:1:0|{dev};IGG_TEST_VARIANT=42;IGG_TEST_FUSED_MODE=12",
                     f"halo:gpu:7:5:6:1:1:1:f64|{dev}",
                     f"gather:gpu:f64|{dev}",
                     f"gather_async|{dev}", timeout=160, env_extra={"GPU_MAX_HW_QUEUES": "1"})
    for o in outs:
        assert "suite OK (5 items" in o, o[-2000:]
