"""Cross-XCD / cross-process coherence of the one-sided exchanges with WARM
reader caches (docs/COHERENCE.md fact 4).

The fused and put exchanges rely on a receiver never reading a stale cached
copy of an arena line that a peer rewrote. In the bench the arena halves are
re-read only after a 3 GiB step has streamed through the L2s, so the bitwise
checks there would rarely see a stale line even if one were possible. Here
the reader's arena is small (64 KiB - 4 MiB), read into every XCD's L2 right
before the writer (a second process on the same GPU, through its IPC
mapping) stores new values with the production ``sc0 sc1`` stores; after the
production synchronisation the reader reads every word from every XCD
(csrc/kernels/coherence_kernels.hip). Both synchronisation forms: the sync
kernels (put_sync_kernel) and the in-kernel step sync (step_sync_enter_wg /
step_sync_exit_wg). The multigpu tier runs the same scenario with the writer
on another GPU (tests/test_multigpu.py).
"""
import pytest

from tests._mp import run_ranks


@pytest.mark.gpu
@pytest.mark.parametrize("form", ["kernel", "inkernel"])
@pytest.mark.parametrize("nbytes,rounds", [(64 << 10, 100), (4 << 20, 30)])
def test_warm_cache_coherence_shared_gpu(form, nbytes, rounds):
    outs = run_ranks(2, "coherence", "gpu", form, nbytes, rounds,
                     env_extra={"IGG_PUT_TIMEOUT": "20"}, timeout=150)
    assert any("stale reads 0" in o for o in outs), outs[0][-2000:]


@pytest.mark.gpu
@pytest.mark.parametrize("l2", [0, 1])
def test_warm_cache_control_without_acquire(l2):
    """The same warm reader re-reading inside one kernel after a relaxed flag
    poll, with no acquire (l2: skipping the L1): records how many stale words
    the caches return without the production synchronisation (the test's
    sensitivity; profiles/r6_coherence/NOTES.md). Only the run is asserted:
    the count is hardware behaviour, not a property of this code."""
    outs = run_ranks(2, "coherence_control", "gpu", 16 << 10, 20, l2, env_extra={"IGG_PUT_TIMEOUT": "20"},
                     timeout=150)
    line = [ln for ln in outs[0].splitlines() if "coherence control" in ln and "stale reads" in ln]
    assert line, outs[0][-2000:]
    print(line[0])


@pytest.mark.gpu
def test_plain_store_writer_control():
    """Positive control: a writer with plain (write-back) stores instead of
    st_sys, same synchronisation. Records how many stale words the reader
    then gets (profiles/r6_coherence/NOTES.md) - the writer-side hazard that
    the production system-scope stores exist for."""
    outs = run_ranks(2, "coherence", "gpu", "kernel", 4 << 20, 20, 1, env_extra={"IGG_PUT_TIMEOUT": "20"},
                     timeout=150)
    line = [ln for ln in outs[0].splitlines() if "PLAIN-STORE WRITER" in ln]
    assert line, outs[0][-2000:]
    print(line[0])
