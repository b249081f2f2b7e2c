"""HIP virtual memory management export of allocations of 2 GiB and more
(csrc/vmm.cpp). hipIpcOpenMemHandle of such an allocation
never returns on this runtime (csrc/include/igg/ipc.hpp IPC_MAX_BYTES); the VMM
route - hipMemCreate, a POSIX file descriptor passed over a Unix socket,
hipMemImportFromShareableHandle + map - is checked here across two processes
sharing a GPU (the multigpu tier maps across devices)."""
import pytest

from tests._mp import ROOT, run_ranks


@pytest.mark.gpu
@pytest.mark.parametrize("source", ["vmm", "malloc"])
def test_vmm_maps_a_3gib_allocation_across_processes(source):
    """source "malloc": a torch (hipMalloc) tensor exported as a dma-buf of its
    allocation range and imported the VMM way."""
    outs = run_ranks(2, "vmm_map", "gpu", 3 << 30, source, env_extra={"IGG_FIRST_CONTACT_TIMEOUT": "60"},
                     timeout=150)
    line = [ln for ln in outs[0].splitlines() if "vmm map of" in ln]
    assert line, outs[0][-2000:]
    print(line[0])


def test_fd_passing_between_processes():
    """The descriptor hand-over itself (no GPU): a pipe's read end passed over
    the abstract Unix socket reads what the owner wrote."""
    import os
    import subprocess
    import sys
    import uuid

    from igg._native import native

    name = f"igg-fdtest-{uuid.uuid4().hex}"
    lis = native.fd_listen(name)
    r, w = os.pipe()
    os.write(w, b"halo")
    os.close(w)
    code = ("import sys, os; sys.path.insert(0, %r); from igg._native import native; "
            "fd = native.fd_fetch(%r, 20.0); print(os.read(fd, 4).decode())") % (ROOT, name)
    child = subprocess.Popen([sys.executable, "-c", code], stdout=subprocess.PIPE, text=True)
    native.fd_serve(lis, r, 1, 20.0)
    out, _ = child.communicate(timeout=60)
    native.fd_close(lis)
    os.close(r)
    assert child.returncode == 0 and out.strip() == "halo", out


@pytest.mark.gpu
def test_gather_pulls_vmm_blocks_and_stages_large_snapshots_in_one_buffer():
    """gather_ maps blocks in VMM memory in place at any size and stages a
    large snapshot (1.1 GiB per rank here) into one VMM buffer instead of IPC
    chunks; three ranks sharing a GPU, every block checked."""
    run_ranks(3, "gather_vmm", 1100, env_extra={"IGG_FIRST_CONTACT_TIMEOUT": "60", "IGG_GATHER_VMM": "1"},
              timeout=170)


@pytest.mark.gpu
@pytest.mark.parametrize("dmabuf", ["1", "0"])
def test_gather_pulls_large_ordinary_blocks(dmabuf):
    """gather_ of torch blocks of 2.1 GiB per rank (above the IPC limit): as a
    dma-buf of the allocation, in place (default), or staged into IPC chunks
    (IGG_GATHER_DMABUF=0); the same array again with new values, then a new
    allocation after the old one was freed; every block checked."""
    outs = run_ranks(2, "gather_dmabuf", 2200, env_extra={"IGG_FIRST_CONTACT_TIMEOUT": "60",
                                                          "IGG_GATHER_DMABUF": dmabuf}, timeout=170)
    line = [ln for ln in outs[0].splitlines() if "gather dmabuf" in ln]
    print(line[0] if line else outs[0][-500:])
