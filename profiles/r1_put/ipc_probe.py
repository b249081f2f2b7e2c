#!/usr/bin/env python3
"""Feasibility probe of the put-transport primitives with 2 processes on one GPU.

For each memory kind of the flag block (0 default, 1 fine-grained, 2 signal,
3 uncached) and of the data arena (0, 3): IPC export/import, a pack-kernel put
into the peer's arena, hipStreamWriteValue64 to the peer's flag,
hipStreamWaitValue64 on the own flag, verification, and the ping-pong latency
of CP flag signalling. Every wait is bounded on the host (stream query with a
deadline; a stuck wait is released by writing the flag from another stream).

Usage: python profiles/r1_put/ipc_probe.py            (launches 2 ranks itself)
"""
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def launch():
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r), LOCAL_WORLD_SIZE="2",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), IGG_PROBE_CHILD="1",
                   IGG_TRANSPORT="staged")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)], env=env))
    rc = 0
    for p in procs:
        try:
            rc |= p.wait(timeout=240)
        except subprocess.TimeoutExpired:
            p.kill()
            rc = 1
    sys.exit(rc)


def child():
    import torch

    import igg
    from igg._native import native

    me, dims, nprocs, coords, comm = igg.init_global_grid(8, 8, 8, quiet=True, select_device=False,
                                                         device_type="AMDGPU")
    peer = 1 - me
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(device=dev)
    rel = torch.cuda.Stream(device=dev)
    log = lambda *a: print(f"[rank {me}]", *a, flush=True)  # noqa: E731
    log("can_stream_wait_value", native.can_stream_wait_value())

    def bounded_sync(stream, flag, what, deadline=10.0):
        t0 = time.time()
        while not stream.query():
            if time.time() - t0 > deadline:
                log(f"TIMEOUT waiting for {what}; releasing")
                native.stream_write_u64(rel.cuda_stream, flag, 1 << 62)
                rel.synchronize()
                stream.synchronize()
                return False
            time.sleep(1e-4)
        return True

    nbytes = 1 << 20
    src = (torch.arange(nbytes // 8, dtype=torch.float64, device=dev) + 1000 * me)
    for kf in (0, 1, 2, 3):
        for ka in (0, 3):
            tag = f"flags={kf} arena={ka}"
            try:
                flags = native.ipc_malloc(4096, kf)
                arena = native.ipc_malloc(nbytes, ka)
                h = (native.ipc_get_handle(flags), native.ipc_get_handle(arena))
                ok_local = True
            except Exception as e:  # noqa: BLE001
                log(tag, "alloc/export failed:", e)
                h, ok_local = None, False
            hs = comm.all_gather_object(h)
            if not ok_local or hs[peer] is None:
                comm.barrier()
                continue
            try:
                pf, pa = native.ipc_open(hs[peer][0]), native.ipc_open(hs[peer][1])
            except Exception as e:  # noqa: BLE001
                log(tag, "open failed:", e)
                comm.barrier()
                continue
            torch.cuda.synchronize()
            comm.barrier()
            # put my pattern into the peer's arena, then raise the peer's flag[0]
            native.copy2d([(src.data_ptr(), pa, 1, nbytes // 8, nbytes // 8, 1, nbytes // 8, 1)], 8, True,
                          s.cuda_stream)
            native.stream_write_u64(s.cuda_stream, pf, 1)
            native.stream_wait_u64_geq(s.cuda_stream, flags, 1)
            got = torch.empty(nbytes // 8, dtype=torch.float64, device=dev)
            native.copy2d([(arena, got.data_ptr(), 1, nbytes // 8, nbytes // 8, 1, nbytes // 8, 1)], 8, True,
                          s.cuda_stream)
            ok = bounded_sync(s, flags, "data flag")
            expect = torch.arange(nbytes // 8, dtype=torch.float64, device=dev) + 1000 * peer
            correct = ok and bool(torch.equal(got, expect))
            comm.barrier()
            # ping-pong latency over flag[1] (8 bytes in)
            n = 200
            torch.cuda.synchronize()
            comm.barrier()
            t0 = time.perf_counter()
            for i in range(1, n + 1):
                if me == 0:
                    native.stream_write_u64(s.cuda_stream, pf + 8, i)
                    native.stream_wait_u64_geq(s.cuda_stream, flags + 8, i)
                else:
                    native.stream_wait_u64_geq(s.cuda_stream, flags + 8, i)
                    native.stream_write_u64(s.cuda_stream, pf + 8, i)
            ok2 = bounded_sync(s, flags + 8, "ping-pong", deadline=20.0)
            dt = (time.perf_counter() - t0) / n * 1e6
            log(tag, f"put+flag correct={correct} pingpong_ok={ok2} round_trip={dt:.2f} us")
            torch.cuda.synchronize()
            comm.barrier()
            native.ipc_close(pf)
            native.ipc_close(pa)
            comm.barrier()
            native.ipc_free(flags)
            native.ipc_free(arena)
    igg.finalize_global_grid()


if __name__ == "__main__":
    child() if os.environ.get("IGG_PROBE_CHILD") else launch()
