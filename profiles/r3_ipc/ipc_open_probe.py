#!/usr/bin/env python3
"""Time hipIpcOpenMemHandle per allocation size and memory kind, 2 processes.

Each rank allocates one buffer of MemKind `kind` (0 default, 1 fine-grained,
3 uncached; csrc/include/igg/ipc.hpp) and `size`, exports its IPC handle,
then opens the peer's and writes 8 bytes into it (hipStreamWriteValue64). The
model fields of the fused exchange are one fine-grained allocation of
3 x n^3 elements (3.2 GiB at 512^3 f64) that every neighbour maps: this
prints how long export, open and first touch take for such sizes.
Every step runs under the caller's `timeout`; a line is printed per step so a
stuck step is named by the last line.

Usage: python profiles/r3_ipc/ipc_open_probe.py [--sizes-mib 64,1024,3300] [--kinds 0,1]
       (launches 2 ranks itself; --share-gpu style: both on device 0 unless
       --per-rank-device)
"""
import argparse
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def launch(argv):
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   GPU_MAX_HW_QUEUES="1")
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__), "--worker", *argv], env=env))
    return max(p.wait() for p in procs)


def worker(a):
    import torch
    import torch.distributed as dist
    from torch.utils import dlpack

    from igg._native import native

    rank = int(os.environ["RANK"])
    dist.init_process_group("gloo", rank=rank, world_size=2)
    torch.cuda.set_device(rank if a.per_rank_device else 0)

    def say(m):
        print(f"rank {rank}: {m}", flush=True)

    for kind in (int(k) for k in a.kinds.split(",")):
        for mib in (int(s) for s in a.sizes_mib.split(",")):
            nb = mib << 20
            t0 = time.perf_counter()
            buf = dlpack.from_dlpack(native.alloc_dlpack(nb, kind))
            t_alloc = time.perf_counter() - t0
            t0 = time.perf_counter()
            h = native.ipc_get_handle(buf.data_ptr())
            t_exp = time.perf_counter() - t0
            hs = [None, None]
            dist.all_gather_object(hs, h)
            say(f"kind {kind} {mib} MiB: alloc {t_alloc:.3f} s, export {t_exp * 1e3:.1f} ms; opening the peer's")
            t0 = time.perf_counter()
            p = native.ipc_open(hs[1 - rank])
            t_open = time.perf_counter() - t0
            say(f"kind {kind} {mib} MiB: open {t_open * 1e3:.1f} ms; touching")
            t0 = time.perf_counter()
            native.stream_write_u64(torch.cuda.current_stream().cuda_stream, p, 7)
            torch.cuda.synchronize()
            t_touch = time.perf_counter() - t0
            dist.barrier()
            native.ipc_close(p)
            dist.barrier()
            say(f"kind {kind} {mib} MiB: touch {t_touch * 1e3:.1f} ms, closed")
            del buf
            torch.cuda.synchronize()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes-mib", default="64,1024,3300")
    ap.add_argument("--kinds", default="0,1")
    ap.add_argument("--per-rank-device", action="store_true")
    ap.add_argument("--worker", action="store_true")
    a, rest = ap.parse_known_args()
    if a.worker:
        worker(a)
        return 0
    return launch([x for x in sys.argv[1:]])


if __name__ == "__main__":
    sys.exit(main())
