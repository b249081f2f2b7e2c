#!/usr/bin/env python3
"""Cost of the timed-region bracket (barrier + synchronize) with an idle GPU.

Run under a launcher for several ranks (ranks may share one GPU here:
select_device is off). Prints, on rank 0, the mean wall time of one bracket:
  thread+monitored: bounded_device_sync (helper thread around
                    hipDeviceSynchronize) + gloo monitored barrier (round 1)
  event+gloo:       native bounded stream-event poll + gloo barrier + synchronize
  rccl+event:       one-element RCCL all-reduce + event poll + synchronize
                    (only with one GPU per rank, or a single rank)

Usage: python -m torch.distributed.run --nproc-per-node N benchmarks/bracket_cost.py [--share-gpu]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import igg  # noqa: E402
from igg.parallel.comm import bounded_device_sync, bounded_stream_sync  # noqa: E402


def main():
    share = "--share-gpu" in sys.argv
    if share:
        os.environ.setdefault("IGG_TRANSPORT", "staged")  # RCCL refuses ranks sharing a GPU
    me, dims, nprocs, coords, comm = igg.init_global_grid(16, 16, 16, quiet=True, select_device=not share)
    torch.cuda.synchronize()

    def t(f, n=100):
        f()
        comm.barrier()
        t0 = time.perf_counter()
        for _ in range(n):
            f()
        return (time.perf_counter() - t0) / n * 1e6

    def old():
        bounded_device_sync(comm=comm)
        comm.barrier()

    def event_gloo():
        bounded_stream_sync(comm=comm)
        comm.barrier()
        torch.cuda.synchronize()

    res = {"thread+monitored": t(old), "event+gloo": t(event_gloo)}
    if not share:
        comm.ensure_rccl() if nprocs > 1 else None

        def rccl():
            comm.device_barrier()
            bounded_stream_sync(comm=comm)
            torch.cuda.synchronize()

        res["rccl+event"] = t(rccl)
    if me == 0:
        print(f"{nprocs} rank(s){' sharing one GPU' if share else ''}: " +
              ", ".join(f"{k} {v:.0f} us" for k, v in res.items()), flush=True)
    igg.finalize_global_grid()


if __name__ == "__main__":
    main()
