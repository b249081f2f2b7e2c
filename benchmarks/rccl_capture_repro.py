#!/usr/bin/env python3
"""Minimal reproducer: RCCL p2p (one rank, send/recv to itself - the loopback
form of the halo exchange) captured into a hipGraph, on the capture-origin
stream and on streams forked from it inside the capture.

Every case runs in its own child process (a crash in one does not hide the
others); the parent never touches the GPU. Each child: capture -> replay 3x ->
check the received bytes -> report. Cases:
  origin     p2p on the capture-origin stream
  fork       p2p on a default-priority stream forked from the origin (event
             record/wait) and joined back before the end of the capture
  fork_prio  same, the forked stream created with the greatest priority (the
             overlapped Diffusion3D step's halo stream)
  fork_mask  same, the forked stream created with a CU mask (cu_partition)
  fork_kern  fork + a kernel on the origin stream concurrent with the p2p
  fork_warm  fork, with the eager warm-up exchange ALSO run on the forked stream
  fork_join_first  the p2p on the origin stream AFTER joining a forked branch
             (the form the overlapped step can take: fork, kernel on the side
             stream, join, then RCCL on the origin)
  side_kern  a kernel on the forked stream CONCURRENT with the p2p on the
             origin stream, joined after both (overlap with the roles swapped:
             interior on the fork, exchange on the origin)

Usage: python benchmarks/rccl_capture_repro.py [case ...]
"""
import os
import subprocess
import sys

CASES = ("origin", "fork", "fork_prio", "fork_mask", "fork_kern", "fork_warm", "fork_join_first", "side_kern")


def child(case: str) -> None:
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch

    import igg  # noqa: F401
    from igg._native import native

    comm = native.RcclComm(native.RcclComm.unique_id(), 1, 0)
    n = 1 << 20
    src = torch.arange(n, dtype=torch.float64, device="cuda")
    dst = torch.zeros_like(src)
    main = torch.cuda.Stream()
    if case == "fork_prio":
        lo, hi = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else (0, -1)
        side = torch.cuda.Stream(priority=min(lo, hi))
    elif case == "fork_mask":
        from igg.utils.streams import cu_partition

        _, side = cu_partition(16)
    else:
        side = torch.cuda.Stream()
    work = torch.empty(4 << 20, dtype=torch.float64, device="cuda")

    def exchange(s):
        comm.p2p([(dst.data_ptr(), n * 8, 0)], [(src.data_ptr(), n * 8, 0)], s.cuda_stream)

    # eager warm-up on the same streams (RCCL's lazy connection setup must not
    # happen inside the capture)
    with torch.cuda.stream(main):
        exchange(main)
    if case == "fork_warm":
        with torch.cuda.stream(side):
            exchange(side)
    torch.cuda.synchronize()
    dst.zero_()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(main):
        with torch.cuda.graph(g, stream=main, capture_error_mode="thread_local"):
            if case == "origin":
                exchange(main)
            elif case == "fork_join_first":
                side.wait_stream(main)
                with torch.cuda.stream(side):
                    work.mul_(1.0000001)
                main.wait_stream(side)
                exchange(main)
            elif case == "side_kern":
                side.wait_stream(main)
                with torch.cuda.stream(side):
                    work.mul_(1.0000001)
                exchange(main)
                main.wait_stream(side)
            else:
                side.wait_stream(main)
                if case == "fork_kern":
                    work.mul_(1.0000001)  # on main, concurrent with the p2p on side
                exchange(side)
                main.wait_stream(side)
            print(f"{case}: capture body done", flush=True)
    print(f"{case}: capture ended", flush=True)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    ok = torch.equal(dst, src)
    print(f"{case}: captured and replayed, data {'OK' if ok else 'WRONG'}", flush=True)
    sys.exit(0 if ok else 3)


def main() -> int:
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(sys.argv[2])
        return 0
    cases = sys.argv[1:] or list(CASES)
    worst = 0
    for c in cases:
        try:
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", c],
                               capture_output=True, text=True, timeout=120)
            tail = (r.stdout + r.stderr).strip().splitlines()
            mine = [ln for ln in tail if ln.startswith(c + ":")]
            if r.returncode == 0 and mine:
                msg = mine[-1]
            else:
                last = mine[-1][len(c) + 2:] if mine else "nothing"
                msg = f"{c}: FAILED rc={r.returncode} after '{last}'"
            print(msg, flush=True)
            worst = max(worst, 0 if r.returncode == 0 else 1)
        except subprocess.TimeoutExpired:
            print(f"{c}: TIMEOUT (120 s)", flush=True)
            worst = 1
    return worst


if __name__ == "__main__":
    sys.exit(main())
