#!/usr/bin/env python3
"""Minimal reproducer: hipGraph replay of a capture that forks onto a second
stream, in a process limited to one hardware queue (GPU_MAX_HW_QUEUES=1).

Round 3 saw the overlapped put step (``Diffusion3D(overlap=True)``: halo
exchange on a high-priority forked stream, interior on the capture stream)
crash with SIGSEGV inside ``CUDAGraph.replay`` on every rank of a 4-rank
shared-GPU rehearsal (profiles/r3_overlap_crash/). Round 4 reproduced it in
ONE process with the 1-GPU loopback (``bench.py --loopback --periodic-dims xy
--overlap --transport put``): it crashes with GPU_MAX_HW_QUEUES=1 (which the
bench's shared-GPU self-launch sets for more than 2 ranks) and replays fine
with the box default of 4 (profiles/r4_overlap_crash/).

This script strips the model away: plain torch elementwise kernels, captured
as ``--steps`` repetitions of [kernel on the capture stream; fork; kernel on the
side stream; join], replayed ``--replays`` times. ``--side`` picks the side
stream's priority (``none`` = no fork). With IGG_CRASH_BACKTRACE=1 the native
runtime prints the C backtrace of a crash before faulthandler's Python stack.

usage: GPU_MAX_HW_QUEUES=1 python benchmarks/graph_fork_repro.py --side high
"""
from __future__ import annotations

import argparse
import faulthandler
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--side", default="high", choices=["none", "default", "high", "low"])
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--replays", type=int, default=50)
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--branches", type=int, default=1,
                    help="side streams forked per step (concurrent graph branches besides the capture stream)")
    ap.add_argument("--kernels", type=int, default=1, help="kernels per branch per step")
    args = ap.parse_args()
    faulthandler.enable()
    import torch

    if os.environ.get("IGG_CRASH_BACKTRACE") == "1":
        from igg import native

        native.install_crash_handler()
    a = torch.zeros(args.n, device="cuda")
    bs = [torch.zeros(args.n, device="cuda") for _ in range(max(1, args.branches))]
    sides = []
    if args.side != "none":
        lo, hi = torch.cuda.Stream.priority_range()
        prio = {"default": 0, "high": hi, "low": lo}[args.side]
        sides = [torch.cuda.Stream(priority=prio) for _ in range(args.branches)]
    main_s = torch.cuda.Stream()

    def step():
        for _ in range(args.kernels):
            a.add_(1.0)
        if sides:
            cur = torch.cuda.current_stream()
            for sd in sides:
                sd.wait_stream(cur)
            for sd, b in zip(sides, bs):
                with torch.cuda.stream(sd):
                    for _ in range(args.kernels):
                        b.add_(1.0)
            for sd in sides:
                cur.wait_stream(sd)
        else:
            for b in bs:
                for _ in range(args.kernels):
                    b.add_(1.0)

    with torch.cuda.stream(main_s):
        step()  # warm-up (allocator, kernels)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(main_s):
        with torch.cuda.graph(g, stream=main_s, capture_error_mode="thread_local"):
            for _ in range(args.steps):
                step()
    torch.cuda.synchronize()
    print(f"captured {args.steps} steps ({args.branches} side stream(s): {args.side}, {args.kernels} kernel(s) "
          f"per branch, GPU_MAX_HW_QUEUES="
          f"{os.environ.get('GPU_MAX_HW_QUEUES')}); replaying {args.replays} times", flush=True)
    for _ in range(args.replays):
        g.replay()
    torch.cuda.synchronize()
    want = args.kernels * (1 + args.steps * args.replays)
    ok = bool((a == want).all().item() and all((b == want).all().item() for b in bs))
    print(f"replays done: a={a[0].item():.0f} b0={bs[0][0].item():.0f} (want {want}): {'OK' if ok else 'WRONG'}",
          flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
