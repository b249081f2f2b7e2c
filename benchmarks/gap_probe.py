#!/usr/bin/env python3
"""Is the placement lottery (profiles/r6_placement/) about WHICH pages an
allocation gets, or about where T, Cp and T2 sit relative to each other?
K fine-grained buffers, each carved with several gaps between the three
arrays; every (buffer, gap) layout timed with the placement probe's sweep
(models/diffusion3d.py _time_placements). If the speed follows the gap within
one buffer, the relative placement decides; if it follows the buffer, the
pages do.

Usage: python benchmarks/gap_probe.py [--n 512] [--dtype float64] [--k 6]
       [--gaps 0,65536,266240,1048576,2363392,16777216] [--kinds 1,5]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--dtype", default="float64")
    ap.add_argument("--k", type=int, default=6)
    ap.add_argument("--gaps", default="0,65536,266240,1048576,2363392,16777216")
    ap.add_argument("--offset", type=int, default=0, help="extra offset of T from the buffer start")
    ap.add_argument("--kinds", default="1", help="native MemKinds of the buffers, cycled (ipc.hpp: 0 coarse, "
                    "1 fine, 4 VMM, 5 contiguous)")
    args = ap.parse_args()
    import torch

    import igg
    from igg.models import diffusion3d as D

    igg.init_global_grid(args.n, args.n, args.n, quiet=True)
    dtype = getattr(torch, args.dtype)
    shape = (args.n, args.n, args.n)
    nbytes = args.n ** 3 * torch.empty(0, dtype=dtype).element_size()
    gaps = [int(g) for g in args.gaps.split(",")]
    size = 3 * nbytes + 2 * max(gaps) + args.offset
    kinds = [int(x) for x in args.kinds.split(",")]
    bufs = [D.native_buffer(size, kinds[i % len(kinds)], torch.device("cuda")) for i in range(args.k)]

    def layout(buf, gap):
        o = args.offset
        return [buf[o + k * (nbytes + gap):o + k * (nbytes + gap) + nbytes].view(dtype).view(shape) for k in range(3)]

    cands, labels = [], []
    for i, b in enumerate(bufs):
        for g in gaps:
            cands.append(layout(b, g))
            labels.append((i, g))
    ms = D._time_placements(cands, dtype)
    print("buffer base      " + "".join(f"{g:>12d}" for g in gaps), flush=True)
    for i, b in enumerate(bufs):
        row = [ms[labels.index((i, g))] for g in gaps]
        print(f"#{i} kind {kinds[i % len(kinds)]} {b.data_ptr():#x} " + "".join(f"{t:12.5f}" for t in row), flush=True)
    igg.finalize_global_grid()


if __name__ == "__main__":
    main()
