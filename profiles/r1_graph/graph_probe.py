#!/usr/bin/env python3
"""Probe hipGraph capture/replay of a diffusion step, printing progress markers.

Usage: python profiles/r1_graph/graph_probe.py {local|loopback} [--mode sequential|onephase] [--n 64]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def mark(msg):
    print(f"[{time.strftime('%H:%M:%S')}] {msg}", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kind", choices=["local", "loopback", "rccl_only"])
    ap.add_argument("--mode", default="sequential")
    ap.add_argument("--n", type=int, default=64)
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    import torch

    import igg
    from igg.models.diffusion3d import Diffusion3D
    from igg.parallel import halo as H

    n = a.n
    igg.init_global_grid(n, n, n, periodx=1, periody=1, periodz=1, quiet=True)
    if a.kind in ("loopback", "rccl_only"):
        H.enable_loopback()
        H.set_halo_mode(a.mode)
    mark(f"init done kind={a.kind} mode={H.halo_mode()}")
    if a.kind == "rccl_only":
        A = torch.zeros(n, n, n, dtype=torch.float64, device="cuda")
        igg.update_halo_(A)
        torch.cuda.synchronize()
        mark("eager update_halo done")
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            igg.update_halo_(A)
        mark("captured")
        g.replay()
        torch.cuda.synchronize()
        mark("replayed")
        return
    m = Diffusion3D(dtype=torch.float64)
    m.step()
    torch.cuda.synchronize()
    mark("eager step done")
    m.capture()
    mark("captured")
    m.graph.replay()
    torch.cuda.synchronize()
    mark("replay 1 done")
    t0 = time.perf_counter()
    m.run(a.steps)
    torch.cuda.synchronize()
    mark(f"run {a.steps}: {(time.perf_counter() - t0) / a.steps * 1e3:.4f} ms/step")
    igg.finalize_global_grid()


if __name__ == "__main__":
    main()
