#!/usr/bin/env python3
"""Where does the autotuned stencil time differ from the timed bench loop?

Builds the 512^3 f64 Diffusion3D model like bench.py (autotuned variant), then
reports, per step (events on the stream):
  * the autotune's own number for the chosen (variant, rounds);
  * fixed-buffer launches T2 = f(T) (the autotune's shape);
  * ping-pong eager steps (T2 = f(T), swap);
  * hipGraph replays of GRAPH_STEPS steps, each replay timed separately
    (the first replay after capture included), and the driver's shape:
    warm-up 5, capture, 20 timed steps with host timing.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

import igg  # noqa: E402
from igg.models.diffusion3d import Diffusion3D  # noqa: E402
from igg.ops import stencil  # noqa: E402


def ev_time(fn, reps=1):
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--variant", default=None)
    a = ap.parse_args()
    if a.variant is not None:
        os.environ["IGG_STENCIL_VARIANT"] = a.variant
    n = a.n
    igg.init_global_grid(n, n, n, quiet=True)
    m = Diffusion3D(dtype=torch.float64)
    out = {"variant": m.variant, "rounds": m.rounds}
    if m.variant_times:
        out["autotune_ms"] = m.variant_times.get(f"{m.variant}@r{m.rounds}")
    rd2 = [1.0 / m.dx ** 2, 1.0 / m.dy ** 2, 1.0 / m.dz ** 2]
    boxes = [(list(b[0]), list(b[1])) for b in m.inner]
    s = torch.cuda.current_stream().cuda_stream

    def fixed():
        stencil.native.diffusion3d(m.T2.data_ptr(), m.T.data_ptr(), m.Cp.data_ptr(), list(m.T.shape), rd2,
                                   m.dt * m.lam, 8, boxes, True, m.variant, s, m.rounds)

    fixed()
    out["fixed_5x_ms"] = [round(ev_time(fixed, 5), 5) for _ in range(5)]
    m.step()
    out["eager_pingpong_20_ms"] = [round(ev_time(m.step, 20), 5) for _ in range(3)]
    out["eager_each_ms"] = [round(ev_time(m.step), 5) for _ in range(10)]
    m.capture()
    k = m.graph_steps
    out["replay_each_ms_per_step"] = [round(ev_time(m.graph.replay) / k, 5) for _ in range(12)]
    # the driver's shape, with a fresh capture: 5 warm-up steps, capture, 20 timed steps (host clock)
    for cap_warm in (0, 1):
        m.graph = None
        for _ in range(5):
            m.step()
        m.capture()
        if cap_warm:
            m.graph.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        m.run(20)
        torch.cuda.synchronize()
        out[f"driver_shape_20_ms{'_after_1_replay' if cap_warm else ''}"] = round((time.perf_counter() - t0) / 20 * 1e3, 5)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    m.run(200)
    torch.cuda.synchronize()
    out["run_200_ms"] = round((time.perf_counter() - t0) / 200 * 1e3, 5)
    print(json.dumps(out))
    igg.finalize_global_grid()


if __name__ == "__main__":
    main()
