"""Minimal in-situ visualisation helpers (the reference examples use Plots.jl
heatmaps + gif/mp4: examples/diffusion3D_multigpu_CuArrays.jl:42-67).

Only numpy + Pillow (no plotting stack on the MI355X image): ``heatmap``
maps a 2-D array through a perceptually ordered colormap to RGB, and
``Animation`` collects frames and writes an animated GIF.
"""
from __future__ import annotations

import numpy as np

# Anchor colours of a viridis-like map (dark blue -> teal -> green -> yellow).
_ANCHORS = np.array([[68, 1, 84], [59, 82, 139], [33, 145, 140], [94, 201, 98], [253, 231, 37]], dtype=np.float64)


def heatmap(a, vmin: float | None = None, vmax: float | None = None, scale: int = 1) -> np.ndarray:
    """RGB uint8 image of the 2-D array ``a`` (torch or numpy; first axis = rows)."""
    if hasattr(a, "detach"):
        a = a.detach().cpu().numpy()
    a = np.asarray(a, dtype=np.float64)
    if a.ndim != 2:
        raise ValueError("heatmap expects a 2-D array")
    lo = np.nanmin(a) if vmin is None else vmin
    hi = np.nanmax(a) if vmax is None else vmax
    t = np.clip((a - lo) / (hi - lo if hi > lo else 1.0), 0.0, 1.0) * (len(_ANCHORS) - 1)
    k = np.minimum(t.astype(np.int64), len(_ANCHORS) - 2)
    f = (t - k)[..., None]
    rgb = (_ANCHORS[k] * (1 - f) + _ANCHORS[k + 1] * f).astype(np.uint8)
    if scale > 1:
        rgb = rgb.repeat(scale, axis=0).repeat(scale, axis=1)
    return rgb[::-1]  # origin at the bottom, like a plot


class Animation:
    """Collect heatmap frames; ``save_gif(path, fps)`` writes them (rank 0 only)."""

    def __init__(self):
        self.frames: list[np.ndarray] = []

    def frame(self, a, **kw) -> None:
        self.frames.append(heatmap(a, **kw))

    def save_gif(self, path: str, fps: int = 15) -> None:
        from PIL import Image

        if not self.frames:
            raise ValueError("Animation has no frames")
        imgs = [Image.fromarray(f) for f in self.frames]
        imgs[0].save(path, save_all=True, append_images=imgs[1:], duration=int(1000 / fps), loop=0)
