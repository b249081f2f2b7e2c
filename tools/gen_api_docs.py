#!/usr/bin/env python3
"""Generate docs/api.md from the package's docstrings (the counterpart of the
reference's Documenter ``@autodocs`` page, docs/src/api.MD).

    python tools/gen_api_docs.py [--check]

``--check`` exits 1 if docs/api.md is out of date.
"""
from __future__ import annotations

import argparse
import inspect
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SECTIONS = [
    ("Grid", "igg", ["init_global_grid", "finalize_global_grid", "get_global_grid", "select_device"]),
    ("Halo update", "igg", ["update_halo_", "select_transport"]),
    ("Gather", "igg", ["gather_", "gather_async_"]),
    ("Global sizes and coordinates, timing", "igg",
     ["nx_g", "ny_g", "nz_g", "x_g", "y_g", "z_g", "coords_g", "tic", "toc"]),
    ("Checkpoint / restart", "igg", ["save_checkpoint", "load_checkpoint"]),
    ("Halo engine knobs", "igg.parallel.halo",
     ["set_transport", "transport_name", "tuned_transports", "set_halo_mode", "halo_mode", "set_pack_mode",
      "pack_mode", "enable_loopback", "sendranges", "recvranges", "halosize", "free_update_halo_buffers"]),
    ("Stencil ops", "igg.ops.stencil", ["diffusion3d_", "diffusion3d_reference", "time_variants", "autotune"]),
    ("Applications", "igg.models.diffusion3d", ["Diffusion3D"]),
    ("", "igg.models.acoustic2d", ["Acoustic2D"]),
    ("Field placement", "igg.utils.placement", ["candidate_count", "time_candidates", "placed"]),
    ("Tracing", "igg.utils.trace", None),
    ("Launcher", "igg.utils.launch", ["launch", "main"]),
]


def _sig(obj) -> str:
    try:
        return str(inspect.signature(obj))
    except (TypeError, ValueError):
        return "(...)"


def _entry(name: str, obj) -> list[str]:
    out = [f"### `{name}{_sig(obj)}`", ""]
    doc = inspect.getdoc(obj) or "(undocumented)"
    out += [doc, ""]
    if inspect.isclass(obj):
        for mname, m in inspect.getmembers(obj):
            if mname.startswith("_") or not (inspect.isfunction(m) or isinstance(m, property)):
                continue
            if isinstance(m, property):
                out += [f"* `{name}.{mname}` (property): {(inspect.getdoc(m) or '').splitlines()[0] if inspect.getdoc(m) else ''}"]
            else:
                d = inspect.getdoc(m)
                out += [f"* `{name}.{mname}{_sig(m)}`: {d.splitlines()[0] if d else ''}"]
        out += [""]
    return out


def render() -> str:
    import importlib

    lines = ["# API reference", "",
             "Generated from the docstrings by `tools/gen_api_docs.py` (do not edit by hand).",
             "Reference names: `update_halo!` → `update_halo_`, `gather!` → `gather_`.", ""]
    for title, modname, names in SECTIONS:
        mod = importlib.import_module(modname)
        if title:
            lines += [f"## {title}", ""]
        if names is None:
            names = [n for n in getattr(mod, "__all__", []) or
                     [n for n, o in vars(mod).items() if not n.startswith("_") and inspect.isfunction(o)
                      and o.__module__ == mod.__name__]]
            lines += [inspect.getdoc(mod) or "", ""]
        for n in names:
            lines += _entry(n, getattr(mod, n))
    return "\n".join(lines).rstrip() + "\n"


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--check", action="store_true")
    a = ap.parse_args()
    text = render()
    path = os.path.join(ROOT, "docs", "api.md")
    if a.check:
        cur = open(path).read() if os.path.exists(path) else ""
        if cur != text:
            print("docs/api.md is out of date: run python tools/gen_api_docs.py")
            return 1
        return 0
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as f:
        f.write(text)
    print(f"wrote {path}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
