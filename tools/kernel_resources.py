#!/usr/bin/env python3
"""Per-kernel resource table of the gfx950 code objects of the native build.

For every HIP object of ``build/native`` (the units ``build.py`` links into
``_igg_native``) the gfx950 code object is unbundled from the object's
``.hip_fatbin`` section (``llvm-objcopy`` + ``clang-offload-bundler``), and
its AMDGPU metadata note (``llvm-readelf --notes``) and symbol table give, per
kernel: arch VGPRs + AGPRs (``.vgpr_count`` is the unified total on gfx950),
AGPRs, SGPRs, VGPR/SGPR spill counts, scratch bytes per lane
(``.private_segment_fixed_size``), static LDS bytes and machine-code bytes.

Kernel resources are what decide occupancy (512 unified VGPRs per SIMD lane:
one wave of a 512-VGPR kernel per SIMD) and whether a hot loop goes through
scratch, so a change in them is a performance change even when every bitwise
test still passes (compiling an unused path made every fused
form 10-20 % slower). ``tests/test_kernel_resources.py`` compares the table
against the checked-in baseline ``profiles/kernel_resources.json``.

Usage: python tools/kernel_resources.py [--write BASELINE] [--markdown OUT]
"""
from __future__ import annotations

import argparse
import json
import os
import re
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
BUILD = ROOT / "build" / "native"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
LLVM = ROCM / "lib" / "llvm" / "bin"
ARCH = os.environ.get("IGG_OFFLOAD_ARCH", "gfx950")
BASELINE = ROOT / "profiles" / "kernel_resources.json"
# what the metadata calls each column of the table
FIELDS = {".vgpr_count": "vgpr", ".agpr_count": "agpr", ".sgpr_count": "sgpr",
          ".vgpr_spill_count": "vgpr_spill", ".sgpr_spill_count": "sgpr_spill",
          ".private_segment_fixed_size": "scratch", ".group_segment_fixed_size": "lds"}


def objects(tag: str = "opt-fpc0") -> list[Path]:
    """The HIP objects of the default optimised build (one per .hip unit)."""
    return sorted(BUILD.glob(f"*.hip.{tag}.o"))


def _code_object(obj: Path, tmp: Path) -> Path:
    fb, co = tmp / (obj.name + ".fatbin"), tmp / (obj.name + ".hsaco")
    subprocess.run([str(LLVM / "llvm-objcopy"), f"--dump-section=.hip_fatbin={fb}", str(obj), str(tmp / "x.o")],
                   check=True, capture_output=True)
    subprocess.run([str(LLVM / "clang-offload-bundler"), "--unbundle", "--type=o",
                    f"--targets=hipv4-amdgcn-amd-amdhsa--{ARCH}", f"--input={fb}", f"--output={co}"],
                   check=True, capture_output=True)
    return co


def _metadata(co: Path) -> list[dict]:
    import yaml

    out = subprocess.run([str(LLVM / "llvm-readelf"), "--notes", str(co)], check=True, capture_output=True,
                         text=True).stdout
    i = out.index("---")
    j = out.index("\n...", i)
    return yaml.safe_load(out[i:j]).get("amdhsa.kernels", [])


def _code_bytes(co: Path) -> dict:
    out = subprocess.run([str(LLVM / "llvm-readelf"), "-s", "--wide", str(co)], check=True, capture_output=True,
                         text=True).stdout
    sizes = {}
    for line in out.splitlines():
        f = line.split()
        if len(f) >= 8 and f[3] == "FUNC":
            sizes[f[7]] = int(f[2], 0) if f[2].startswith("0x") else int(f[2])
    return sizes


def _demangle(names: list[str]) -> list[str]:
    for tool in (str(LLVM / "llvm-cxxfilt"), "c++filt"):
        try:
            r = subprocess.run([tool], input="\n".join(names), capture_output=True, text=True, check=True)
            return r.stdout.splitlines()
        except (OSError, subprocess.CalledProcessError):
            continue
    return names


def short_name(demangled: str) -> str:
    """Kernel template name with its arguments, without namespaces and the
    parameter list: ``diffusion3d_hx_kernel<double, 4, 8, 4, false, 1, true, 2359499>``."""
    s = re.sub(r"\((?:[^()]|\([^()]*\))*\)$", "", demangled)
    s = s.replace("igg::(anonymous namespace)::", "").replace("igg::", "")
    return s.replace("void ", "", 1) if s.startswith("void ") else s


def table(objs: list[Path] | None = None) -> dict:
    """{unit: {kernel short name: {vgpr, agpr, sgpr, vgpr_spill, sgpr_spill,
    scratch, lds, code_bytes}}} for the gfx950 code objects of ``objs``."""
    objs = objects() if objs is None else objs
    res = {}
    with tempfile.TemporaryDirectory() as td:
        tmp = Path(td)
        for obj in objs:
            co = _code_object(obj, tmp)
            md = _metadata(co)
            sizes = _code_bytes(co)
            names = _demangle([k[".name"] for k in md])
            unit = obj.name.split(".hip.")[0]
            rows = {}
            for k, dn in zip(md, names):
                row = {v: int(k.get(f, 0)) for f, v in FIELDS.items()}
                row["code_bytes"] = sizes.get(k[".name"], 0)
                rows[short_name(dn)] = row
            res[unit] = dict(sorted(rows.items()))
    return res


def markdown(t: dict) -> str:
    lines = ["| unit | kernel | VGPR (arch+acc) | AGPR | SGPR | VGPR spill | SGPR spill | scratch B | LDS B | code B |",
             "|---|---|---|---|---|---|---|---|---|---|"]
    for unit, rows in t.items():
        for name, r in rows.items():
            lines.append(f"| {unit} | `{name}` | {r['vgpr']} | {r['agpr']} | {r['sgpr']} | {r['vgpr_spill']} | "
                         f"{r['sgpr_spill']} | {r['scratch']} | {r['lds']} | {r['code_bytes']} |")
    return "\n".join(lines) + "\n"


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--write", default=None, help="write the table as JSON (the baseline: profiles/kernel_resources.json)")
    ap.add_argument("--markdown", default=None, help="write the table as a markdown file")
    a = ap.parse_args()
    objs = objects()
    if not objs:
        print("no HIP objects under build/native: run `python build.py` first", file=sys.stderr)
        return 1
    t = table(objs)
    if a.write:
        Path(a.write).write_text(json.dumps(t, indent=1, sort_keys=True) + "\n")
    if a.markdown:
        Path(a.markdown).write_text(markdown(t))
    if not a.write and not a.markdown:
        sys.stdout.write(markdown(t))
    n = sum(len(r) for r in t.values())
    spills = [(u, k) for u, rows in t.items() for k, r in rows.items() if r["scratch"] or r["vgpr_spill"]]
    print(f"{n} kernels in {len(t)} units; {len(spills)} with scratch or VGPR spills", file=sys.stderr)
    return 0


if __name__ == "__main__":
    sys.exit(main())
