#!/usr/bin/env python3
"""Build the native IGG runtime (`_igg_native`) in-tree for gfx950.

Every ``csrc/**/*.cpp`` (host C++) and ``csrc/kernels/*.hip`` (HIP device code)
is compiled with ``hipcc --offload-arch=gfx950`` and linked into one Python
extension next to the package sources, so it travels with the repository
snapshot to the GPU box. Incremental: objects are rebuilt only when a source or
any header is newer. No torch headers are used (the runtime takes raw
pointers), so a full build takes seconds.

Usage: ``python build.py [--clean] [-j N] [--debug] [--asan] [--probes]``

``--probes`` also compiles the measurement-only kernel forms of rounds 1-2
(stencil tilings and fused variants that lost their A/B, timing probes whose
results are wrong on purpose); the default build holds only what the autotune
shortlist, the fused A/B and their fallbacks use.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent
CSRC = ROOT / "csrc"
PKG = ROOT / "implicitglobalgrid.jl_amd"
BUILD = ROOT / "build" / "native"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
ARCH = os.environ.get("IGG_OFFLOAD_ARCH", "gfx950")
EXT_NAME = "_igg_native"


def ext_path() -> Path:
    return PKG / (EXT_NAME + sysconfig.get_config_var("EXT_SUFFIX"))


def _includes() -> list[str]:
    import pybind11

    return [
        f"-I{CSRC / 'include'}",
        f"-I{pybind11.get_include()}",
        f"-I{sysconfig.get_paths()['include']}",
        f"-I{ROCM / 'include'}",
    ]


def _sources() -> list[Path]:
    return sorted(CSRC.glob("*.cpp")) + sorted((CSRC / "kernels").glob("*.hip"))


def _headers_mtime() -> float:
    hs = list((CSRC / "include").rglob("*.hpp"))
    return max((h.stat().st_mtime for h in hs), default=0.0)


def _compile(src: Path, obj: Path, flags: list[str]) -> tuple[Path, str]:
    hipcc = str(ROCM / "bin" / "hipcc")
    lang = ["-x", "hip", f"--offload-arch={ARCH}"] if src.suffix == ".hip" else ["-x", "c++", "-D__HIP_PLATFORM_AMD__"]
    cmd = [hipcc, *lang, *flags, *_includes(), "-c", str(src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj, r.stderr


def build(jobs: int | None = None, debug: bool = False, asan: bool = False, verbose: bool = False,
          probes: bool = False) -> Path:
    BUILD.mkdir(parents=True, exist_ok=True)
    flags = ["-std=c++17", "-fPIC", "-fvisibility=hidden", "-Wall", "-Wno-unused-result"]
    flags += ["-O0", "-g"] if debug else ["-O3"]
    # No floating-point contraction: the stencil variants, the fused exchange
    # forms and the plain steps must compute bitwise the same values (the
    # bench's checks and tests compare them exactly), and with contraction on
    # the compiler fuses a*b+c into an FMA per instantiation as register
    # pressure and scheduling dictate - one changed fused form differed from
    # the plain step by 1 ulp at 2 cells (round 4, f32 tiling 40 direct z).
    # Formulas that want an FMA spell it out (__builtin_fma).
    flags += ["-ffp-contract=off"]
    if asan:
        # Host-code sanitizer only (GPU ASan is not available on the pool).
        flags += ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fno-omit-frame-pointer"]
    if probes:
        flags += ["-DIGG_PROBES"]
    # measurement builds only (e.g. "-DIGG_WAVES_PER_EU=2"); part of the object tag
    extra = os.environ.get("IGG_EXTRA_FLAGS", "").split()
    flags += extra
    tag = ("dbg" if debug else "opt") + ("-asan" if asan else "") + ("-probes" if probes else "") + "-fpc0"
    if extra:
        tag += "-x" + "".join(c for c in "".join(extra) if c.isalnum())
    hdr_t = _headers_mtime()
    todo = []
    objs = []
    for src in _sources():
        obj = BUILD / f"{src.stem}.{src.suffix[1:]}.{tag}.o"
        objs.append(obj)
        if not obj.exists() or obj.stat().st_mtime < max(src.stat().st_mtime, hdr_t):
            todo.append((src, obj))
    # the heavy fused-kernel units first (longest job first: the clean build's
    # wall time is the slowest unit's, ~2.2 min, not a tail behind the others)
    todo.sort(key=lambda t: (not t[0].name.startswith("fused_t"), t[0].name))
    jobs = jobs or min(8, os.cpu_count() or 4)
    if todo:
        with cf.ThreadPoolExecutor(jobs) as ex:
            for obj, err in ex.map(lambda t: _compile(t[0], t[1], flags), todo):
                if verbose and err.strip():
                    print(err, file=sys.stderr)
    out = ext_path()
    newest = max(o.stat().st_mtime for o in objs)
    stamp = BUILD / "last_link_tag"
    same_tag = stamp.exists() and stamp.read_text() == tag
    if not out.exists() or out.stat().st_mtime < newest or todo or not same_tag:
        link = [
            str(ROCM / "bin" / "hipcc"), "-shared", "-fPIC", f"--offload-arch={ARCH}",
            *map(str, objs), "-o", str(out) + ".tmp",
            f"-L{ROCM / 'lib'}", "-lrccl", "-lamdhip64", "-ldl", f"-Wl,-rpath,{ROCM / 'lib'}",
        ]
        if asan:
            link += ["-fsanitize=address"]
        r = subprocess.run(link, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed\n{' '.join(link)}\n{r.stdout}\n{r.stderr}")
        os.replace(str(out) + ".tmp", out)
        stamp.write_text(tag)
    return out


def main() -> None:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("-j", type=int, default=None)
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--asan", action="store_true")
    ap.add_argument("--probes", action="store_true", help="also compile the measurement-only kernel forms")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args()
    if a.clean:
        shutil.rmtree(BUILD, ignore_errors=True)
        ext_path().unlink(missing_ok=True)
    out = build(a.j, a.debug, a.asan, a.verbose, a.probes)
    print(f"built {out.relative_to(ROOT)}")


if __name__ == "__main__":
    main()
