#!/usr/bin/env python3
"""Static instruction census of the loops of one gfx950 kernel.

Disassembles a kernel of the native build (``llvm-objdump -d`` of the code
object that ``tools/kernel_resources.py`` unbundles), finds its loops (every
backward branch closes one: [target, branch]) and counts, per loop, the
instruction classes that decide a memory-bound sweep's issue budget: VALU,
cross-lane moves (``v_readlane``/``v_writelane``: also what SGPR spills
compile to), AGPR copies (``v_accvgpr_*``: what VGPR pressure above the 256
arch VGPRs compiles to), selects, scratch, vector memory and LDS. The x-march
loop of each per-wave sweep form of the fused kernel is one of the large
loops, so the per-form cost of the exchange can be read without a GPU.

Usage: python tools/loop_census.py UNIT|OBJECT.o KERNEL_SUBSTRING [--min 300] [--all]
  e.g. python tools/loop_census.py fused_t9_f64 'ELb0ELi2359503E'
"""
from __future__ import annotations

import argparse
import re
import subprocess
import sys
import tempfile
from collections import Counter
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
import kernel_resources as kr  # noqa: E402

CLASSES = (
    ("readlane", lambda m: m.startswith("v_readlane")),
    ("writelane", lambda m: m.startswith("v_writelane")),
    ("accvgpr", lambda m: m.startswith("v_accvgpr")),
    ("cndmask", lambda m: m.startswith("v_cndmask")),
    ("fp64", lambda m: m.endswith("_f64") or "_f64_" in m),
    ("valu", lambda m: m.startswith("v_")),
    ("salu", lambda m: m.startswith("s_") and not m.startswith(("s_load", "s_buffer", "s_waitcnt", "s_cbranch",
                                                                   "s_branch", "s_nop"))),
    ("smem", lambda m: m.startswith(("s_load", "s_buffer_load"))),
    ("vmem_load", lambda m: m.startswith(("global_load", "buffer_load", "flat_load"))),
    ("vmem_store", lambda m: m.startswith(("global_store", "buffer_store", "flat_store"))),
    ("scratch", lambda m: m.startswith("scratch_")),
    ("lds", lambda m: m.startswith("ds_")),
    ("waitcnt", lambda m: m.startswith("s_waitcnt")),
    ("nop", lambda m: m == "s_nop"),
)

LINE = re.compile(r"^\s+(\S+)(.*?)//\s*([0-9A-Fa-f]+):")
TARGET = re.compile(r"<[^>]*\+0x([0-9a-f]+)>")


def disassemble(unit: str) -> str:
    """``unit``: a unit of build/native, or the path of any HIP object."""
    obj = Path(unit) if unit.endswith(".o") else kr.BUILD / f"{unit}.hip.opt-fpc0.o"
    with tempfile.TemporaryDirectory() as td:
        co = kr._code_object(obj, Path(td))
        return subprocess.run([str(kr.LLVM / "llvm-objdump"), "-d", f"--mcpu={kr.ARCH}", str(co)],
                              check=True, capture_output=True, text=True).stdout


def functions(text: str) -> dict:
    """{symbol: [(address, mnemonic, operands, branch target or None)]}"""
    out, cur, base = {}, None, 0
    for line in text.splitlines():
        m = re.match(r"^([0-9a-f]+) <(.+)>:$", line)
        if m:
            base = int(m.group(1), 16)
            cur = out.setdefault(m.group(2), [])
            continue
        m = LINE.match(line)
        if m and cur is not None:
            tgt = TARGET.search(line)
            t = base + int(tgt.group(1), 16) if tgt and ("branch" in m.group(1)) else None
            cur.append((int(m.group(3), 16), m.group(1), m.group(2).strip(), t))
    return out


def census(ins: list) -> Counter:
    c = Counter(total=len(ins))
    for _a, mn, _ops, _t in ins:
        for name, f in CLASSES:
            if f(mn):
                c[name] += 1
    return c


def loops(ins: list, min_len: int) -> list:
    """Loop regions [start, end]: backward branches of at least ``min_len``
    instructions, overlapping ones merged."""
    addr = [a for a, *_ in ins]
    idx = {a: i for i, a in enumerate(addr)}
    found = []
    for i, (a, mn, _ops, t) in enumerate(ins):
        if t is not None and t <= a and t in idx:
            j = idx[t]
            if i - j + 1 >= min_len:
                found.append((j, i))
    # overlapping backward branches into one loop body (the row loop's
    # per-row conditions branch back to several points) form one region
    merged = []
    for j, i in sorted(set(found)):
        if merged and j <= merged[-1][1]:
            merged[-1] = (merged[-1][0], max(merged[-1][1], i))
        else:
            merged.append((j, i))
    return merged


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("unit")
    ap.add_argument("kernel", help="substring of the (mangled) kernel symbol")
    ap.add_argument("--min", type=int, default=300, help="smallest loop (instructions) to report")
    ap.add_argument("--all", action="store_true", help="every kernel matching the substring")
    a = ap.parse_args()
    fns = functions(disassemble(a.unit))
    hits = [k for k in fns if a.kernel in k]
    if not hits or (len(hits) > 1 and not a.all):
        print(f"{len(hits)} kernels match {a.kernel!r}: {hits[:4]}", file=sys.stderr)
        return 1
    cols = ["total"] + [n for n, _ in CLASSES]
    for h in hits:
        ins = fns[h]
        print(f"{h}: {len(ins)} instructions")
        print("| loop | " + " | ".join(cols) + " |")
        print("|---" * (len(cols) + 1) + "|")
        for j, i in loops(ins, a.min):
            c = census(ins[j:i + 1])
            print(f"| {ins[j][0]:x}-{ins[i][0]:x} | " + " | ".join(str(c[k]) for k in cols) + " |")
    return 0


if __name__ == "__main__":
    sys.exit(main())
