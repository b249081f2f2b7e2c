#!/usr/bin/env python3
"""What the z face of a C-ordered field costs, per element.

The z face of an n^3 C-ordered field holds one element per row of n elements
(4 KiB apart at 512^3 f64). Cases, each one side of the face (n^2 elements):

  contig_pack     the x face (one contiguous n^2 block) through the copy kernel: control
  z_pack_copy     z = 1 -> buffer through the copy kernel's gather path (update_halo_'s pack)
  z_unpack_copy   buffer -> z = 0 through the copy kernel (update_halo_'s unpack)
  z_{pack,unpack}_copy_sys   the same with the put transport's system-scope stores
  stride_pack_{64..2048}B    n^2 single-element reads 64 B .. 2 KiB apart (row-hit control)
  zcol_{pack,unpack}_aux{A}   the same column with one buffer load / store per
                  element and cache-policy bits A on the strided access
                  (gfx950: 1 sc0, 2 nt, 3 sc0+nt, 16 sc1, 17 sc0+sc1, 18 sc1+nt)

Timing mode (default): median of 5 x --reps event-timed calls per case.
Counter mode (--pmc): every case runs exactly 1 + --reps times, back to back,
in the printed order, nothing else on the GPU, for
``rocprofv3 --pmc <counters> -- python3 benchmarks/zface_counters.py --pmc``;
``--parse DIR`` then maps the counter CSV's dispatches onto the cases (in
dispatch order) and prints per-element request counts and bytes.
"""
import argparse
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

AUX = (0, 1, 2, 3, 16, 17, 18)
PITCHES = (8, 16, 32, 64, 128, 256)  # elements (64 B .. 2 KiB); the z face is 512 (4 KiB)


def cases(n, T, buf, s):
    from igg._native import native

    eb = 8
    base, b = T.data_ptr(), buf.data_ptr()
    st = T.stride()
    out = [("contig_pack", lambda: native.copy2d([(base + 1 * st[0] * eb, b, n, n, st[1], st[2], n, 1)], eb, True, s)),
           ("z_pack_copy", lambda: native.copy2d([(base + 1 * eb, b, n, n, st[0], st[1], n, 1)], eb, True, s)),
           ("z_unpack_copy", lambda: native.copy2d([(b, base, n, n, n, 1, st[0], st[1])], eb, True, s)),
           # the put transport's form: system-scope (sc0 sc1, write-through) stores
           ("z_pack_copy_sys", lambda: native.copy2d([(base + 1 * eb, b, n, n, st[0], st[1], n, 1)], eb, True, s,
                                                     True)),
           ("z_unpack_copy_sys", lambda: native.copy2d([(b, base, n, n, n, 1, st[0], st[1])], eb, True, s, True))]
    rows, pitch = n * n, n
    # the same number of single-element requests at smaller strides: 64 B
    # apart every request is a new line of the SAME DRAM row as its
    # neighbours; 4 KiB apart (the z face) every request opens a new row
    for p in PITCHES:
        out.append((f"stride_pack_{p * 8}B", lambda p=p: native.zcol_probe(0, base + 1 * eb, b, rows, p, 0, s)))
    for a in AUX:
        out.append((f"zcol_pack_aux{a}", lambda a=a: native.zcol_probe(0, base + 1 * eb, b, rows, pitch, a, s)))
    for a in AUX:
        out.append((f"zcol_unpack_aux{a}", lambda a=a: native.zcol_probe(1, b, base, rows, pitch, a, s)))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--pmc", action="store_true", help="counter mode: 1 + reps untimed calls per case")
    ap.add_argument("--parse", default=None, help="parse a rocprofv3 --pmc output directory (no GPU)")
    a = ap.parse_args()
    if a.parse:
        return parse(a.parse, a.n, a.reps)
    import torch

    import igg  # noqa: F401

    n = a.n
    T = torch.rand(n, n, n, dtype=torch.float64, device="cuda")
    buf = torch.empty(n * n, dtype=torch.float64, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    cs = cases(n, T, buf, s)
    if a.pmc:
        for name, fn in cs:
            for _ in range(1 + a.reps):
                fn()
            torch.cuda.synchronize()
            print(f"case {name} x {1 + a.reps}", flush=True)
    else:
        for name, fn in cs:
            fn()
            torch.cuda.synchronize()
            ts = []
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    fn()
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1) / a.reps * 1e3)
            t = sorted(ts)[2]
            print(f"{name:20s} {t:8.2f} us  {n * n / t / 1e3:7.2f} Gelem/s  "
                  f"({n * n * 128 / t / 1e6:6.2f} TB/s at 128 B/elem, {n * n * 64 / t / 1e6:6.2f} at 64 B)", flush=True)
    if a.pmc:
        return 0
    # correctness of the probe forms: a pack then an unpack of every policy moves the column
    ref = T[:, :, 1].clone()
    for aux in AUX:
        buf.zero_()
        from igg._native import native

        native.zcol_probe(0, T.data_ptr() + 8, buf.data_ptr(), n * n, n, aux, s)
        torch.cuda.synchronize()
        assert torch.equal(buf.view(n, n), ref), f"zcol pack aux {aux}"
        T[:, :, 0].zero_()
        native.zcol_probe(1, buf.data_ptr(), T.data_ptr(), n * n, n, aux, s)
        torch.cuda.synchronize()
        assert torch.equal(T[:, :, 0], ref), f"zcol unpack aux {aux}"
    print("probe forms: bitwise OK", flush=True)


def parse(d, n, reps):
    """Counter CSV (one row per dispatch x counter) -> per-case means."""
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    if not rows:
        print(f"no counter_collection.csv under {d}")
        return 1
    by = {}
    for r in rows:
        did = int(r.get("Dispatch_Id") or r.get("Dispatch_ID") or 0)
        e = by.setdefault(did, {"kernel": r.get("Kernel_Name", "")})
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    # the cases' kernels only (torch's own kernels and the correctness
    # check after the cases run in between / after): the first
    # len(names) * per copy / zcol dispatches, in dispatch order
    disp = [by[k] for k in sorted(by) if "copy2d_batch_kernel" in by[k]["kernel"] or "zcol_kernel" in by[k]["kernel"]]
    names = ["contig_pack", "z_pack_copy", "z_unpack_copy", "z_pack_copy_sys", "z_unpack_copy_sys"] + \
            [f"stride_pack_{p * 8}B" for p in PITCHES] + [f"zcol_pack_aux{a}" for a in AUX] + \
            [f"zcol_unpack_aux{a}" for a in AUX]
    per = 1 + reps
    disp = disp[:len(names) * per]
    elems = n * n
    counters = sorted({k for x in disp for k in x if k != "kernel"})
    print("| case | " + " | ".join(f"{c} / elem" for c in counters) + " |")
    print("|---" * (len(counters) + 1) + "|")
    for i, name in enumerate(names):
        grp = disp[i * per + 1:(i + 1) * per]  # without the first (cold) call
        vals = [sum(x.get(c, 0.0) for x in grp) / len(grp) / elems for c in counters]
        print(f"| {name} | " + " | ".join(f"{v:.3f}" for v in vals) + " |")
    return 0


if __name__ == "__main__":
    sys.exit(main() or 0)
