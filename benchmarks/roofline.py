#!/usr/bin/env python3
"""HBM roofline probes on one GPU: triad (2 reads + 1 write, the stencil's mix)
and copy, 16 B/lane, with/without non-temporal stores, several grid sizes.
Bytes counted = compulsory bytes (3 x 1 GiB for triad)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import igg  # noqa: E402
from igg._native import native  # noqa: E402

KINDS = {0: "triad_nt", 1: "triad", 2: "copy_nt", 3: "copy", 4: "triad_nt_u8", 5: "read2_nt", 6: "write_nt"}


def main():
    n = 2 ** 27  # 1 GiB of f64 per array (= 512^3)
    a = torch.rand(n, dtype=torch.float64, device="cuda")
    b = torch.rand(n, dtype=torch.float64, device="cuda")
    o = torch.empty_like(a)
    s = torch.cuda.current_stream()
    res = {}
    for kind, name in KINDS.items():
        for blocks in (1024, 2048, 4096, 8192, 16384):
            args = (kind, o.data_ptr(), a.data_ptr(), b.data_ptr(), n, blocks, s.cuda_stream)
            native.stream_probe(*args)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(20):
                native.stream_probe(*args)
            e1.record(s)
            e1.synchronize()
            ms = e0.elapsed_time(e1) / 20
            nbytes = (3 if "triad" in name else 1 if name == "write_nt" else 2) * n * 8
            res[f"{name}@{blocks}"] = {"ms": round(ms, 4), "GBs": round(nbytes / (ms * 1e-3) / 1e9, 1)}
    best = max(res.items(), key=lambda kv: kv[1]["GBs"] if "triad" in kv[0] else 0)
    for kind in ("read2_nt", "write_nt", "copy_nt", "triad_nt"):
        b = max(((k, v) for k, v in res.items() if k.startswith(kind + "@")), key=lambda kv: kv[1]["GBs"])
        print(f"best {kind}: {b[0]} {b[1]['GBs']} GB/s", flush=True)
    print(json.dumps({"roofline": res, "best_triad": best}), flush=True)


if __name__ == "__main__":
    main()
