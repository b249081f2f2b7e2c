"""Kernel resource guard.

The gfx950 code objects of the build are read back (tools/kernel_resources.py:
AMDGPU metadata of every kernel) and compared with the checked-in baseline
``profiles/kernel_resources.json``. A kernel's VGPRs decide its occupancy (512
unified registers per SIMD lane) and scratch puts a hot loop's spills in
memory: round 5 saw every fused form get 10-20 % slower when an unused path
was merely compiled in, with every bitwise test still green. So any increase
fails here, and the baseline is updated on purpose
(``python tools/kernel_resources.py --write profiles/kernel_resources.json
--markdown profiles/kernel_resources.md``) with the measurement that justifies it.
CPU-only: the objects are cross-compiled in this container.
"""
import importlib.util as ilu
import json
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
_spec = ilu.spec_from_file_location("kernel_resources", ROOT / "tools" / "kernel_resources.py")
kr = ilu.module_from_spec(_spec)
_spec.loader.exec_module(kr)

# Kernels that may use scratch (baseline value, never more). Each is either
# not on a product path or measured with its spill (profiles/kernel_resources.md):
#  * tiling 141 f64 (plain variant 43, the headline's usual autotune pick):
#    4 VGPRs spilled at the 256-VGPR / 2-waves-per-SIMD point; a 1-wave form
#    would lose half the occupancy;
#  * deferred-send (DF) and edge-lane direct-z forms of the 512-VGPR fused
#    tilings 9 / 14 (f64): not in the bench's f64 candidate lists.
SCRATCH_OK_UNITS = {"fused_kernels", "fused_t9_f64", "fused_t14_f64"}


@pytest.fixture(scope="module")
def current():
    objs = kr.objects()
    if not objs:
        pytest.skip("no HIP objects under build/native (run `python build.py`)")
    return kr.table(objs)


@pytest.fixture(scope="module")
def baseline():
    return json.loads(kr.BASELINE.read_text())


def test_every_kernel_is_in_the_baseline(current, baseline):
    new = [f"{u}: {k}" for u, rows in current.items() for k in rows if k not in baseline.get(u, {})]
    assert not new, ("kernels without a baseline entry (update profiles/kernel_resources.json on purpose): "
                     + "; ".join(new[:10]))


def test_no_resource_increase(current, baseline):
    grew = []
    for u, rows in current.items():
        for k, r in rows.items():
            b = baseline.get(u, {}).get(k)
            if b is None:
                continue
            for f in ("vgpr", "agpr", "scratch", "vgpr_spill", "lds"):
                if r[f] > b[f]:
                    grew.append(f"{u}: {k}: {f} {b[f]} -> {r[f]}")
    assert not grew, "kernel resources grew: " + "; ".join(grew[:10])


def test_scratch_only_where_recorded(current):
    bad = [f"{u}: {k} ({r['scratch']} B)" for u, rows in current.items() for k, r in rows.items()
           if r["scratch"] and u not in SCRATCH_OK_UNITS]
    assert not bad, "scratch in a kernel outside the recorded units: " + "; ".join(bad)


def test_product_paths_without_scratch(current):
    """The copy kernel (every generic update_halo_ pack/unpack), the gather,
    put and acoustic kernels and the plain stencil kernels keep every value in
    registers (a 16-B element array went to scratch before round 6)."""
    for u in ("copy_kernels", "gather_kernels", "put_kernels", "acoustic_kernels", "stencil_kernels"):
        for k, r in current.get(u, {}).items():
            assert r["scratch"] == 0 and r["vgpr_spill"] == 0, (u, k, r)


def test_markdown_table_matches_baseline(baseline):
    """profiles/kernel_resources.md is the readable form of the same baseline."""
    md = (kr.BASELINE.parent / "kernel_resources.md").read_text()
    assert md == kr.markdown(baseline)
