"""Loader of the native runtime extension ``_igg_native`` (C++/HIP + RCCL).

The extension is built in-tree by ``python build.py`` (or
``__graft_entry__.build()``). ``torch`` is imported first so that the HIP
runtime and RCCL libraries already loaded by PyTorch-ROCm are the ones the
extension binds to (same sonames: one HIP runtime per process).

There is no pure-Python fallback: a missing extension is a hard error.
"""
from __future__ import annotations

import importlib
import os

import torch  # noqa: F401  (must precede the extension: shared HIP runtime / RCCL)

_PKG_DIR = os.path.dirname(os.path.abspath(__file__))


def _load():
    name = __package__ + "._igg_native" if __package__ else "_igg_native"
    try:
        return importlib.import_module(name)
    except ImportError as e:  # pragma: no cover - exercised only on broken installs
        if os.environ.get("IGG_AUTOBUILD", "1") != "0":
            import importlib.util as ilu

            bpath = os.path.join(os.path.dirname(_PKG_DIR), "build.py")
            if not os.path.exists(bpath):
                raise
            spec = ilu.spec_from_file_location("_igg_build", bpath)
            mod = ilu.module_from_spec(spec)
            spec.loader.exec_module(mod)
            mod.build()
            return importlib.import_module(name)
        raise ImportError(
            "The native IGG runtime (_igg_native) is not built. Run `python build.py` "
            "in the repository root."
        ) from e


native = _load()
IGGError = native.IGGError
PROC_NULL = int(native.PROC_NULL)
NDIMS = int(native.NDIMS)
NNEIGHBORS = int(native.NNEIGHBORS)
ALLOC_GRANULARITY = int(native.ALLOC_GRANULARITY)
THREADCOPY_THRESHOLD = int(native.THREADCOPY_THRESHOLD)

if os.environ.get("IGG_CRASH_BACKTRACE") == "1":
    # native backtrace of a fatal signal first, then faulthandler's Python
    # stack (enable faulthandler before importing igg for the chain)
    native.install_crash_handler()


def native_path() -> str:
    return native.__file__
