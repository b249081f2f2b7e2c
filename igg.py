"""Import shim for the ``implicitglobalgrid.jl_amd`` package directory.

The framework's sources live in ``implicitglobalgrid.jl_amd/`` (a directory
name that is not a valid Python identifier). ``import igg`` loads that
directory as the package ``igg`` so that ``igg.parallel``, ``igg.models`` etc.
resolve to its sub-packages.
"""
import importlib.util as _ilu
import os as _os
import sys as _sys

_DIR = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "implicitglobalgrid.jl_amd")
_spec = _ilu.spec_from_file_location(
    __name__, _os.path.join(_DIR, "__init__.py"), submodule_search_locations=[_DIR]
)
_mod = _ilu.module_from_spec(_spec)
_sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
