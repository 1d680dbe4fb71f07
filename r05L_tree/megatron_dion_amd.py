"""Import shim: exposes the `megatron-dion_amd/` directory as the package `megatron_dion_amd`.

The package directory carries the project's name (with a hyphen), which is not
a valid Python identifier; this module loads it under an importable name.
"""
import importlib.util
import os
import sys

_PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "megatron-dion_amd")
_spec = importlib.util.spec_from_file_location(
    __name__, os.path.join(_PKG_DIR, "__init__.py"), submodule_search_locations=[_PKG_DIR])
_pkg = importlib.util.module_from_spec(_spec)
sys.modules[__name__] = _pkg
_spec.loader.exec_module(_pkg)
