"""Import shim for the ``sg-nerf_amd/`` package directory.

The package directory name is not a Python identifier, so ``import sgnerf_amd``
lands here and re-binds itself to ``sg-nerf_amd/__init__.py`` as a regular
package (its submodules then import as ``sgnerf_amd.<name>``).
"""
import importlib.util
import os
import sys

_PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "sg-nerf_amd")
_spec = importlib.util.spec_from_file_location(
    __name__, os.path.join(_PKG_DIR, "__init__.py"), submodule_search_locations=[_PKG_DIR])
_module = importlib.util.module_from_spec(_spec)
sys.modules[__name__] = _module
_spec.loader.exec_module(_module)
