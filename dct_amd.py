"""Import alias for the framework package.

The package directory is named
``distributed-continuous-training-with-airflow-pytorch-distributed-ddp-_amd`` (the
project's canonical name), which is not a valid Python identifier.  Importing
``dct_amd`` loads that directory as a regular package and registers it under the
importable name, so ``import dct_amd.models`` / ``python -m dct_amd.jobs.train``
work from the repository root (and from any process that has the root on
``sys.path``, e.g. torchrun workers).
"""
import importlib.util as _ilu
import os as _os
import sys as _sys

PACKAGE_DIRNAME = "distributed-continuous-training-with-airflow-pytorch-distributed-ddp-_amd"
_PKG_DIR = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), PACKAGE_DIRNAME)

_spec = _ilu.spec_from_file_location(
    __name__, _os.path.join(_PKG_DIR, "__init__.py"), submodule_search_locations=[_PKG_DIR]
)
_mod = _ilu.module_from_spec(_spec)
_mod.PACKAGE_DIRNAME = PACKAGE_DIRNAME
_sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
