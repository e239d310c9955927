"""Import shim: exposes the package directory ``temporal-asymmetric-graph-attention-network_amd/``
(whose name is not a Python identifier) as the module ``tagan_amd``."""
import importlib.util as _ilu
import os as _os
import sys as _sys

_DIR = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "temporal-asymmetric-graph-attention-network_amd")
_spec = _ilu.spec_from_file_location("tagan_amd", _os.path.join(_DIR, "__init__.py"), submodule_search_locations=[_DIR])
_mod = _ilu.module_from_spec(_spec)
_sys.modules["tagan_amd"] = _mod
_spec.loader.exec_module(_mod)
