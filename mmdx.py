"""Import shim: `import mmdx` loads the package stored in the hyphenated directory
`multi-modal-medical-imaging-and-report-ml-diagnosis-system_amd/` (not a valid identifier)."""
import importlib.util
import os
import sys

_PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)),
                        "multi-modal-medical-imaging-and-report-ml-diagnosis-system_amd")
_spec = importlib.util.spec_from_file_location(
    __name__, os.path.join(_PKG_DIR, "__init__.py"), submodule_search_locations=[_PKG_DIR])
_mod = importlib.util.module_from_spec(_spec)
sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
