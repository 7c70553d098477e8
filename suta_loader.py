"""Import helper: the package directory is `test-time-adaptation-asr-suta_amd/` (a name with
hyphens, not importable by `import`), so it is registered as the module `suta_amd`."""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "test-time-adaptation-asr-suta_amd")


def load():
    if "suta_amd" in sys.modules:
        return sys.modules["suta_amd"]
    spec = importlib.util.spec_from_file_location(
        "suta_amd", os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["suta_amd"] = mod
    spec.loader.exec_module(mod)
    return mod
