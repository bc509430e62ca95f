"""Import helper: registers camera-aware-neural-networks-for-few-view-depth-estimation_amd/ (not a valid
Python identifier) as the package `cad_amd`."""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "camera-aware-neural-networks-for-few-view-depth-estimation_amd")


def load():
    if "cad_amd" in sys.modules:
        return sys.modules["cad_amd"]
    spec = importlib.util.spec_from_file_location("cad_amd", os.path.join(PKG_DIR, "__init__.py"),
                                                  submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["cad_amd"] = mod
    spec.loader.exec_module(mod)
    return mod
