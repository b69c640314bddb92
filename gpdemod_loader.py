"""Load the package `gppupildemodulation.jl_amd/` (dotted directory name) as module `gpdemod`."""
from __future__ import annotations

import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "gppupildemodulation.jl_amd")


def load():
    if "gpdemod" in sys.modules:
        return sys.modules["gpdemod"]
    spec = importlib.util.spec_from_file_location(
        "gpdemod", os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["gpdemod"] = mod
    spec.loader.exec_module(mod)
    return mod


def load_build():
    spec = importlib.util.spec_from_file_location("gpdemod_build", os.path.join(PKG_DIR, "build.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod
