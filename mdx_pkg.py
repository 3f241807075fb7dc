"""Import helper: the package directory is named ``moseq2-detectron-extract_amd``
(not a valid Python identifier), so it is registered under the module name
``moseq2_detectron_extract_amd`` from its path.  ``load()`` is idempotent."""
from __future__ import annotations

import importlib.util
import os
import sys

NAME = "moseq2_detectron_extract_amd"
ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "moseq2-detectron-extract_amd")


def load():
    if NAME in sys.modules:
        return sys.modules[NAME]
    spec = importlib.util.spec_from_file_location(
        NAME, os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[NAME] = mod
    spec.loader.exec_module(mod)
    return mod
