"""Import helper for the product package.

The package directory is named ``template-matching-and-regression-mapreduce_amd``
(not a valid Python identifier), so it is registered in ``sys.modules`` under
the import name ``tmr_amd``.  After ``load_package()`` ordinary
``import tmr_amd`` / ``from tmr_amd import matching_net`` work.
"""
from __future__ import annotations

import importlib.util
import os
import sys

PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)),
                       "template-matching-and-regression-mapreduce_amd")
PKG_NAME = "tmr_amd"


def load_package():
    if PKG_NAME in sys.modules:
        return sys.modules[PKG_NAME]
    spec = importlib.util.spec_from_file_location(
        PKG_NAME, os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[PKG_NAME] = mod
    try:
        spec.loader.exec_module(mod)
    except BaseException:
        sys.modules.pop(PKG_NAME, None)
        raise
    return mod
