"""Register the ``raft-stereo_amd/`` directory as the importable package
``raft_stereo_amd`` (the directory name carries a hyphen, which ``import``
cannot spell).  Used by tests/conftest.py, bench.py and __graft_entry__.py."""
import importlib.util
import os
import sys

NAME = "raft_stereo_amd"
ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "raft-stereo_amd")


def load():
    if NAME in sys.modules:
        return sys.modules[NAME]
    spec = importlib.util.spec_from_file_location(
        NAME, os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[NAME] = mod
    spec.loader.exec_module(mod)
    return mod
