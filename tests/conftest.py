import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import pkgload  # noqa: E402

pkgload.load()  # registers raft-stereo_amd/ as `raft_stereo_amd`

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X)")


def _gpu_ok():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _gpu_ok():
        return
    skip = pytest.mark.skip(reason="no HIP device")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


class _DevLibraryOrSkip:
    """``_lib.dev_library()`` for the variant bit-identity tests: the dev
    library (libraftcorr_dev.so: A/B knobs, ablation variants) is not pushed
    to the GPU box by default (.gpurunignore), so a test that needs it skips
    when it is absent instead of failing; the product library never needs it."""

    def __init__(self):
        from raft_stereo_amd import _lib
        self._inner = _lib._DevLibrary()

    def __enter__(self):
        from raft_stereo_amd import _lib
        if not os.path.exists(_lib.DEV_LIB_PATH):
            pytest.skip("libraftcorr_dev.so not present (dev-library variant test)")
        return self._inner.__enter__()

    def __exit__(self, *exc):
        return self._inner.__exit__(*exc)


def _install_dev_library_skip():
    from raft_stereo_amd import _lib
    _lib.dev_library = _DevLibraryOrSkip


_install_dev_library_skip()
