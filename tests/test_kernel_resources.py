"""Every gfx950 kernel in the product library runs out of registers: no
scratch (private segment) and no spills.  A dynamically indexed register
array is the usual way to lose that silently -- the pair lookup once put a
tap window in scratch (112 B/lane, 87 instead of 14 vector loads per wave,
+28 % time) with nothing else failing.  CPU only: reads the code object's
metadata from the built .so (tools/kernel_resources.py)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from kernel_resources import kernels  # noqa: E402

LIB = os.path.join(ROOT, "raft-stereo_amd", "_build", "libraftcorr.so")


@pytest.mark.skipif(not os.path.exists(LIB), reason="libraftcorr.so not built")
def test_no_product_kernel_uses_scratch():
    ks = kernels(LIB)
    assert len(ks) > 20, "code object metadata not found"
    # (SGPR spills go to VGPR lanes, not memory: allowed)
    bad = [(k["name"], k["scratch"], k["vgpr_spill"]) for k in ks
           if k["scratch"] or k["vgpr_spill"]]
    assert not bad, bad
    names = " ".join(k["name"] for k in ks)
    for must in ("lookup_pair_kernel", "lookup_chain_kernel", "build_f32_ring_kernel",
                 "volume_bwd_kernel", "lookup_bwd_pre_kernel"):
        assert must in names
