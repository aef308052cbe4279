"""raft_stereo_amd -- MI355X-native correlation path for RAFT-Stereo.

The package holds only the hot path named by BASELINE.json's north_star:
  * ``csrc/``   hand-written gfx950 HIP kernels (volume + fused pyramid,
                lookup, pool) behind the C-ABI in include/raftcorr.h;
  * ``corr``    the drop-in ``CorrBlock1D`` mirroring /root/reference/model.py:283-326
                (constructor, ``__call__(coords)``, ``corr`` staticmethod,
                ``corr_pyramid`` attribute) plus ``coords_grid`` (:329-332);
  * ``_lib``    the ctypes binding of libraftcorr.so.  There is no CPU
                fallback: without the built library or a HIP device the
                calls raise.
"""
from .corr import CorrBlock1D, coords_grid  # noqa: F401

__all__ = ["CorrBlock1D", "coords_grid"]
