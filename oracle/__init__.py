"""CPU oracle for the correlation path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg
may import this package.  The product path (``raft-stereo_amd``) never does and
fails loudly when its HIP library is missing.

Two restatements of /root/reference/model.py:267-326 live here:
  * ``corr_oracle.c`` via :mod:`oracle.coracle` -- plain C, bit-exact fp32
    sampler/pooling, fp64-accumulated volume (the parity checker);
  * :mod:`oracle.torch_ref` -- the reference's own ATen op sequence restated
    (einsum, avg_pool2d, grid_sample + torch.unique assert), timed as the CPU
    baseline (``cpu_baseline.kind == "port"``).
Both are pinned against tests/golden/*.npz (made by tests/golden/make_golden.py
from the patched reference in the build container).
"""
