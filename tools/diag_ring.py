import os, sys
sys.path.insert(0, "/root/repo")
import pkgload; pkgload.load()
import torch, numpy as np
from raft_stereo_amd import CorrBlock1D, _lib
DEV = torch.device("cuda", 0)
for (B, D, H, W1, W2) in [(2, 256, 2, 311, 311), (1, 32, 2, 311, 311), (1, 32, 1, 128, 320), (1, 32, 1, 100, 100), (1, 32, 2, 128, 320)]:
    g = torch.Generator().manual_seed(5)
    f1 = torch.randn(B, D, H, W1, generator=g).bfloat16()
    f2 = torch.randn(B, D, H, W2, generator=g).bfloat16()
    with torch.no_grad():
        a = CorrBlock1D(f1.to(DEV), f2.to(DEV), num_levels=1, radius=2, pyramid_dtype=torch.float32, lazy_levels=False).corr_pyramid[0]
        a = a.reshape(B, H, W1, W2).cpu()
    ref = torch.einsum("bdhi,bdhj->bhij", f1.float(), f2.float()) / D ** 0.5
    d = (a - ref).abs() > 1e-3
    print((B, D, H, W1, W2), "bad", int(d.sum()), "of", d.numel())
    if d.any():
        idx = d.nonzero()
        for dim, name in enumerate("bhij"):
            u = torch.unique(idx[:, dim])
            print("  ", name, u[:40].tolist(), len(u))
        k = idx[0]
        print("   first bad", k.tolist(), float(a[tuple(k)]), float(ref[tuple(k)]))
