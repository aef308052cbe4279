"""Generate the golden fixtures in tests/golden/ from the reference itself.

Runs ONLY in the build container (it reads /root/reference/model.py, which
does not exist on the GPU box).  The reference as shipped cannot run its
correlation path (D2/D3 crash CorrBlock1D, D1/D4-D7 crash
RAFTStereo), so this script reads model.py as TEXT, applies the seven one-token
fixes in memory, and exec()s the result into a private module object.  Nothing
from the reference is written to disk except the numeric outputs below
(inputs + expected outputs = data, not source).

Usage:  python tests/golden/make_golden.py      (rewrites tests/golden/*.npz)
"""
import hashlib
import json
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference/model.py"
OUT = os.path.dirname(os.path.abspath(__file__))

# SURVEY.md Appendix A, D1-D7 (one token each).  D8 (the missing loop tail) is
# only needed for the end-to-end forward and is appended separately below.
FIXES = [
    ("nn.ReLU(in_planes=True)", "nn.ReLU(inplace=True)"),                       # D1 :22
    (".continguous()", ".contiguous()"),                                       # D2 :325
    ("torch.tensor(D).float)", "torch.tensor(D).float())"),                    # D3 :326
    ("BasicMultiUpdateBlock(self.args.hidden_dims==args.hidden_dims)",
     "BasicMultiUpdateBlock(self.args, hidden_dims=args.hidden_dims)"),        # D4 :341
    ("torch.cat(image1,image2,dim=0)", "torch.cat((image1,image2),dim=0)"),    # D5 :359
    ("out_chasnnels", "out_channels"),                                         # D6 :365
    ("radis=", "radius="),                                                     # D7 :367
]


# D8: the forward loop ends at model.py:383 with no
# coordinate update and no return.  Appended after the update_block call:
# zero the y component, step the coordinates, record the low-res flow.
D8_ANCHOR = ("net_list, up_mask, delta_flow = self.update_block(net_list, inp_list, corr, flow, "
             "iter32=self.args.n_gru_layers==3, iter16=self.args.n_gru_layers>=2)\n")
D8_TAIL = ("            delta_flow[:,1] = 0.0\n"
           "            coords1 = coords1 + delta_flow\n"
           "            flow_predictions.append(coords1 - coords0)\n"
           "        return flow_predictions\n")


def load_reference():
    sys.dont_write_bytecode = True
    with open(REF) as fh:
        text = fh.read()
    digest = hashlib.sha256(text.encode()).hexdigest()
    for old, new in FIXES:
        assert text.count(old) == 1, old
        text = text.replace(old, new)
    assert text.count(D8_ANCHOR) == 1
    text = text.replace(D8_ANCHOR, D8_ANCHOR + D8_TAIL)
    mod = types.ModuleType("patched_reference")
    exec(compile(text, "patched_reference", "exec"), mod.__dict__)
    return mod, digest


def gen(seed):
    return torch.Generator().manual_seed(seed)


def volume_case(ref, name, B, D, H, W1, W2, L, seed):
    g = gen(seed)
    f1 = torch.randn(B, D, H, W1, generator=g)
    f2 = torch.randn(B, D, H, W2, generator=g)
    blk = ref.CorrBlock1D(f1, f2, num_levels=L, radius=4)
    d = {"fmap1": f1.numpy(), "fmap2": f2.numpy(), "num_levels": np.int32(L)}
    for i, lvl in enumerate(blk.corr_pyramid):
        d[f"level{i}"] = lvl.reshape(lvl.shape[0], -1).numpy()
    np.savez_compressed(os.path.join(OUT, f"volume_{name}.npz"), **d)
    return {"kind": "volume", "B": B, "D": D, "H": H, "W1": W1, "W2": W2, "L": L,
            "widths": [int(blk.corr_pyramid[i].shape[-1]) for i in range(L + 1)]}


def lookup_coords(B, H, W1, W2, g, special=False):
    """x: grid minus a random disparity, with integer, negative, beyond-W and
    far out-of-bounds entries mixed in; y: random (the reference ignores it)."""
    w = torch.arange(W1, dtype=torch.float32).view(1, 1, W1).expand(B, H, W1)
    x = w - torch.rand(B, H, W1, generator=g) * min(64.0, W2 / 2)
    flat = x.reshape(-1).clone()
    n = flat.numel()
    idx = torch.randperm(n, generator=g)
    k = max(1, n // 10)
    flat[idx[:k]] = torch.randint(-6, W2 + 6, (k,), generator=g).float()         # integers
    flat[idx[k:2 * k]] = -torch.rand(k, generator=g) * 12.0                        # negative
    flat[idx[2 * k:3 * k]] = W2 - 6 + torch.rand(k, generator=g) * 20.0            # beyond W
    flat[idx[3 * k:3 * k + max(1, k // 4)]] = torch.tensor(
        [1e6, -1e6, 3.5e4, -7e5, 2.0 ** 24], dtype=torch.float32).repeat(k)[:max(1, k // 4)]
    if special:
        vals = [float("nan"), float("inf"), -float("inf"), 1e30, -1e30, 0.0, -0.0,
                0.5, W2 - 1.0, W2 - 0.5, W2 + 3.999, -4.0, -4.5, -5.0,
                np.nextafter(np.float32(7.0), np.float32(0.0)), np.float32(7.0) + np.float32(4.8e-7),
                3.0e-39, -3.0e-39]
        flat[:len(vals)] = torch.tensor(vals, dtype=torch.float32)
    x = flat.view(B, 1, H, W1)
    y = torch.randn(B, 1, H, W1, generator=g) * 5.0
    return torch.cat([x, y], dim=1)


def lookup_case(ref, name, B, D, H, W1, W2, L, r, seed, special=False):
    g = gen(seed)
    f1 = torch.randn(B, D, H, W1, generator=g)
    f2 = torch.randn(B, D, H, W2, generator=g)
    blk = ref.CorrBlock1D(f1, f2, num_levels=L, radius=r)
    coords = lookup_coords(B, H, W1, W2, g, special)
    out = blk(coords)
    d = {"fmap1": f1.numpy(), "fmap2": f2.numpy(), "coords": coords.numpy(),
         "out": out.numpy(), "num_levels": np.int32(L), "radius": np.int32(r)}
    for i in range(L):
        lvl = blk.corr_pyramid[i]
        d[f"level{i}"] = lvl.reshape(lvl.shape[0], -1).numpy()
    np.savez_compressed(os.path.join(OUT, f"lookup_{name}.npz"), **d)
    return {"kind": "lookup", "B": B, "D": D, "H": H, "W1": W1, "W2": W2, "L": L,
            "r": r, "special": special,
            "nan_out": int(np.isnan(out.numpy()).sum())}


def backward_case(ref, name, B, D, H, W1, W2, L, r, calls, seed):
    """Autograd of the reference path: fmaps require grad, ``calls`` lookups at
    different coordinates, loss = sum_k <out_k, G_k>.  Records the fmap
    gradients and every read level's total gradient (retain_grad)."""
    g = gen(seed)
    f1 = torch.randn(B, D, H, W1, generator=g).requires_grad_(True)
    f2 = torch.randn(B, D, H, W2, generator=g).requires_grad_(True)
    blk = ref.CorrBlock1D(f1, f2, num_levels=L, radius=r)
    for i in range(L):
        blk.corr_pyramid[i].retain_grad()
    coords = torch.stack([lookup_coords(B, H, W1, W2, g) for _ in range(calls)])
    gouts = torch.randn(calls, B, L * (2 * r + 1), H, W1, generator=g)
    loss = sum((blk(coords[k]) * gouts[k]).sum() for k in range(calls))
    loss.backward()
    d = {"fmap1": f1.detach().numpy(), "fmap2": f2.detach().numpy(), "coords": coords.numpy(),
         "grad_out": gouts.numpy(), "grad_fmap1": f1.grad.numpy(), "grad_fmap2": f2.grad.numpy(),
         "num_levels": np.int32(L), "radius": np.int32(r)}
    for i in range(L):
        lvl = blk.corr_pyramid[i]
        d[f"grad_level{i}"] = lvl.grad.reshape(lvl.shape[0], -1).numpy()
    np.savez_compressed(os.path.join(OUT, f"backward_{name}.npz"), **d)
    return {"kind": "backward", "B": B, "D": D, "H": H, "W1": W1, "W2": W2, "L": L, "r": r,
            "calls": calls}


class Args:
    """The seven attributes model.py reads (SURVEY.md §5 'Config / flags')."""
    def __init__(self, **kw):
        self.hidden_dims = [128] * 3
        self.n_downsample = 2
        self.n_gru_layers = 3
        self.corr_levels = 4
        self.corr_radius = 4
        self.mixed_precision = False
        self.slow_fast_gru = False
        self.__dict__.update(kw)


def state_hash(model):
    h = hashlib.sha256()
    for k, v in model.state_dict().items():
        h.update(k.encode())
        h.update(v.detach().contiguous().numpy().tobytes())
    return h.hexdigest()


sys.path.insert(0, os.path.dirname(OUT))
from golden_util import image_digest, stereo_pair  # noqa: E402  (one generator for both sides)


def e2e_case(ref, name, H, W, iters, seed, **kw):
    args = Args(**kw)
    torch.manual_seed(0)
    model = ref.RAFTStereo(args).eval()
    img1, img2 = stereo_pair(1, H, W, seed)
    with torch.no_grad():
        flows = model(img1, img2, iters=iters)
    disp = torch.stack([f[:, 0] for f in flows], 0).numpy()   # (iters, B, H1, W1)
    np.savez_compressed(os.path.join(OUT, f"e2e_{name}.npz"), image1=img1.numpy(),
                        image2=img2.numpy(), disparity=disp, iters=np.int32(iters))
    return {"kind": "e2e", "H": H, "W": W, "iters": iters, "args": vars(args),
            "state_sha256": state_hash(model),
            "n_tensors": len(model.state_dict()),
            "n_params": int(sum(p.numel() for p in model.parameters()))}


def e2e_seeded_case(ref, name, H, W, iters, seed, **kw):
    """A BASELINE-size end-to-end case whose images are NOT stored: the GPU
    test regenerates them with golden_util.stereo_pair(seed) and checks their
    sha256 against ``image_sha256``.  Only the final disparity is stored."""
    args = Args(**kw)
    torch.manual_seed(0)
    model = ref.RAFTStereo(args).eval()
    img1, img2 = stereo_pair(1, H, W, seed)
    with torch.no_grad():
        flows = model(img1, img2, iters=iters)
    disp = flows[-1][:, 0].numpy()                            # (B, H1, W1), final iteration
    np.savez_compressed(os.path.join(OUT, f"e2e_{name}.npz"), disparity=disp,
                        iters=np.int32(iters))
    return {"kind": "e2e_seeded", "H": H, "W": W, "iters": iters, "seed": seed,
            "args": vars(args), "image_sha256": image_digest(img1, img2),
            "state_sha256": state_hash(model)}


def main():
    only = sys.argv[1:]          # case names to (re)generate; default: all
    ref, digest = load_reference()
    torch.set_num_threads(8)
    manifest = {"reference_sha256": digest, "torch": torch.__version__,
                "fixes": [f[1] for f in FIXES], "cases": {}}
    if only:
        with open(os.path.join(OUT, "manifest.json")) as fh:
            manifest["cases"] = json.load(fh)["cases"]
    todo = {
        "v_w37": lambda: volume_case(ref, "w37", 2, 16, 3, 37, 37, 4, 1),
        "v_d256": lambda: volume_case(ref, "d256", 1, 256, 2, 24, 40, 4, 2),
        "v_d128": lambda: volume_case(ref, "d128", 1, 128, 2, 20, 33, 3, 3),
        "v_w70": lambda: volume_case(ref, "w70", 1, 64, 1, 70, 70, 4, 4),
        "v_w240": lambda: volume_case(ref, "w240", 1, 256, 1, 16, 240, 4, 5),
        "l_w37": lambda: lookup_case(ref, "w37", 2, 16, 3, 37, 37, 4, 4, 11),
        "l_w240": lambda: lookup_case(ref, "w240", 1, 32, 2, 16, 240, 4, 4, 12),
        "l_w311_r3": lambda: lookup_case(ref, "w311_r3", 1, 32, 2, 12, 311, 4, 3, 13),
        "l_w720": lambda: lookup_case(ref, "w720", 1, 16, 2, 8, 720, 4, 4, 14),
        "l_w60_L3": lambda: lookup_case(ref, "w60_L3", 2, 24, 2, 15, 60, 3, 4, 15),
        "l_special": lambda: lookup_case(ref, "special", 1, 16, 2, 16, 45, 4, 4, 16, special=True),
        "l_tiny": lambda: lookup_case(ref, "tiny", 1, 8, 2, 9, 16, 4, 2, 17),
        "b_w37": lambda: backward_case(ref, "w37", 2, 16, 3, 37, 37, 4, 4, 3, 31),
        "b_w64_L3": lambda: backward_case(ref, "w64_L3", 1, 32, 2, 40, 64, 3, 3, 2, 32),
        "b_d256": lambda: backward_case(ref, "d256", 1, 256, 2, 24, 40, 4, 4, 2, 33),
        "b_w45_L2": lambda: backward_case(ref, "w45_L2", 1, 8, 2, 16, 45, 2, 2, 3, 34),
        "e2e_default": lambda: e2e_case(ref, "default", 64, 96, 12, 21),
        "e2e_sfgru": lambda: e2e_case(ref, "sfgru", 64, 80, 6, 22, slow_fast_gru=True,
                                      corr_levels=3, corr_radius=3),
        "e2e_gru2_ds3": lambda: e2e_case(ref, "gru2_ds3", 96, 128, 5, 23, n_gru_layers=2,
                                         n_downsample=3, hidden_dims=[96, 96, 96]),
        # BASELINE.json configs[0]: one 1x3x320x720 pair, 12 iterations, default args
        "e2e_config1": lambda: e2e_seeded_case(ref, "config1", 320, 720, 12, 101),
        # BASELINE.json configs[2]'s image size: one 1x3x375x1242 pair, 32 iterations
        # (the fp32 reference; the GPU test runs the bf16 corr path against it)
        "e2e_config3": lambda: e2e_seeded_case(ref, "config3", 375, 1242, 32, 103),
        # BASELINE.json configs[1]'s image size: one 1x3x540x960 pair, 32 iterations
        "e2e_config2": lambda: e2e_seeded_case(ref, "config2", 540, 960, 32, 102),
        # BASELINE.json configs[3]: one 1x3x1984x2880 pair, 32 iterations (the
        # output RowShardedStereo's 1/2/4/8-GPU runs are checked against)
        "e2e_config4": lambda: e2e_seeded_case(ref, "config4", 1984, 2880, 32, 104),
    }
    for name, make in todo.items():
        if not only or name in only:
            manifest["cases"][name] = make()
    with open(os.path.join(OUT, "manifest.json"), "w") as fh:
        json.dump(manifest, fh, indent=1)
    print(json.dumps(manifest, indent=1))


if __name__ == "__main__":
    main()
