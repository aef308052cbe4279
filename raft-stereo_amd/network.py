"""RAFT-Stereo host network around the MI355X correlation path.

Counterpart of ``RAFTStereo`` in /root/reference/model.py (:335-383) -- the
caller of the hot path.  Per north_star the encoders, ConvGRUs and heads stay
on ordinary PyTorch ops; only the correlation block (``corr_block``, default
:class:`raft_stereo_amd.CorrBlock1D`) runs on the gfx950 kernels.  The module
tree (attribute names, construction order, init calls) reproduces the
reference's so that ``torch.manual_seed(s); RAFTStereo(args)`` yields the
same weights and the same ``state_dict`` keys; tests pin the weight hash and
the per-iteration disparity against goldens made from the reference.

Reference defects are repaired as SURVEY.md Appendix A lists (D1 ReLU kwarg,
D4 update-block args, D5 cat tuple, D6 out_channels, D7 radius kwarg) and the
truncated loop (D8) is completed the way the golden generator completes it:
y-flow zeroed, coordinates stepped, low-resolution flow appended, list
returned.  Everything else -- the missing final ReLU in residual blocks, the
never-applied dropout, the unused ``test_mode`` -- is kept.

``args`` is any object with the seven attributes the reference reads
(SURVEY.md §5): hidden_dims, n_downsample, n_gru_layers, corr_levels,
corr_radius, mixed_precision, slow_fast_gru.  ``StereoArgs`` supplies them.
"""
from dataclasses import dataclass, field

import torch
import torch.nn as nn
import torch.nn.functional as F

from .corr import CorrBlock1D, coords_grid


@dataclass
class StereoArgs:
    hidden_dims: list = field(default_factory=lambda: [128] * 3)
    n_downsample: int = 2
    n_gru_layers: int = 3
    corr_levels: int = 4
    corr_radius: int = 4
    mixed_precision: bool = False
    slow_fast_gru: bool = False


def _make_norm(kind, channels, groups):
    """The four normalisation options of model.py:25-44 / :71-78."""
    table = {
        "group": lambda: nn.GroupNorm(num_groups=groups, num_channels=channels),
        "batch": lambda: nn.BatchNorm2d(channels),
        "instance": lambda: nn.InstanceNorm2d(channels),
    }
    return table.get(kind, nn.Sequential)()


class ResidualBlock(nn.Module):
    """Two 3x3 conv+norm+ReLU stages plus an (optionally projected) skip;
    note: no ReLU after the sum (model.py:63)."""

    def __init__(self, in_planes, planes, norm_fn="group", stride=1):
        super().__init__()
        self.conv1 = nn.Conv2d(in_planes, planes, kernel_size=3, padding=1, stride=stride)
        self.conv2 = nn.Conv2d(planes, planes, kernel_size=3, padding=1)
        self.relu = nn.ReLU(inplace=True)
        keeps_shape = stride == 1 and in_planes == planes
        self.norm1 = _make_norm(norm_fn, planes, planes // 8)
        self.norm2 = _make_norm(norm_fn, planes, planes // 8)
        if keeps_shape:
            self.downsample = None
        else:
            self.norm3 = _make_norm(norm_fn, planes, planes // 8)
            self.downsample = nn.Sequential(
                nn.Conv2d(in_planes, planes, kernel_size=1, stride=stride), self.norm3)

    def forward(self, x):
        branch = self.relu(self.norm1(self.conv1(x)))
        branch = self.relu(self.norm2(self.conv2(branch)))
        skip = x if self.downsample is None else self.downsample(x)
        return skip + branch


class BasicEncoder(nn.Module):
    """Shared feature/context encoder (model.py:65-161).  ``output_dim`` is a
    list of [d32, d16, d08] triples; one head per triple at each scale."""

    def __init__(self, output_dim=((128, 128, 128),), norm_fn="batch", dropout=0.0, downsample=3):
        super().__init__()
        self.norm_fn = norm_fn
        self.downsample = downsample
        self.norm1 = _make_norm(norm_fn, 64, 8)
        self.conv1 = nn.Conv2d(3, 64, kernel_size=7, stride=1 + (downsample > 2), padding=3)
        self.relu1 = nn.ReLU(inplace=True)
        self.in_planes = 64
        strides = (1, 1 + (downsample > 1), 1 + (downsample > 0), 2, 2)
        for idx, (width, stride) in enumerate(zip((64, 96, 128, 128, 128), strides), start=1):
            setattr(self, f"layer{idx}", self._stage(width, stride))
        heads08, heads16, heads32 = [], [], []
        for dims in output_dim:
            heads08.append(nn.Sequential(ResidualBlock(128, 128, norm_fn, stride=1),
                                         nn.Conv2d(128, dims[2], 3, padding=1)))
        for dims in output_dim:
            heads16.append(nn.Sequential(ResidualBlock(128, 128, norm_fn, stride=1),
                                         nn.Conv2d(128, dims[1], 3, padding=1)))
        for dims in output_dim:
            heads32.append(nn.Conv2d(128, dims[0], 3, padding=1))
        self.outputs08 = nn.ModuleList(heads08)
        self.outputs16 = nn.ModuleList(heads16)
        self.outputs32 = nn.ModuleList(heads32)
        self.dropout = nn.Dropout2d(p=dropout) if dropout > 0 else None  # never applied (:136-161)
        for mod in self.modules():
            if isinstance(mod, nn.Conv2d):
                nn.init.kaiming_normal_(mod.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(mod, (nn.BatchNorm2d, nn.InstanceNorm2d, nn.GroupNorm)):
                if mod.weight is not None:
                    nn.init.constant_(mod.weight, 1)
                if mod.bias is not None:
                    nn.init.constant_(mod.bias, 0)

    def _stage(self, width, stride):
        first = ResidualBlock(self.in_planes, width, self.norm_fn, stride=stride)
        second = ResidualBlock(width, width, self.norm_fn, stride=1)
        self.in_planes = width
        return nn.Sequential(first, second)

    def forward(self, x, dual_inp=False, num_layers=3):
        x = self.layer3(self.layer2(self.layer1(self.relu1(self.norm1(self.conv1(x))))))
        both = x
        if dual_inp:
            x = x[: x.shape[0] // 2]
        outs = [[head(x) for head in self.outputs08]]
        if num_layers >= 2:
            y = self.layer4(x)
            outs.append([head(y) for head in self.outputs16])
            if num_layers >= 3:
                outs.append([head(self.layer5(y)) for head in self.outputs32])
        if dual_inp:
            outs.append(both)
        return tuple(outs)


class ConvGRU(nn.Module):
    """Convolutional GRU with additive context biases cz, cr, cq (model.py:164-179)."""

    def __init__(self, hidden_dim, input_dim, kernel_size=3):
        super().__init__()
        pad = kernel_size // 2
        for gate in ("convz", "convr", "convq"):
            setattr(self, gate, nn.Conv2d(hidden_dim + input_dim, hidden_dim, kernel_size, padding=pad))

    def forward(self, h, cz, cr, cq, *x_list):
        x = torch.cat(x_list, dim=1)
        hx = torch.cat([h, x], dim=1)
        z = torch.sigmoid(self.convz(hx) + cz)
        r = torch.sigmoid(self.convr(hx) + cr)
        q = torch.tanh(self.convq(torch.cat([r * h, x], dim=1)) + cq)
        return (1 - z) * h + z * q


def pool2x(x):
    """3x3/2 average pool, zero padding counted (model.py:182-183)."""
    return F.avg_pool2d(x, 3, stride=2, padding=1)


def interp(x, dest):
    """Bilinear resize to dest's spatial size, align_corners=True (model.py:184-186)."""
    return F.interpolate(x, dest.shape[2:], mode="bilinear", align_corners=True)


class BasicMotionEncoder(nn.Module):
    """Fuses the lookup output (corr) with the current flow (model.py:192-213);
    convc1 is the consumer of the correlation path."""

    def __init__(self, args):
        super().__init__()
        self.args = args
        corr_channels = args.corr_levels * (2 * args.corr_radius + 1)
        self.convc1 = nn.Conv2d(corr_channels, 64, 1, padding=0)
        self.convc2 = nn.Conv2d(64, 64, 3, padding=1)
        self.convf1 = nn.Conv2d(2, 64, 7, padding=3)
        self.convf2 = nn.Conv2d(64, 64, 3, padding=1)
        self.conv = nn.Conv2d(128, 126, 3, padding=1)

    def forward(self, flow, corr, corr_is_convc1=False):
        # corr_is_convc1: ``corr`` already is relu(convc1(corr)) (the fused
        # lookup, CorrBlock1D.lookup_convc1)
        c1 = corr if corr_is_convc1 else F.relu(self.convc1(corr))
        c = F.relu(self.convc2(c1))
        f = F.relu(self.convf2(F.relu(self.convf1(flow))))
        return torch.cat([F.relu(self.conv(torch.cat([c, f], dim=1))), flow], dim=1)


class FlowHead(nn.Module):
    def __init__(self, input_dim=128, hidden_dim=256, output_dim=2):
        super().__init__()
        self.conv1 = nn.Conv2d(input_dim, hidden_dim, 3, padding=1)
        self.conv2 = nn.Conv2d(hidden_dim, output_dim, 3, padding=1)
        self.relu = nn.ReLU(inplace=True)

    def forward(self, x):
        return self.conv2(self.relu(self.conv1(x)))


class BasicMultiUpdateBlock(nn.Module):
    """Three-scale GRU update (model.py:226-265).  ``net`` is updated in place."""

    def __init__(self, args, hidden_dims=()):
        super().__init__()
        self.args = args
        self.encoder = BasicMotionEncoder(args)
        n = args.n_gru_layers
        self.gru08 = ConvGRU(hidden_dims[2], 128 + hidden_dims[1] * (n > 1))
        self.gru16 = ConvGRU(hidden_dims[1], hidden_dims[0] * (n == 3) + hidden_dims[2])
        self.gru32 = ConvGRU(hidden_dims[0], hidden_dims[1])
        self.flow_head = FlowHead(hidden_dims[2], hidden_dim=256, output_dim=2)
        factor = 2 ** self.args.n_downsample
        self.mask = nn.Sequential(nn.Conv2d(hidden_dims[2], 256, 3, padding=1), nn.ReLU(inplace=True),
                                  nn.Conv2d(256, (factor ** 2) * 9, 1, padding=0))

    def forward(self, net, inp, corr=None, flow=None, iter08=True, iter16=True, iter32=True,
                update=True, corr_is_convc1=False):
        n = self.args.n_gru_layers
        if iter32:
            net[2] = self.gru32(net[2], *inp[2], pool2x(net[1]))
        if iter16:
            extra = (interp(net[2], net[1]),) if n > 2 else ()
            net[1] = self.gru16(net[1], *inp[1], pool2x(net[0]), *extra)
        if iter08:
            motion = self.encoder(flow, corr, corr_is_convc1)
            extra = (interp(net[1], net[0]),) if n > 1 else ()
            net[0] = self.gru08(net[0], *inp[0], motion, *extra)
        if not update:
            return net
        return net, 0.25 * self.mask(net[0]), self.flow_head(net[0])


class RAFTStereo(nn.Module):
    """model.py:335-383 with the correlation block pluggable (``corr_block``)."""

    def __init__(self, args, corr_block=None, fuse_convc1=False, fuse_step=False):
        super().__init__()
        self.args = args
        context_dims = args.hidden_dims
        self.cnet = BasicEncoder(output_dim=[args.hidden_dims, context_dims], norm_fn="batch",
                                 downsample=args.n_downsample)
        self.update_block = BasicMultiUpdateBlock(self.args, hidden_dims=args.hidden_dims)
        self.context_zqr_convs = nn.ModuleList(
            [nn.Conv2d(context_dims[i], args.hidden_dims[i] * 3, 3, padding=1)
             for i in range(self.args.n_gru_layers)])
        self.conv2 = nn.Sequential(ResidualBlock(128, 128, "instance", stride=1),
                                   nn.Conv2d(128, 256, 3, padding=1))
        self.corr_block = corr_block or CorrBlock1D
        # run convc1 + ReLU inside the lookup launch
        self.fuse_convc1 = fuse_convc1
        # the loop's coords update and flow inside the
        # lookup launch (CorrBlock1D.lookup_step); exclusive with fuse_convc1
        self.fuse_step = fuse_step

    def initialize_flow(self, img):
        N, _, H, W = img.shape
        return (coords_grid(N, H, W).to(img.device), coords_grid(N, H, W).to(img.device))

    def _autocast(self):
        enabled = bool(self.args.mixed_precision)
        dtype = getattr(self.args, "autocast_dtype", torch.float16)
        dev = "cuda" if torch.cuda.is_available() else "cpu"
        return torch.autocast(dev, dtype=dtype, enabled=enabled and dev == "cuda")

    def features(self, image1, image2):
        """Encoders (stay on PyTorch ops): fmaps for the corr path + GRU state."""
        image1 = (2 * (image1 / 255.0) - 1.0).contiguous()
        image2 = (2 * (image2 / 255.0) - 1.0).contiguous()
        with self._autocast():
            *cnet_list, x = self.cnet(torch.cat((image1, image2), dim=0), dual_inp=True,
                                      num_layers=self.args.n_gru_layers)
            fmap1, fmap2 = self.conv2(x).split(dim=0, split_size=x.shape[0] // 2)
            net_list = [torch.tanh(pair[0]) for pair in cnet_list]
            inp_list = [torch.relu(pair[1]) for pair in cnet_list]
            inp_list = [list(conv(i).split(dim=1, split_size=conv.out_channels // 3))
                        for i, conv in zip(inp_list, self.context_zqr_convs)]
        return fmap1, fmap2, net_list, inp_list

    def forward(self, image1, image2, iters=12, flow_init=None, test_mode=False, upsample=False):
        """Per-iteration low-resolution flow (the reference's D8 tail), or with
        ``upsample=True`` the full-resolution x-flow of each iteration through
        the convex upsampler (``upsample.convex_upsample``)
        using the update block's mask (model.py:238-241, :264)."""
        a = self.args
        fmap1, fmap2, net_list, inp_list = self.features(image1, image2)
        corr_fn = self.corr_block(fmap1, fmap2, radius=a.corr_radius, num_levels=a.corr_levels)
        coords0, coords1 = self.initialize_flow(net_list[0])
        if flow_init is not None:
            coords1 = coords1 + flow_init
        step = self.fuse_step and hasattr(corr_fn, "lookup_step")
        fused = self.fuse_convc1 and not step and hasattr(corr_fn, "lookup_convc1")
        enc = self.update_block.encoder
        predictions = []
        masks = []
        delta = None
        for itr in range(iters):
            coords1 = coords1.detach()
            if step:
                # previous iteration's coords update + flow + lookup, one launch;
                # its flow is that iteration's prediction (coords1 - coords0)
                corr, coords1, flow = corr_fn.lookup_step(coords1, delta)
                if itr > 0:
                    predictions.append(flow)
            else:
                if fused:                               # lookup + convc1 + ReLU, one launch
                    corr = corr_fn.lookup_convc1(coords1, enc.convc1.weight, enc.convc1.bias)
                else:
                    corr = corr_fn(coords1)             # the hot path, every iteration
                flow = coords1 - coords0
            with self._autocast():
                if a.n_gru_layers == 3 and a.slow_fast_gru:
                    net_list = self.update_block(net_list, inp_list, iter32=True, iter16=False,
                                                 iter08=False, update=False)
                if a.n_gru_layers >= 2 and a.slow_fast_gru:
                    net_list = self.update_block(net_list, inp_list, iter32=a.n_gru_layers == 3,
                                                 iter16=True, iter08=False, update=False)
                net_list, up_mask, delta_flow = self.update_block(
                    net_list, inp_list, corr, flow, iter32=a.n_gru_layers == 3,
                    iter16=a.n_gru_layers >= 2, corr_is_convc1=fused)
            if upsample:
                masks.append(up_mask)
            if step:
                delta = delta_flow.float()              # applied by the next launch
                continue
            delta_flow[:, 1] = 0.0                       # D8 tail (see module docstring)
            coords1 = coords1 + delta_flow.float()
            predictions.append(coords1 - coords0)
        if step and delta is not None:                   # the last iteration's update
            delta[:, 1] = 0.0
            coords1 = coords1 + delta
            predictions.append(coords1 - coords0)
        if upsample:
            from .upsample import convex_upsample
            f = 2 ** a.n_downsample
            predictions = [convex_upsample(p[:, :1], m, f) for p, m in zip(predictions, masks)]
        return predictions
