"""UNet family with the reference's parameter names and semantics.

Parity target: reference ``model/unet_parts.py:6-77`` and ``model/unet_model.py:4-62``.

* ``ConvBlock`` == reference ``conv_block`` (unet_parts.py:6-17): two 3x3 pad-1 convs with bias,
  each followed by ReLU, no BatchNorm by default.  State-dict keys ``conv_block.{0,2}.*``.
* ``Encoder`` == unet_parts.py:19-41: ``conv1..convD`` + one shared 2x2 max-pool; returns
  ``(pooled, skip_D, ..., skip_1)`` (deepest skip first, unet_parts.py:41).
* ``Decoder`` == unet_parts.py:43-77: per level ConvTranspose2d(k2,s2) -> center-crop of the
  skip -> ``cat((skip, up), 1)`` (skip first) -> ConvBlock.
* ``UNet`` == unet_model.py:4-21: encoder -> mid -> decoder -> 1x1 ``segmap`` -> sigmoid.

The default configuration (in=3, out=1, base=32, depth=4, no BN, transposed-conv up path)
reproduces the reference's 46 tensors / 7,760,097 parameters and its exact key names,
so checkpoints round-trip with the reference.  Variants (base width, depth, BatchNorm, bilinear
up-sampling, the ``xl`` preset used for the 1024^2 pipeline config) are additions.

This module is the *reference-semantics* implementation on stock torch ops (CPU and GPU).  The
MI355X fast path is :mod:`distributedpytorch_amd.models.engine`, which runs the same parameters
through hand-written HIP kernels in NHWC bf16 with an explicit backward schedule.
"""
from __future__ import annotations

from dataclasses import dataclass, asdict
from typing import List, Sequence, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F


@dataclass(frozen=True)
class UNetConfig:
    in_channels: int = 3
    out_channels: int = 1
    base: int = 32
    depth: int = 4
    batchnorm: bool = False
    bilinear: bool = False

    @property
    def widths(self) -> List[int]:
        return [self.base * (2 ** i) for i in range(self.depth)]

    @property
    def mid_width(self) -> int:
        return self.base * (2 ** self.depth)

    def to_dict(self):
        return asdict(self)


PRESETS = {
    # reference architecture (model/modelsummary.txt:1-72)
    "unet": UNetConfig(),
    # larger model used by the 1024x1024 8-stage pipeline config (BASELINE.json configs[4])
    "unet-xl": UNetConfig(base=64, depth=5),
    # milesial-style variant listed in model/modelsummary.txt:153-247 (BN, base 64)
    "unet-bn64": UNetConfig(base=64, batchnorm=True),
    # north-star block variants at the reference width: DoubleConv = Conv2d+BN+ReLU, bilinear Up
    "unet-bn": UNetConfig(batchnorm=True),
    "unet-bilinear": UNetConfig(bilinear=True),
    "unet-bn-bilinear": UNetConfig(batchnorm=True, bilinear=True),
    # tiny configs for fast CPU tests
    "unet-tiny": UNetConfig(base=8, depth=2),
    "unet-tiny-bn": UNetConfig(base=8, depth=2, batchnorm=True, bilinear=True),
    # reference depth at a tiny width: up to 10 pipeline stages in CPU tests
    "unet-tiny4": UNetConfig(base=8, depth=4),
}


def center_crop(t: torch.Tensor, h: int, w: int) -> torch.Tensor:
    """torchvision ``CenterCrop((h, w))`` semantics for h<=H, w<=W (unet_parts.py:58)."""
    H, W = t.shape[-2], t.shape[-1]
    if H == h and W == w:
        return t
    top = int(round((H - h) / 2.0))
    left = int(round((W - w) / 2.0))
    return t[..., top:top + h, left:left + w]


class ConvBlock(nn.Module):
    """conv3x3(+BN)+ReLU, twice.  Keys ``conv_block.{0,2}`` (no BN) / ``{0,1,3,4}`` (BN)."""

    def __init__(self, insize: int, outsize: int, batchnorm: bool = False):
        super().__init__()
        layers: List[nn.Module] = []
        for cin in (insize, outsize):
            layers.append(nn.Conv2d(cin, outsize, kernel_size=3, padding=1))
            if batchnorm:
                layers.append(nn.BatchNorm2d(outsize))
            layers.append(nn.ReLU())
        self.conv_block = nn.Sequential(*layers)
        self.batchnorm = batchnorm

    def convs(self) -> List[nn.Conv2d]:
        return [m for m in self.conv_block if isinstance(m, nn.Conv2d)]

    def bns(self) -> List[nn.BatchNorm2d]:
        return [m for m in self.conv_block if isinstance(m, nn.BatchNorm2d)]

    def forward(self, x):
        return self.conv_block(x)

    def half(self, x, part: str):
        """Part ``a`` (first conv [+BN] + ReLU) or ``b`` (the second) -- a pipeline cut between the two."""
        n = len(self.conv_block) // 2
        return self.conv_block[:n](x) if part == "a" else self.conv_block[n:](x)


class Encoder(nn.Module):
    def __init__(self, cfg: UNetConfig):
        super().__init__()
        cin = cfg.in_channels
        for i, w in enumerate(cfg.widths):
            setattr(self, f"conv{i + 1}", ConvBlock(cin, w, cfg.batchnorm))
            cin = w
        self.depth = cfg.depth
        self.maxpool = nn.MaxPool2d(2, 2)

    def blocks(self) -> List[ConvBlock]:
        return [getattr(self, f"conv{i + 1}") for i in range(self.depth)]

    def forward(self, x) -> Tuple[torch.Tensor, ...]:
        skips = []
        for blk in self.blocks():
            x = blk(x)
            skips.append(x)
            x = self.maxpool(x)
        return (x, *reversed(skips))


class Up(nn.Module):
    """Bilinear x2 up-sampling followed by a 1x1 conv halving the channels (variant only)."""

    def __init__(self, cin: int, cout: int):
        super().__init__()
        self.proj = nn.Conv2d(cin, cout, kernel_size=1)

    def forward(self, x):
        return self.proj(F.interpolate(x, scale_factor=2, mode="bilinear", align_corners=False))


class Decoder(nn.Module):
    def __init__(self, cfg: UNetConfig):
        super().__init__()
        widths = list(reversed(cfg.widths))  # 256,128,64,32
        cin = cfg.mid_width
        for i, w in enumerate(widths):
            setattr(self, f"conv{i + 1}", ConvBlock(2 * w, w, cfg.batchnorm))
        for i, w in enumerate(widths):
            up = Up(cin, w) if cfg.bilinear else nn.ConvTranspose2d(cin, w, 2, 2)
            setattr(self, f"deconv{i + 1}", up)
            cin = w
        self.depth = cfg.depth

    def blocks(self) -> List[ConvBlock]:
        return [getattr(self, f"conv{i + 1}") for i in range(self.depth)]

    def ups(self) -> List[nn.Module]:
        return [getattr(self, f"deconv{i + 1}") for i in range(self.depth)]

    def level(self, i: int, x, skip, part: str = "full"):
        out = self.ups()[i](x)
        skip = center_crop(skip, out.shape[2], out.shape[3])
        cat = torch.cat((skip, out), dim=1)
        return self.blocks()[i](cat) if part == "full" else self.blocks()[i].half(cat, "a")

    def forward(self, x, *skips):
        for i, skip in enumerate(skips):
            x = self.level(i, x, skip)
        return x


class UNet(nn.Module):
    """Reference-parity UNet (unet_model.py:4-62).  ``forward(x[B,C,H,W]) -> probs[B,1,H,W]``.

    ``UNet(pipe=True)`` keeps the reference constructor (unet_model.py:5,14-21): encoder + mid on
    the first device, decoder + head on the second (``cuda:0``/``cuda:1``; both stages on one device
    when the box has a single GPU, CPU without one), and ``forward`` runs the 2-microbatch
    pipelined schedule (unet_model.py:24-53) through
    :class:`distributedpytorch_amd.parallel.pipeline.GPipeLocal`, returning the probabilities on
    the first device like the reference.  ``train.py -t MP`` uses the pipeline strategies directly.
    """

    def __init__(self, cfg: UNetConfig | None = None, pipe: bool = False, devices=None, microbatches: int = 2,
                 **kw):
        super().__init__()
        if isinstance(cfg, bool):          # UNet(True): the reference's positional ``pipe``
            cfg, pipe = None, cfg
        cfg = cfg or UNetConfig(**kw)
        self.cfg = cfg
        self.encoder = Encoder(cfg)
        self.mid = ConvBlock(cfg.widths[-1], cfg.mid_width, cfg.batchnorm)
        self.decoder = Decoder(cfg)
        self.segmap = nn.Conv2d(cfg.base, cfg.out_channels, 1)
        self.sigmoid = nn.Sigmoid()
        self.pipe = bool(pipe)
        self._pipe = None
        if self.pipe:
            from ..parallel.pipeline import GPipeLocal
            if devices is None:
                n = torch.cuda.device_count() if torch.cuda.is_available() else 0
                devices = ["cuda:0", "cuda:1"] if n >= 2 else (["cuda:0", "cuda:0"] if n == 1 else ["cpu", "cpu"])
            # the pipeline is not a submodule: state_dict keys stay the reference's
            object.__setattr__(self, "_pipe", GPipeLocal(self, devices, microbatches, backend="torch",
                                                         dtype="fp32", mode="reference"))

    def logits(self, x):
        x, *skips = self.encoder(x)
        x = self.mid(x)
        x = self.decoder(x, *skips)
        return self.segmap(x)

    def forward(self, x):
        if self._pipe is not None:
            return self._pipe.forward_probs(x)
        return self.sigmoid(self.logits(x))

    # ---- introspection used by the engine / pipeline partitioner ----
    def conv_blocks(self) -> List[ConvBlock]:
        return self.encoder.blocks() + [self.mid] + self.decoder.blocks()


def backward_param_order(model: "UNet") -> List[str]:
    """Parameter names in the order their gradients become final during backward (head first, then
    each decoder level conv2 -> conv1 -> up-conv, the bottleneck, the encoder deepest first).

    :class:`..optim.FlatParameterSpace` lays the flat gradient buffer out in this order, so the
    data-parallel buckets (contiguous slices) complete one after another while the backward is
    still running; with plain reversed-registration order the decoder's up-convs (registered
    after all decoder convs) would hold the first buckets back until the decoder had finished."""
    names = [n for n, _ in model.named_parameters()]
    order = [n for n in names if n.startswith("segmap.")]
    for i in range(model.cfg.depth, 0, -1):
        blk = [n for n in names if n.startswith(f"decoder.conv{i}.")]
        order += list(reversed(blk))                       # conv_block.2 before conv_block.0 (+BN)
        order += [n for n in names if n.startswith(f"decoder.deconv{i}.")]
    order += list(reversed([n for n in names if n.startswith("mid.")]))
    for i in range(model.cfg.depth, 0, -1):
        order += list(reversed([n for n in names if n.startswith(f"encoder.conv{i}.")]))
    rest = [n for n in names if n not in set(order)]
    return order + rest


def build_model(name: str = "unet", **overrides) -> UNet:
    cfg = PRESETS[name]
    if overrides:
        cfg = UNetConfig(**{**cfg.to_dict(), **overrides})
    return UNet(cfg)


def count_params(model: nn.Module) -> int:
    return sum(p.numel() for p in model.parameters())


def forward_flops(cfg: UNetConfig, h: int, w: int) -> float:
    """Forward FLOPs per image (2*MACs) over conv / deconv layers (96.6 GF @ 512^2)."""
    fl = 0.0
    H, W, cin = h, w, cfg.in_channels
    for wd in cfg.widths:
        fl += 2 * H * W * 9 * (cin * wd + wd * wd)
        H, W, cin = H // 2, W // 2, wd
    fl += 2 * H * W * 9 * (cin * cfg.mid_width + cfg.mid_width ** 2)
    cin = cfg.mid_width
    for wd in reversed(cfg.widths):
        fl += 2 * H * W * cin * wd * 4  # deconv: every input pixel -> 2x2 outputs
        H, W = H * 2, W * 2
        fl += 2 * H * W * 9 * (2 * wd * wd + wd * wd)
        cin = wd
    fl += 2 * H * W * cfg.base * cfg.out_channels
    return fl


if __name__ == "__main__":   # reference smoke self-test (model/unet_model.py:64-67)
    import sys

    name = sys.argv[1] if len(sys.argv) > 1 else "unet"
    m = build_model(name)
    with torch.no_grad():
        print(m(torch.rand(1, 3, 640, 960)).shape)
