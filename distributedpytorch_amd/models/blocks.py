"""Block-level execution API shared by every strategy and both backends.

A UNet of depth D is executed as a chain of ``2D+2`` blocks:

    idx 0..D-1   enc_l   : x -> (skip_l, pooled)          (conv_block + maxpool, unet_parts.py:28-41)
    idx D        mid     : x -> x                          (unet_model.py:57)
    idx D+1..2D  dec_i   : (x, skip_{D+1-i}) -> x          (deconv + crop + cat + conv_block, :56-77)
    idx 2D+1     head    : x -> loss partial sums / probs  (segmap + sigmoid [+ fused loss])

Backends implement ``enc/mid/dec/head_partials/head_probs`` (:class:`TorchBlocks` here, the HIP
kernels in :mod:`.hip_unet`).  :func:`run_segment` executes any contiguous block range on a dict of
named tensors - ``x`` plus the skips ``skip{l}`` still to be consumed - which is exactly what a
pipeline stage sends/receives; :func:`partition` balances block ranges over stages by FLOPs.

Cuts may also fall INSIDE a DoubleConv block (a pipeline stage boundary between its two convs, for
the time-balanced partitions of ``parallel/schedule.py``): a cut ``b + 0.5`` splits block ``b`` into
its part ``a`` (encoder / mid: the first conv; decoder: transposed conv + crop + concat + first conv)
and part ``b`` (the second conv; encoder: + max-pool), and the tensor crossing it is ``x`` = the first
conv's output.  Backends provide ``enc_a/enc_b/mid_a/mid_b/dec_a/dec_b`` for those halves; a block
whose both halves run in one segment still runs as ONE fused block.
"""
from __future__ import annotations

import contextlib
from typing import Dict, List, Sequence, Tuple

import torch
import torch.nn.functional as F

from ..utils.tracing import trace_range
from .unet import UNet, UNetConfig


def n_blocks(depth: int) -> int:
    return 2 * depth + 2


def block_kind(idx: int, depth: int) -> Tuple[str, int]:
    if idx < depth:
        return "enc", idx
    if idx == depth:
        return "mid", 0
    if idx <= 2 * depth:
        return "dec", idx - depth - 1
    return "head", 0


def skip_name(level: int) -> str:
    return f"skip{level}"


def produced(idx: int, depth: int) -> List[str]:
    kind, i = block_kind(idx, depth)
    return [skip_name(i)] if kind == "enc" else []


def consumed(idx: int, depth: int) -> List[str]:
    kind, i = block_kind(idx, depth)
    return [skip_name(depth - 1 - i)] if kind == "dec" else []


def boundary_names(cut: float, depth: int) -> List[str]:
    """Tensors crossing a cut placed before block ``cut`` (or inside block ``cut - 0.5``): ``x`` + the
    skips produced before it (at the END of encoder block l) and consumed after it (at the START of
    their decoder block, by its part a)."""
    names = ["x"]
    for lvl in range(depth):
        cons_idx = depth + 1 + (depth - 1 - lvl)
        if lvl + 1 <= cut <= cons_idx:
            names.append(skip_name(lvl))
    return names


def splittable(idx: int, depth: int) -> bool:
    """Blocks that may be cut between their two convs (all but the head)."""
    return 0 <= idx < n_blocks(depth) - 1


def segment_units(start: float, end: float, depth: int) -> List[Tuple[int, str]]:
    """(block, part) units of the segment [start, end): part ``full`` for whole blocks, ``a`` / ``b``
    for the halves at a fractional start / end (a cut ``b + 0.5`` lies inside block ``b``)."""
    for c in (start, end):
        f = c - int(c)
        assert f in (0.0, 0.5) and (f == 0.0 or splittable(int(c), depth)), f"invalid cut {c}"
    out = []
    idx = int(start)
    while idx < end:
        lo = max(start, idx)
        hi = min(end, idx + 1)
        if lo == idx and hi == idx + 1:
            out.append((idx, "full"))
        elif lo == idx:
            out.append((idx, "a"))
        else:
            assert hi == idx + 1, (start, end)
            out.append((idx, "b"))
        idx += 1
    return out


class TorchBlocks:
    """Stock-PyTorch block implementations (bf16 autocast + channels_last on GPU)."""

    name = "torch"

    def __init__(self, model: UNet, dtype: str = "bf16", channels_last: bool = True):
        self.model = model
        dev = next(model.parameters()).device
        self.autocast = dtype == "bf16" and dev.type == "cuda"
        # activations only: parameters must stay views of the flat fp32 buffer (optim.py)
        self.channels_last = channels_last and dev.type == "cuda"

    def ctx(self):
        return torch.autocast("cuda", dtype=torch.bfloat16) if self.autocast else contextlib.nullcontext()

    def prep(self, x):
        return x.contiguous(memory_format=torch.channels_last) if self.channels_last else x

    def enc(self, l: int, x):
        with self.ctx():
            s = self.model.encoder.blocks()[l](x)
            return s, F.max_pool2d(s, 2, 2)

    def mid(self, x):
        with self.ctx():
            return self.model.mid(x)

    def dec(self, i: int, x, skip):
        with self.ctx():
            return self.model.decoder.level(i, x, skip)

    # halves of a block cut between its two convs (pipeline stage boundaries inside a DoubleConv)
    def enc_a(self, l: int, x):
        with self.ctx():
            return self.model.encoder.blocks()[l].half(x, "a")

    def enc_b(self, l: int, x):
        with self.ctx():
            s = self.model.encoder.blocks()[l].half(x, "b")
            return s, F.max_pool2d(s, 2, 2)

    def mid_a(self, x):
        with self.ctx():
            return self.model.mid.half(x, "a")

    def mid_b(self, x):
        with self.ctx():
            return self.model.mid.half(x, "b")

    def dec_a(self, i: int, x, skip):
        with self.ctx():
            return self.model.decoder.level(i, x, skip, part="a")

    def dec_b(self, i: int, x):
        with self.ctx():
            return self.model.decoder.blocks()[i].half(x, "b")

    def head_logits(self, x):
        with self.ctx():
            return self.model.segmap(x).float()

    def head_probs(self, x):
        return torch.sigmoid(self.head_logits(x))

    def head_partials(self, x, t):
        from ..compute import loss_partials_from_probs
        return loss_partials_from_probs(self.head_probs(x), t)


def run_segment(blocks, start: int, end: int, depth: int, env: Dict[str, torch.Tensor],
                target: torch.Tensor = None, want: str = "partials", emit=None) -> Dict[str, torch.Tensor]:
    """Run blocks ``[start, end)`` on ``env`` (mutated copy returned).

    If the head block is included the result holds ``partials`` (training, needs ``target``) or
    ``probs`` (inference) instead of ``x``.  ``emit(name, tensor)`` is called as soon as an encoder
    level's skip exists (a pipeline stage starts sending it while its deeper levels compute).
    """
    env = dict(env)
    if want == "partials" and end == n_blocks(depth) and hasattr(blocks, "expect_target"):
        blocks.expect_target(target)      # lets a backend fuse the head into the last decoder conv
    if start == 0:
        env["x"] = blocks.prep(env["x"])
    units = segment_units(start, end, depth)
    if hasattr(blocks, "skip_z_levels"):
        # a backend may keep a skip in an internal form (models/hip_unet.py: a BatchNorm's input z, normalised
        # by its consumer on load) only when that consumer runs inside THIS call: the hand-over is keyed in the
        # engine and reset by prep(), so a skip consumed by another segment (a pipeline's other stage, the
        # second segment of a mirrored placement, the next microbatch's prep in between) must stay plain
        enc_here = {i for idx, part in units for k, i in [block_kind(idx, depth)] if k == "enc" and part != "a"}
        dec_here = {depth - 1 - i for idx, part in units for k, i in [block_kind(idx, depth)]
                    if k == "dec" and part != "b"}
        blocks.skip_z_levels = (enc_here & dec_here) - set(getattr(blocks, "dense_skips", ()))
    for u, (idx, part) in enumerate(units):
        kind, i = block_kind(idx, depth)
        if kind == "dec" and hasattr(blocks, "next_dec_local"):
            # the next unit is a whole decoder block of this same segment: a backend may hand it its input in
            # an internal form (models/hip_unet.py: a BatchNorm's input z, normalised on load)
            nxt = units[u + 1] if u + 1 < len(units) else None
            blocks.next_dec_local = (part == "full" and nxt is not None and nxt[1] == "full"
                                     and block_kind(nxt[0], depth)[0] == "dec")
        tag = (f"{kind}{i}" if kind in ("enc", "dec") else kind) + ("" if part == "full" else part)
        with trace_range(tag):
            if kind == "enc":
                if part == "a":
                    env["x"] = blocks.enc_a(i, env["x"])
                else:
                    s, env["x"] = blocks.enc(i, env["x"]) if part == "full" else blocks.enc_b(i, env["x"])
                    env[skip_name(i)] = s
                    if emit is not None:
                        emit(skip_name(i), s)
            elif kind == "mid":
                env["x"] = {"full": blocks.mid, "a": blocks.mid_a, "b": blocks.mid_b}[part](env["x"])
            elif kind == "dec":
                if part == "b":
                    env["x"] = blocks.dec_b(i, env["x"])
                else:
                    name = skip_name(depth - 1 - i)
                    fn = blocks.dec if part == "full" else blocks.dec_a
                    env["x"] = fn(i, env["x"], env.pop(name))
            else:
                x = env.pop("x")
                if want == "partials":
                    env["partials"] = blocks.head_partials(x, target)
                else:
                    env["probs"] = blocks.head_probs(x)
    return env


# ------------------------------------------------------------------------------------ partitioner
def block_costs(cfg: UNetConfig, h: int, w: int) -> List[float]:
    """Forward FLOPs per block per image (training cost is ~3x, same proportions)."""
    costs = []
    H, W, cin = h, w, cfg.in_channels
    for wd in cfg.widths:
        costs.append(2 * H * W * 9 * (cin * wd + wd * wd))
        H, W, cin = H // 2, W // 2, wd
    costs.append(2 * H * W * 9 * (cin * cfg.mid_width + cfg.mid_width ** 2))
    cin = cfg.mid_width
    for wd in reversed(cfg.widths):
        c = 2 * H * W * cin * wd * 4
        H, W = H * 2, W * 2
        costs.append(c + 2 * H * W * 9 * (3 * wd * wd))
        cin = wd
    costs.append(2 * H * W * cfg.base * (cfg.out_channels + 8))  # head + fused loss (memory-bound)
    return costs


def partition(cfg: UNetConfig, stages: int, h: int = 512, w: int = 512, mode: str = "balanced") -> List[int]:
    """Return ``stages+1`` cut points over ``2D+2`` blocks.

    ``mode='reference'`` with 2 stages reproduces the reference split (encoder+mid | decoder+head,
    unet_model.py:14-20).  ``balanced`` minimises the max stage FLOPs with contiguous ranges
    (exact DP over the <= 14 blocks).
    """
    nb = n_blocks(cfg.depth)
    if stages < 1 or stages > nb:
        raise ValueError(f"stages must be in [1, {nb}] for depth {cfg.depth}")
    if mode == "reference" and stages == 2:
        return [0, cfg.depth + 1, nb]
    c = block_costs(cfg, h, w)
    pre = [0.0]
    for v in c:
        pre.append(pre[-1] + v)
    INF = float("inf")
    best = [[INF] * (nb + 1) for _ in range(stages + 1)]
    arg = [[0] * (nb + 1) for _ in range(stages + 1)]
    best[0][0] = 0.0
    for s in range(1, stages + 1):
        for j in range(s, nb + 1):
            for i in range(s - 1, j):
                v = max(best[s - 1][i], pre[j] - pre[i])
                if v < best[s][j]:
                    best[s][j], arg[s][j] = v, i
    cuts = [nb]
    j = nb
    for s in range(stages, 0, -1):
        j = arg[s][j]
        cuts.append(j)
    return list(reversed(cuts))
