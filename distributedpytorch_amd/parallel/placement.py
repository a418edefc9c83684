"""Pipeline stage placements: which block ranges (segments) of the UNet chain each stage owns.

The reference pipeline (``model/unet_model.py:14-53``) cuts the UNet once, encoder+mid on cuda:0 and
decoder+head on cuda:1, so the bottleneck AND all four skips cross the cut every microbatch (SURVEY
§2.6 N10: 145 MiB per image at 640x960 fp32; 31 MiB per image at 512^2 bf16).  A contiguous GPipe
partition of a UNet always pays that: every skip whose encoder level and decoder level land on
different stages crosses the cut.

A :class:`Placement` cuts the block chain (``models/blocks.py``: enc_0..enc_{D-1}, mid, dec_0..dec_{D-1},
head; cut positions may be ``b + 0.5`` = between the two convs of block b) into K segments and gives
every segment an owner stage.  Two families:

* ``contiguous``: K = S, segment k on stage k (the reference cut is ``[0, D+1, 2D+2]``);
* ``v`` (mirrored): K = 2S-1, segment k on stage ``min(k, 2S-2-k)``: stage s owns the encoder levels on
  the way down AND the mirrored decoder levels on the way up, so the forward runs 0 -> S-1 -> 0 and a
  skip whose encoder and decoder level share a stage never leaves its GPU.  At two stages GPU0 = {enc0,
  enc1, dec2, dec3, head} sends the pooled enc1 output down (2 MiB/img at 512^2 bf16) and receives the
  dec1 output back (4 MiB/img) instead of 31 MiB; every stage has two segments (except the bottom one),
  which halves the fill / drain bubble; the images and the loss both live on stage 0.

:func:`seg_io` gives the tensors every segment receives and sends (``x`` along the chain, each skip
straight from its producer segment to its consumer segment: one xGMI hop on the fully connected
MI355X mesh, never relayed).  :func:`stage_orders` is the static per-stage op order the engine
(:class:`.pipeline.GPipeDist`) issues and the schedule model (:mod:`.schedule`) simulates.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

from ..models.blocks import block_kind, n_blocks, skip_name, splittable


def _pos(v) -> float:
    f = float(v)
    return int(f) if f == int(f) else f


@dataclass(frozen=True)
class Placement:
    cuts: Tuple[float, ...]        # K+1 block positions: 0 = cuts[0] < ... < cuts[K] = n_blocks
    owner: Tuple[int, ...]         # K segment owners (stages 0..S-1)

    def __post_init__(self):
        object.__setattr__(self, "cuts", tuple(_pos(c) for c in self.cuts))
        object.__setattr__(self, "owner", tuple(int(o) for o in self.owner))
        c, o = self.cuts, self.owner
        if len(c) != len(o) + 1 or c[0] != 0 or any(b <= a for a, b in zip(c, c[1:])):
            raise ValueError(f"bad placement cuts {c} for owners {o}")
        if any(2 * x != int(2 * x) for x in c):
            raise ValueError(f"cuts must be whole or half blocks: {c}")
        if sorted(set(o)) != list(range(max(o) + 1)):
            raise ValueError(f"every stage 0..S-1 must own a segment: {o}")
        if any(a == b for a, b in zip(o, o[1:])):
            raise ValueError(f"adjacent segments on one stage must be merged: {o}")

    # ------------------------------------------------------------------ construction
    @staticmethod
    def contiguous(cuts: Sequence[float]) -> "Placement":
        return Placement(tuple(cuts), tuple(range(len(cuts) - 1)))

    @staticmethod
    def mirrored(cuts: Sequence[float]) -> "Placement":
        """V placement from its 2S cut positions (2S-1 segments): segment k on stage min(k, 2S-2-k)."""
        K = len(cuts) - 1
        if K % 2 != 1:
            raise ValueError(f"a mirrored placement has an odd number of segments (2S-1), got {K}")
        S = (K + 1) // 2
        return Placement(tuple(cuts), tuple(min(k, 2 * S - 2 - k) for k in range(K)))

    @staticmethod
    def from_plan(p: dict) -> "Placement":
        if p.get("owner") is not None:
            return Placement(tuple(p["cuts"]), tuple(p["owner"]))
        if p.get("placement", "contiguous") == "v":
            return Placement.mirrored(p["cuts"])
        return Placement.contiguous(p["cuts"])

    def to_plan(self) -> dict:
        return {"cuts": list(self.cuts), "owner": list(self.owner), "placement": self.kind}

    def validate(self, depth: int) -> "Placement":
        """Check the placement against a UNet of ``depth``: ends at the head, no cut inside it."""
        nb = n_blocks(depth)
        if self.cuts[-1] != nb:
            raise ValueError(f"placement ends at {self.cuts[-1]}, the model has {nb} blocks")
        for c in self.cuts[1:-1]:
            if c != int(c) and not splittable(int(c), depth):
                raise ValueError(f"cut {c} falls inside block {int(c)}, which has no halves")
        return self

    # ------------------------------------------------------------------ queries
    @property
    def K(self) -> int:
        return len(self.owner)

    @property
    def S(self) -> int:
        return max(self.owner) + 1

    @property
    def kind(self) -> str:
        if self.owner == tuple(range(self.K)):
            return "contiguous"
        S = self.S
        if self.K == 2 * S - 1 and self.owner == tuple(min(k, 2 * S - 2 - k) for k in range(self.K)):
            return "v"
        return "custom"

    def seg_range(self, j: int) -> Tuple[float, float]:
        return self.cuts[j], self.cuts[j + 1]

    def segments(self, s: int) -> List[int]:
        return [j for j, o in enumerate(self.owner) if o == s]

    def seg_of(self, pos: float) -> int:
        """Segment containing block position ``pos`` (``b + 0.5``: part b of block b)."""
        for j in range(self.K):
            if self.cuts[j] <= pos < self.cuts[j + 1]:
                return j
        raise ValueError(pos)

    @property
    def head_seg(self) -> int:
        return self.K - 1

    def __str__(self):
        return f"{self.kind}{list(self.cuts)}@{list(self.owner)}"


def seg_io(pl: Placement, depth: int):
    """Per segment: ``ins[j]`` = [(name, producer segment)], ``outs[j]`` = [(name, consumer segment)].

    ``x`` flows along the chain (segment j-1 -> j); the skip of encoder level l leaves the segment
    holding part b of enc_l and enters the segment holding part a of its decoder block, directly.  A
    skip produced and consumed inside one segment does not appear."""
    K = pl.K
    ins: List[List[Tuple[str, int]]] = [[] for _ in range(K)]
    outs: List[List[Tuple[str, int]]] = [[] for _ in range(K)]
    for j in range(1, K):
        ins[j].append(("x", j - 1))
        outs[j - 1].append(("x", j))
    for lvl in range(depth):
        p = pl.seg_of(lvl + 0.5)
        c = pl.seg_of(depth + 1 + (depth - 1 - lvl))
        if p != c:
            ins[c].append((skip_name(lvl), p))
            outs[p].append((skip_name(lvl), c))
    return ins, outs


def stage_io(pl: Placement, depth: int):
    """Stage-level view of :func:`seg_io`: ``recv[s]`` = [(name, src stage)], ``send[s]`` =
    [(name, dst stage)] over the tensors that change STAGE (segments of one stage hand over locally)."""
    ins, outs = seg_io(pl, depth)
    recv = [[] for _ in range(pl.S)]
    send = [[] for _ in range(pl.S)]
    for j in range(pl.K):
        for name, p in ins[j]:
            if pl.owner[p] != pl.owner[j]:
                recv[pl.owner[j]].append((name, pl.owner[p]))
        for name, c in outs[j]:
            if pl.owner[c] != pl.owner[j]:
                send[pl.owner[j]].append((name, pl.owner[c]))
    return recv, send


def channel_members(pl: Placement, depth: int) -> List[List[int]]:
    """Members of each segment's communicator: its owner (the only rank that ever SENDS on it:
    activations to the stages of its consumer segments, gradients to the stages of its producer
    segments) plus those stages.  One sender per communicator means a receive pre-posted on one RCCL
    stream can never hold back a send of the same rank (``tests/test_pipeline_p2p_order.py``)."""
    ins, outs = seg_io(pl, depth)
    out = []
    for j in range(pl.K):
        m = {pl.owner[j]}
        m |= {pl.owner[c] for _, c in outs[j]}
        m |= {pl.owner[p] for _, p in ins[j]}
        out.append(sorted(m))
    return out


def remote_groups(pl: Placement, edges: Sequence[Tuple[str, int]], me: int) -> Dict[int, List[Tuple[str, int]]]:
    """Edges (name, other segment) grouped by the OTHER segment's stage, leaving out this stage;
    names sorted so both ends of a message list its tensors in one order."""
    g: Dict[int, List[Tuple[str, int]]] = {}
    for name, other in edges:
        st = pl.owner[other]
        if st != me:
            g.setdefault(st, []).append((name, other))
    return {st: sorted(v) for st, v in sorted(g.items())}


# ------------------------------------------------------------------------------------ op order
def stage_orders(pl: Placement, depth: int, M: int, fwd_ms: Optional[Sequence[float]] = None,
                 bwd_ms: Optional[Sequence[float]] = None, policy: str = "further") -> List[Dict[str, List[int]]]:
    """Static op order of every stage: ``{"fwd": [segment, ...], "bwd": [segment, ...]}`` (segment j's
    microbatches run in order 0..M-1 forward and M-1..0 backward, so the segment sequence fixes the
    order).  Obtained by list-scheduling the step with per-segment costs (``fwd_ms`` / ``bwd_ms``;
    default: equal costs per segment); :func:`.schedule.simulate_placement` with ``orders=None``
    is the same scheduler, so a plan's simulated timeline is exactly the order the engine issues."""
    from .schedule import SegCost, simulate_placement
    f = list(fwd_ms) if fwd_ms is not None else [1.0] * pl.K
    b = list(bwd_ms) if bwd_ms is not None else [2.0 * v for v in f]
    costs = [SegCost(f[j], b[j]) for j in range(pl.K)]
    tl = simulate_placement(pl, depth, M, costs, policy=policy)
    return tl.orders


def flop_orders(pl: Placement, cfg, M: int, h: int, w: int, policy: str = "further"):
    """:func:`stage_orders` with forward-FLOP segment costs (deterministic on every rank, no table)."""
    from ..models.blocks import block_costs, segment_units
    c = block_costs(cfg, h, w)
    f = []
    for j in range(pl.K):
        a, b = pl.seg_range(j)
        f.append(sum(c[i] * (1.0 if part == "full" else 0.5) for i, part in segment_units(a, b, cfg.depth)) / 1e9)
    return stage_orders(pl, cfg.depth, M, f, [2 * v for v in f], policy)


def parse_placement(spec: str) -> Placement:
    """``"v:0,2,7,10"`` / ``"contiguous:0,5,10"`` / ``"0,2,7,10@0,1,0"`` (cuts @ owners)."""
    spec = spec.strip()
    if "@" in spec:
        c, o = spec.split("@")
        return Placement(tuple(float(v) for v in c.split(",")), tuple(int(v) for v in o.split(",")))
    kind, _, c = spec.partition(":")
    cuts = tuple(float(v) for v in c.split(","))
    if kind == "v":
        return Placement.mirrored(cuts)
    if kind == "contiguous":
        return Placement.contiguous(cuts)
    raise ValueError(f"unknown placement {spec!r}")


def describe(pl: Placement, depth: int) -> List[str]:
    """Human-readable block lists per stage (for logs / BASELINE tables)."""
    from ..models.blocks import segment_units
    names = []
    for s in range(pl.S):
        parts = []
        for j in pl.segments(s):
            a, b = pl.seg_range(j)
            for idx, part in segment_units(a, b, depth):
                kind, i = block_kind(idx, depth)
                tag = f"{kind}{i}" if kind in ("enc", "dec") else kind
                parts.append(tag + ("" if part == "full" else part))
        names.append(f"stage {s}: " + " ".join(parts))
    return names


def v_partition(cfg, stages: int, h: int = 512, w: int = 512) -> Placement:
    """FLOP-balanced skip-local V placement (no table needed): among the mirrored placements of
    :func:`.schedule.mirrored_starts` (whole-block cuts, half-block ones when there are more stages than
    encoder levels), the one whose largest stage has the fewest training FLOPs."""
    from ..models.blocks import block_costs, segment_units
    from .schedule import mirrored_starts
    if stages == 1:
        return Placement.contiguous([0, n_blocks(cfg.depth)])
    c = block_costs(cfg, h, w)
    best = None
    whole = list(mirrored_starts(cfg.depth, stages, half=False))
    for cuts in whole or mirrored_starts(cfg.depth, stages, half=True):    # half-block cuts when needed
        pl = Placement.mirrored(cuts)
        load = [0.0] * stages
        for j in range(pl.K):
            a, b = pl.seg_range(j)
            load[pl.owner[j]] += sum(c[i] * (1.0 if part == "full" else 0.5)
                                     for i, part in segment_units(a, b, cfg.depth))
        if best is None or max(load) < best[0]:
            best = (max(load), pl)
    if best is None:
        raise ValueError(f"no V placement of {stages} stages for depth {cfg.depth}")
    return best[1]
