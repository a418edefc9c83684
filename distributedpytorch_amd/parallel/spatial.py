"""Row-split (spatial) full-resolution level for deep UNet pipelines: BASELINE config 5, UNet-XL 1024^2 on 8
MI355X (reference pipeline: ``model/unet_model.py:14-53``; SURVEY §5 "Long-context / sequence parallelism":
the image analogue of context parallelism, an H split with halo rows, in scope once 1024^2 UNet-XL needs it).

Why: at 1024^2 one 64-channel full-resolution activation is 134 MB per image -- 1.3 ms on a 100 GB/s xGMI
link, more than a stage's compute per image at 8 stages -- so every whole-level placement keeps the
full-resolution level (enc0 + dec_{D-1} + head: 25 % of the UNet-XL step) on ONE GPU and the 8-stage
efficiency stays near 0.3 (``profiles/pipeline_plan_r05.txt``).  Splitting that level by image ROWS over all
S stages instead moves only the level's small boundary tensors:

* stage s owns rows [r0, r1) = [s H/S, (s+1) H/S) of the full-resolution level of every image.  Its
  enc0 runs on image rows [r0 - 4, r1 + 4) (clipped at the image border): two stacked 3x3 convs are exact on
  [r0 - 2, r1 + 2), so the skip the stage's own dec_{D-1} needs (rows r0 - 2 .. r1 + 2) is computed locally,
  REDUNDANTLY -- no halo exchange at all, 4 extra rows of enc0 per 1024 / S;
* the pooled rows [r0/2, r1/2) go to the stage that owns enc1 (each stage sends 1/S of the pooled tensor;
  on the fully connected xGMI mesh the S - 1 slices arrive over S - 1 different links at once);
* the inner chain (enc1 .. dec_{D-2}: 2D - 1 blocks) is an ordinary placement (mirrored V or contiguous)
  over the S stages;
* the stage owning dec_{D-2} sends each stage its output rows [r0/2 - 1, r1/2 + 1) (the transposed conv
  maps input row i to output rows 2i, 2i + 1, so the up-sampled rows r0 - 2 .. r1 + 2 need no halo
  either); dec_{D-1}'s DoubleConv on rows [r0 - 2, r1 + 2) is exact on [r0, r1), whose head / loss partial
  sums the stage adds to the others' (global Dice = sums over every row of the batch).

Backward: every stage back-propagates its own slice graph; the redundantly computed halo rows make each
stage's graph a complete function of (parameters, image rows, received rows) for its own loss rows, so the
parameter gradients of the split level are the SUM over stages (one all-reduce of the level's ~0.7 MB of
fp32 gradients) and the gradient of the dec_{D-2} output is the sum of the stages' (overlapping) row
slices -- exact, not an approximation.  BatchNorm would need its statistics reduced across the stages:
row-split levels are for the BN-free reference block (``models/unet.py`` ``batchnorm=False``).

This module holds the geometry (:func:`row_plan`), the schedule model (:func:`simulate_spatial`, the same
link-queued list scheduler as :func:`.schedule.simulate_placement` on a general op graph) and the plan
search (:func:`search_spatial`); :class:`.pipeline.SpatialGPipe` is the engine.
"""
from __future__ import annotations

import itertools
import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

from .schedule import (DEFAULT_LINK_GBS, DEFAULT_LINK_LATENCY_MS, CostTable, Timeline, single_device_ms,
                       unit_boundary_bytes)

# ------------------------------------------------------------------------------------ geometry
def _clip(a: int, b: int, n: int) -> Tuple[int, int]:
    return max(0, a), min(n, b)


@dataclass(frozen=True)
class RowSlice:
    """Row ranges (at each split level's own resolution) of one stage's share of the top ``L`` levels.

    ``enc_in[l]``: rows encoder level l runs on (its input rows = its output rows, conv zero padding at the
    ends); ``dec_in[l]``: rows decoder level l (block dec_{D-1-l}) runs on; ``own``: the stage's rows of the
    full-resolution output; ``recv``: rows of the inner chain's output (level L) the stage receives; ``send``:
    its pooled rows of level L (the inner chain's input)."""
    L: int
    own: Tuple[int, int]
    enc_in: Tuple[Tuple[int, int], ...]
    dec_in: Tuple[Tuple[int, int], ...]
    recv: Tuple[int, int]
    send: Tuple[int, int]

    @property
    def rows(self) -> int:
        return self.own[1] - self.own[0]

    def enc_next_off(self, l: int) -> int:
        """Rows of encoder level l+1's input inside level l's pooled output."""
        return self.enc_in[l + 1][0] - self.enc_in[l][0] // 2

    def send_off(self) -> int:
        return self.send[0] - self.enc_in[self.L - 1][0] // 2

    def skip_off(self, l: int) -> int:
        """Decoder level l's rows inside encoder level l's output (the skip)."""
        return self.dec_in[l][0] - self.enc_in[l][0]

    def up_src(self, l: int) -> Tuple[int, int]:
        """Rows of level l+1 that decoder level l's transposed conv reads (its output rows / 2)."""
        d = self.dec_in[l]
        return d[0] // 2, d[1] // 2

    def up_off(self, l: int) -> int:
        """Those rows inside what level l+1 provides: decoder level l+1's rows, or the received rows."""
        src = self.recv if l == self.L - 1 else self.dec_in[l + 1]
        return self.up_src(l)[0] - src[0]

    def out_off(self) -> int:
        return self.own[0] - self.dec_in[0][0]


def row_plan(H: int, S: int, L: int = 1, bounds: Optional[Sequence[int]] = None) -> List[RowSlice]:
    """Row slices of the top ``L`` levels for S stages: own rows [bounds[s], bounds[s+1]) (default: equal
    slices; every bound a multiple of 2^L), halos sized so that every split level's two 3x3 convs are exact
    on the rows the next consumer needs -- all halos are computed REDUNDANTLY by the stage itself, so no rows
    are exchanged between neighbours."""
    q = 2 ** L
    if bounds is None:
        if L < 1 or H % (q * S):
            raise ValueError(f"image height {H} cannot be split into {S} equal row slices over {L} levels")
        bounds = [s * (H // S) for s in range(S + 1)]
    bounds = [int(b) for b in bounds]
    if (L < 1 or len(bounds) != S + 1 or bounds[0] != 0 or bounds[-1] != H or any(b % q for b in bounds)
            or any(b - a < 2 * q for a, b in zip(bounds, bounds[1:]))):
        raise ValueError(f"bad row bounds {bounds} for {S} stages, {L} split levels, height {H}")
    out = []
    for s in range(S):
        r0, r1 = bounds[s], bounds[s + 1]
        Hl = [H >> l for l in range(L + 1)]
        # decoder side, from the full-resolution output up: exact rows D_l need input rows D_l +- 2
        dec_in, exact = [], (r0, r1)
        for l in range(L):
            a, b = _clip(exact[0] - 2, exact[1] + 2, Hl[l])
            a -= a % 2                                  # even: the up-sampled rows of level l+1 map exactly
            b = min(b + b % 2, Hl[l])
            dec_in.append((a, b))
            exact = (a // 2, b // 2)                    # rows of level l+1 the transposed conv reads
        recv = exact
        # encoder side, from level L-1 down: exact rows E_l cover the skip rows dec_in[l] and the next
        # level's input (x2); each level runs on E_l +- 2 (even, so its pooled rows align)
        send = (r0 >> L, r1 >> L)
        enc_in = [None] * L
        need = (send[0] * 2, send[1] * 2)               # level L-1 rows whose pool is the sent rows
        for l in range(L - 1, -1, -1):
            a = min(need[0], dec_in[l][0])
            b = max(need[1], dec_in[l][1])
            a, b = _clip(a - 2, b + 2, Hl[l])
            a -= a % 2
            b += b % 2
            enc_in[l] = (a, min(b, Hl[l]))
            need = (2 * enc_in[l][0], 2 * enc_in[l][1]) if l > 0 else None
        out.append(RowSlice(L, (r0, r1), tuple(enc_in), tuple(dec_in), recv, send))
    return out


# ------------------------------------------------------------------------------------ op graph
@dataclass
class GNode:
    name: str
    stage: int
    fwd: float                                   # ms per microbatch
    bwd: float
    ins: List[Tuple[int, int]] = field(default_factory=list)   # (producer node, bytes per microbatch)
    head: bool = False                           # the loss needs its forward (all microbatches)
    wgrad: float = 0.0                           # deferred weight gradient: one launch after its last backward


def simulate_graph(nodes: Sequence[GNode], S: int, M: int, wgrad: Sequence[float] = None,
                   opt: Sequence[float] = None, tail: Sequence[float] = None, loss_ms: float = 0.0,
                   link_gbs: float = DEFAULT_LINK_GBS, link_latency_ms: float = DEFAULT_LINK_LATENCY_MS,
                   policy: str = "further") -> Timeline:
    """GPipe all-forward / all-backward step of an op graph (:func:`.schedule.simulate_placement` on a
    general graph): node n's microbatch m forward after every producer's (a message on the directed peer
    link when the stages differ: FIFO, one message per (op, destination stage), latency once), backward
    after every consumer's backward and, for head nodes, after the loss; each stage runs its ops one at a
    time, all forwards first, by list scheduling (earliest start; ties: ``policy``).  A node's deferred
    weight gradient (``GNode.wgrad``: the engine's merged launch of all microbatches, issued once its last
    microbatch's backward is done) is an op of its own that becomes ready then and loses ties to the
    forward / backward ops -- it fills the stage's idle time of the drain instead of following the last op.
    ``wgrad[s]``: weight-gradient time that does follow the last op; ``tail[s]``: time after that before the
    optimizer (e.g. a gradient all-reduce)."""
    K = len(nodes)
    outs: List[List[Tuple[int, int]]] = [[] for _ in range(K)]
    for n, nd in enumerate(nodes):
        for p, b in nd.ins:
            outs[p].append((n, b))
    wgrad = list(wgrad) if wgrad is not None else [0.0] * S
    opt = list(opt) if opt is not None else [0.0] * S
    tail = list(tail) if tail is not None else [0.0] * S
    segs = [[n for n in range(K) if nodes[n].stage == s] for s in range(S)]
    fwd = [[None] * M for _ in range(K)]
    bwd = [[None] * M for _ in range(K)]
    arrive: Dict[Tuple[str, int, int, int], float] = {}
    link_free: Dict[Tuple[int, int], float] = {}
    link_busy: Dict[Tuple[int, int], float] = {}
    link_bytes: Dict[Tuple[int, int], int] = {}
    free = [0.0] * S
    fnext, bnext = [0] * K, [M - 1] * K
    done_f, done_b = [0] * S, [0] * S
    nf = [len(segs[s]) * M for s in range(S)]
    heads = [n for n in range(K) if nodes[n].head]
    head_done = 0
    loss_t = None
    got = [{"fwd": [], "bwd": []} for _ in range(S)]

    def ready(kind, n, m):
        me = nodes[n].stage
        t = 0.0
        if kind == "fwd":
            for p, _ in nodes[n].ins:
                if fwd[p][m] is None:
                    return None
                t = max(t, fwd[p][m][1] if nodes[p].stage == me else arrive[("fwd", p, m, me)])
            return t
        if nodes[n].head:
            if loss_t is None:
                return None
            t = loss_t
        for c, _ in outs[n]:
            if bwd[c][m] is None:
                return None
            t = max(t, bwd[c][m][1] if nodes[c].stage == me else arrive[("bwd", c, m, me)])
        return t

    def send(kind, n, m, end):
        src = nodes[n].stage
        per: Dict[int, int] = {}
        edges = outs[n] if kind == "fwd" else nodes[n].ins
        for other, b in edges:
            d = nodes[other].stage
            if d != src:
                per[d] = per.get(d, 0) + b
        for d, nbytes in sorted(per.items()):
            dur = nbytes / (link_gbs * 1e6)
            st = max(end, link_free.get((src, d), 0.0))
            link_free[(src, d)] = st + dur
            link_busy[(src, d)] = link_busy.get((src, d), 0.0) + dur
            link_bytes[(src, d)] = link_bytes.get((src, d), 0) + nbytes
            arrive[(kind, n, m, d)] = st + dur + link_latency_ms

    wg_done = [nodes[n].wgrad <= 0 for n in range(K)]
    wg_span: Dict[int, Tuple[float, float]] = {}
    total = 2 * K * M + sum(1 for v in wg_done if not v)
    done = 0
    while done < total:
        best = None
        for s in range(S):
            kind = "fwd" if done_f[s] < nf[s] else "bwd"
            if kind == "bwd" and done_b[s] >= nf[s]:
                kind = None
            for n in (segs[s] if kind else ()):
                m = fnext[n] if kind == "fwd" else bnext[n]
                if (kind == "fwd" and m >= M) or (kind == "bwd" and m < 0):
                    continue
                r = ready(kind, n, m)
                if r is None:
                    continue
                pr = -n if kind == "fwd" else n
                key = (max(free[s], r), 0, pr if policy == "further" else -pr, s)
                if best is None or key < best[0]:
                    best = (key, s, kind, n, m)
            for n in segs[s]:
                if not wg_done[n] and bnext[n] < 0:
                    key = (max(free[s], bwd[n][0][1]), 1, n, s)
                    if best is None or key < best[0]:
                        best = (key, s, "wg", n, 0)
        if best is None:
            raise RuntimeError("spatial schedule deadlock")
        (start, _, _, _), s, kind, n, m = best
        if kind == "wg":
            free[s] = start + nodes[n].wgrad
            wg_done[n] = True
            wg_span[n] = (start, free[s])
            done += 1
            continue
        dur = nodes[n].fwd if kind == "fwd" else nodes[n].bwd
        end = start + dur
        free[s] = end
        if kind == "fwd":
            fwd[n][m] = (start, end)
            fnext[n] += 1
            done_f[s] += 1
            if nodes[n].head and fnext[n] == M:
                head_done += 1
                if head_done == len(heads):
                    loss_t = max(fwd[h][M - 1][1] for h in heads) + loss_ms
        else:
            bwd[n][m] = (start, end)
            bnext[n] -= 1
            done_b[s] += 1
        got[s][kind].append(n)
        send(kind, n, m, end)
        done += 1
    stage_end = [free[s] + wgrad[s] + tail[s] + opt[s] for s in range(S)]
    busy = [M * sum(nodes[n].fwd + nodes[n].bwd for n in segs[s]) + sum(nodes[n].wgrad for n in segs[s])
            + wgrad[s] + opt[s] for s in range(S)]
    return Timeline(max(stage_end), fwd, bwd, stage_end, busy, got, link_busy, link_bytes)


# ------------------------------------------------------------------------------------ the plan
@dataclass(frozen=True)
class SpatialPlan:
    """The top ``L`` levels (encoder blocks 0..L-1, decoder blocks dec_{D-L}..dec_{D-1} and the head) row-split
    over all S stages + the inner chain [L, 2D+1-L) on ``inner_cuts`` / ``inner_owner`` (block positions;
    ``b + 0.5`` = between block b's two convs)."""
    S: int
    inner_cuts: Tuple[float, ...]
    inner_owner: Tuple[int, ...]
    L: int = 1
    bounds: Optional[Tuple[int, ...]] = None       # own full-resolution rows per stage (None: equal slices)

    @property
    def K(self) -> int:
        return len(self.inner_owner)

    def seg_range(self, j: int) -> Tuple[float, float]:
        return self.inner_cuts[j], self.inner_cuts[j + 1]

    def seg_of(self, pos: float) -> int:
        for j in range(self.K):
            if self.inner_cuts[j] <= pos < self.inner_cuts[j + 1]:
                return j
        raise ValueError(pos)

    def segments(self, s: int) -> List[int]:
        return [j for j, o in enumerate(self.inner_owner) if o == s]

    @property
    def first_stage(self) -> int:
        """Owner of the inner chain's first block (receives the pooled slices)."""
        return self.inner_owner[0]

    @property
    def last_stage(self) -> int:
        """Owner of the inner chain's last block (sends the up-path rows)."""
        return self.inner_owner[-1]

    def validate(self, depth: int) -> "SpatialPlan":
        nb = 2 * depth + 2
        c = self.inner_cuts
        if not 1 <= self.L < depth or c[0] != self.L or c[-1] != nb - 1 - self.L:
            raise ValueError(f"inner chain of {self} must run from block {self.L} to {nb - 1 - self.L}")
        if any(b <= a for a, b in zip(c, c[1:])) or any(2 * x != int(2 * x) for x in c):
            raise ValueError(f"bad inner cuts {c}")
        if len(c) != len(self.inner_owner) + 1 or sorted(set(self.inner_owner)) != list(range(self.S)):
            raise ValueError(f"every stage 0..{self.S - 1} must own an inner segment: {self.inner_owner}")
        return self

    def to_plan(self) -> dict:
        return {"spatial": True, "split_levels": self.L, "stages": self.S, "inner_cuts": list(self.inner_cuts),
                "inner_owner": list(self.inner_owner), "row_bounds": None if self.bounds is None else list(self.bounds)}

    @staticmethod
    def from_plan(p: dict) -> "SpatialPlan":
        b = p.get("row_bounds")
        return SpatialPlan(int(p["stages"]), tuple(p["inner_cuts"]), tuple(int(o) for o in p["inner_owner"]),
                           int(p.get("split_levels", 1)), None if b is None else tuple(int(v) for v in b))

    def rows(self, H: int) -> List[RowSlice]:
        return row_plan(H, self.S, self.L, self.bounds)

    def with_bounds(self, bounds) -> "SpatialPlan":
        return SpatialPlan(self.S, self.inner_cuts, self.inner_owner, self.L, None if bounds is None else tuple(bounds))

    def __str__(self):
        b = "" if self.bounds is None else f"rows{list(self.bounds)}"
        return f"spatial{self.S}x{self.L}lvl{b}+inner{list(self.inner_cuts)}@{list(self.inner_owner)}"


def mirrored_inner(depth: int, S: int, cuts_left: Sequence[float], L: int = 1) -> SpatialPlan:
    """Inner V: stage s owns the inner encoder range [L_s, L_{s+1}) and the mirrored decoder blocks
    (encoder level l <-> decoder block 2D - l, so a left cut p mirrors to 2D + 1 - p)."""
    right = [2 * depth + 1 - p for p in reversed(cuts_left)]
    cuts = (L, *cuts_left, *right, 2 * depth + 1 - L)
    K = len(cuts) - 1
    return SpatialPlan(S, tuple(cuts), tuple(min(k, 2 * S - 2 - k) for k in range(K)), L)


def contiguous_inner(depth: int, S: int, cuts_mid: Sequence[float], L: int = 1) -> SpatialPlan:
    cuts = (L, *cuts_mid, 2 * depth + 1 - L)
    return SpatialPlan(S, tuple(cuts), tuple(range(len(cuts) - 1)), L)


def _slice_cost(table: dict, blocks: Sequence[int], halo: Sequence[float], frac: float, M: int):
    """(fwd, bwd without weight gradient, deferred weight gradient over all M microbatches) ms of ``blocks``
    run on ``frac`` images' worth of rows, block b scaled by ``halo[i]`` (its computed / own rows).  Priced
    from the table's per-image time at the largest measured batch <= frac; below one image from the
    one-image time scaled by the pixel fraction and a small-launch penalty: the table's own one-image /
    two-image per-image ratio per halving (UNet-XL enc0: 1.12 per halving, so a 1/8-image slice is priced
    at 1.4x the one-image per-pixel rate)."""
    per = table["per_mb"]
    sizes = sorted(int(k) for k in per)

    def rate(n):
        if n >= 1:
            k = max(v for v in sizes if v <= n)
            return per[str(k)], n / k, 1.0
        r, r2 = per["1"], per.get("2")
        pen = 1.0
        if r2 is not None:
            num = sum(r["fwd"][b] + r["bwd"][b] for b in blocks)
            den = sum(r2["fwd"][b] + r2["bwd"][b] for b in blocks) / 2
            pen = max(1.0, num / den) ** math.log2(1 / n)
        return r, n, pen

    r, sc, pen = rate(frac)
    f = sum(r["fwd"][b] * h for b, h in zip(blocks, halo)) * sc * pen
    bnw = sum(r["bwd_nowgrad"][b] * h for b, h in zip(blocks, halo)) * sc * pen
    rr, sc2, pen2 = rate(frac * M)          # the deferred weight gradients: all microbatches in one launch
    wg = sum((rr["bwd"][b] - rr["bwd_nowgrad"][b]) * h for b, h in zip(blocks, halo)) * sc2 * pen2
    return f, bnw, max(wg, 0.0)


def split_param_bytes(widths: Sequence[int], L: int, in_ch: int = 3) -> int:
    """fp32 bytes of the split levels' parameters (encoder convs, transposed convs, decoder convs, head)."""
    n, cin = 0, in_ch
    for l in range(L):
        w = widths[l]
        n += 9 * cin * w + w + 9 * w * w + w                         # encoder DoubleConv
        n += 4 * widths[l + 1] * w + w                                # transposed conv (2x2) into level l
        n += 9 * 2 * w * w + w + 9 * w * w + w                        # decoder DoubleConv over the concat
        cin = w
    return 4 * (n + widths[0] + 1)


def spatial_graph(table: dict, plan: SpatialPlan, batch: int, M: int):
    """Op graph of one step: nodes ``L0f{s}`` (the split encoder levels on stage s's rows), the inner
    segments, ``L0g{s}`` (the split decoder levels + head); per-stage deferred weight-gradient ms, optimizer
    ms and the split levels' gradient all-reduce."""
    depth, S, L = table["depth"], plan.S, plan.L
    H, W = table["img"]
    widths, mid = table["widths"], table["mid_width"]
    mb = batch // M
    nbk = 2 * depth + 2
    bt = table.get("block_table", table)
    rp = plan.rows(H)
    nodes: List[GNode] = []
    wg = [0.0] * S
    opt = [0.0] * S
    bopt = bt.get("opt_ms", [0.0] * nbk)
    enc_blocks = list(range(L))
    dec_blocks = [nbk - 2 - l for l in range(L)]          # dec at level l = block nbk-2-l
    split_opt = sum(bopt[b] for b in enc_blocks + dec_blocks) + bopt[nbk - 1]
    gs = []
    for s in range(S):
        sl = rp[s]
        h = sl.rows
        eh = [(sl.enc_in[l][1] - sl.enc_in[l][0]) / (h / 2 ** l) for l in range(L)]
        dh = [(sl.dec_in[l][1] - sl.dec_in[l][0]) / (h / 2 ** l) for l in range(L)]
        f0, b0, w0 = _slice_cost(bt, enc_blocks, eh, mb * h / H, M)
        g0, gb0, gw0 = _slice_cost(bt, dec_blocks + [nbk - 1], dh + [1.0], mb * h / H, M)
        nodes.append(GNode(f"L0f{s}", s, f0, b0, wgrad=w0))
        gs.append((g0, gb0, gw0))
        opt[s] += split_opt
    ct = CostTable(table, mb, M)
    base = S
    for j in range(plan.K):
        a, b = plan.seg_range(j)
        f, bw, w_, o_ = ct.range(ct.idx(a), ct.idx(b))
        nodes.append(GNode(f"in{j}", plan.inner_owner[j], f, bw, wgrad=w_))
        opt[plan.inner_owner[j]] += o_
    # inner edges: every boundary tensor whose producer and consumer units both lie in the inner chain
    lo, hi = 2 * L, 2 * (nbk - 1 - L)
    ins: Dict[int, Dict[int, int]] = {}
    for name, (pu, cu, nbytes) in unit_boundary_bytes(depth, widths, mid, mb, H, W).items():
        if not (lo <= pu < hi and lo <= cu < hi):
            continue
        p, c = plan.seg_of(pu / 2), plan.seg_of(cu / 2)
        if p != c:
            ins.setdefault(c, {})
            ins[c][p] = ins[c].get(p, 0) + nbytes
    for c, d in ins.items():
        nodes[base + c].ins = sorted((base + p, nb) for p, nb in d.items())
    Wl = W >> L
    for s in range(S):
        sl = rp[s]
        nodes[base].ins.append((s, mb * widths[L - 1] * (sl.send[1] - sl.send[0]) * Wl * 2))
    for s in range(S):
        sl = rp[s]
        nbytes = mb * widths[L] * (sl.recv[1] - sl.recv[0]) * Wl * 2
        nodes.append(GNode(f"L0g{s}", s, gs[s][0], gs[s][1], ins=[(base + plan.K - 1, nbytes)], head=True,
                           wgrad=gs[s][2]))
    # the split levels' parameter gradients: summed over the S stages (ring all-reduce of fp32 grads)
    pb = split_param_bytes(widths, L)
    ar = 2 * (S - 1) / S * pb / (DEFAULT_LINK_GBS * 1e6) + 2 * (S - 1) * DEFAULT_LINK_LATENCY_MS
    return nodes, wg, opt, [ar] * S


def placement_graph(table: dict, pl, batch: int, M: int) -> Tuple[List[GNode], List[float]]:
    """A whole-level :class:`.placement.Placement` as an op graph for :func:`simulate_graph` (the same
    per-segment costs and boundary bytes as :func:`.schedule.placement_costs`), so whole-level and row-split
    plans are compared under one model (deferred weight gradients in the drain's idle time for both)."""
    from .placement import seg_io
    from .schedule import edge_bytes
    mb = batch // M
    ct = CostTable(table, mb, M)
    opt = [0.0] * pl.S
    nodes = []
    for j in range(pl.K):
        a, b = pl.seg_range(j)
        f, bw, w_, o_ = ct.range(ct.idx(a), ct.idx(b))
        nodes.append(GNode(f"seg{j}", pl.owner[j], f, bw, wgrad=w_, head=(j == pl.head_seg)))
        opt[pl.owner[j]] += o_
    h, w = table["img"]
    eb = edge_bytes(pl, table["depth"], table["widths"], table["mid_width"], mb, h, w)
    ins, _ = seg_io(pl, table["depth"])
    for j in range(pl.K):
        nodes[j].ins = sorted((p, eb.get((p, j), 0)) for p in {p for _, p in ins[j]})
    return nodes, opt


def simulate_placement_graph(table: dict, pl, batch: int, M: int, policy: str = "further", **link) -> Timeline:
    nodes, opt = placement_graph(table, pl, batch, M)
    return simulate_graph(nodes, pl.S, M, None, opt, None, policy=policy, **link)


def simulate_spatial(table: dict, plan: SpatialPlan, batch: int, M: int, policy: str = "further",
                     **link) -> Timeline:
    nodes, wg, opt, tail = spatial_graph(table, plan, batch, M)
    return simulate_graph(nodes, plan.S, M, wg, opt, tail, policy=policy, **link)


def balance_rows(table: dict, plan: SpatialPlan, batch: int, M: int) -> SpatialPlan:
    """Uneven row slices that even out the stages' busy time: a stage whose inner segments are light takes
    more rows of the split levels (busy = its inner segments + rows x the split levels' per-row cost, the
    halo rows priced on the equal-slice geometry); bounds multiples of 2^L, >= 2^(L+1) rows each."""
    H = table["img"][0]
    S, L = plan.S, plan.L
    q = 2 ** L
    eq = plan.with_bounds(None)
    nodes, wg, _, _ = spatial_graph(table, eq, batch, M)
    inner = [0.0] * S
    for nd in nodes[S:S + plan.K]:
        inner[nd.stage] += M * (nd.fwd + nd.bwd) + nd.wgrad
    split = [M * (nodes[s].fwd + nodes[s].bwd + nodes[S + plan.K + s].fwd + nodes[S + plan.K + s].bwd)
             + nodes[s].wgrad + nodes[S + plan.K + s].wgrad for s in range(S)]
    per_row = sum(split) / H
    # target T: sum_s (T - inner_s) / per_row = H  (rows never below the minimum)
    lo, hi = 0.0, max(inner) + H * per_row
    for _ in range(60):
        T = (lo + hi) / 2
        rows = [max(2 * q, (T - inner[s]) / per_row) for s in range(S)]
        if sum(rows) > H:
            hi = T
        else:
            lo = T
    rows = [max(2 * q, (lo - inner[s]) / per_row) for s in range(S)]
    # round to multiples of q keeping the total
    cum, bounds = 0.0, [0]
    for s in range(S - 1):
        cum += rows[s]
        b = int(round(cum / q)) * q
        b = max(b, bounds[-1] + 2 * q)
        bounds.append(min(b, H - 2 * q * (S - 1 - s)))
    bounds.append(H)
    try:
        return plan.with_bounds(bounds) if row_plan(H, S, L, bounds) else plan
    except ValueError:
        return plan


def search_spatial(table: dict, S: int, batch: int, Ms: Optional[Sequence[int]] = None, levels=(1, 2),
                   policies: Sequence[str] = ("feed", "further"), top: int = 3, **link) -> List[dict]:
    """Best row-split plan per microbatch count: for each number of split levels, every skip-local inner V
    (half-block cuts) and a sample of contiguous inner chains, each simulated with both op-order policies;
    the best ``top`` refined by single half-block cut moves."""
    depth = table["depth"]
    t1 = single_device_ms(table, batch)
    step = 0.5 if table.get("unit_space") else 1.0
    sizes = sorted(int(k) for k in table["per_mb"])
    H = table["img"][0]
    out = []
    for M in (Ms or sorted({batch // k for k in sizes if batch % k == 0})):
        mb = batch // M
        if str(mb) not in table["per_mb"]:
            continue
        cands = []
        for L in levels:
            try:
                row_plan(H, S, L)
            except ValueError:
                continue
            left = [L + step * i for i in range(1, int((depth + 1 - L) / step))]            # (L, D + 1)
            inner_all = [L + step * i for i in range(1, int((2 * depth + 1 - 2 * L) / step))]
            cands += [mirrored_inner(depth, S, c, L) for c in itertools.combinations(left, S - 1)]
            cands += [contiguous_inner(depth, S, c, L)
                      for c in itertools.islice(itertools.combinations(inner_all, S - 1), 300)]
        scored = []
        for pl in cands:
            try:
                pl.validate(depth)
            except ValueError:
                continue
            for p2 in (pl, balance_rows(table, pl, batch, M)):
                for pol in policies:
                    tl = simulate_spatial(table, p2, batch, M, policy=pol, **link)
                    scored.append((tl.step_ms, p2, pol, tl))
        scored.sort(key=lambda r: r[0])
        best = None
        for _, pl, pol, tl in scored[:top]:
            cur, cur_tl = pl, tl
            improved = True
            while improved:
                improved = False
                for k in range(1, len(cur.inner_cuts) - 1):
                    for d in (-step, step):
                        c = list(cur.inner_cuts)
                        c[k] += d
                        cand = SpatialPlan(S, tuple(c), cur.inner_owner, cur.L, cur.bounds)
                        try:
                            cand.validate(depth)
                        except ValueError:
                            continue
                        for c2 in ((cand, balance_rows(table, cand, batch, M)) if cur.bounds is not None
                                   else (cand,)):
                            t2 = simulate_spatial(table, c2, batch, M, policy=pol, **link)
                            if t2.step_ms < cur_tl.step_ms - 1e-9:
                                cur, cur_tl, improved = c2, t2, True
            if best is None or cur_tl.step_ms < best[2].step_ms:
                best = (cur, pol, cur_tl)
        if best is None:
            continue
        pl, pol, tl = best
        r = {"stages": S, "microbatches": M, "mb": mb, "placement": "spatial", **pl.to_plan(), "policy": pol,
             "step_ms": round(tl.step_ms, 3), "img_s": round(batch * 1000.0 / tl.step_ms, 1),
             "utilisation": round(tl.efficiency(), 3),
             "max_link_busy_ms": round(max(tl.link_busy.values()), 3) if tl.link_busy else 0.0,
             "max_link_gb": round(max(tl.link_bytes.values()) / 1e9, 3) if tl.link_bytes else 0.0}
        if t1 is not None:
            r["speedup_vs_1gpu"] = round(t1 / tl.step_ms, 3)
            r["scaling_efficiency"] = round(t1 / tl.step_ms / S, 3)
        out.append(r)
    return out


def default_plan(cfg, S: int, h: int, w: int, L: int = 0) -> SpatialPlan:
    """A row-split plan without a measured table: the fewest split levels the image height allows
    (``L``: force), equal row slices, the inner chain cut into S contiguous FLOP-balanced half-block ranges
    (exact min-max DP over the units)."""
    from ..models.blocks import block_costs
    depth = cfg.depth
    nb = 2 * depth + 2
    for L_ in ([L] if L else range(1, depth)):
        try:
            row_plan(h, S, L_)
        except ValueError:
            continue
        c = block_costs(cfg, h, w)
        units = []                       # (position, cost) of every half block of the inner chain
        for b in range(L_, nb - 1 - L_):
            units += [(b, c[b] / 2), (b + 0.5, c[b] / 2)]
        U = len(units)
        if U < S:
            continue
        pre = [0.0]
        for _, v in units:
            pre.append(pre[-1] + v)
        INF = float("inf")
        best = [[INF] * (U + 1) for _ in range(S + 1)]
        arg = [[0] * (U + 1) for _ in range(S + 1)]
        best[0][0] = 0.0
        for k in range(1, S + 1):
            for j in range(k, U + 1):
                for i in range(k - 1, j):
                    v = max(best[k - 1][i], pre[j] - pre[i])
                    if v < best[k][j]:
                        best[k][j], arg[k][j] = v, i
        idx, j = [U], U
        for k in range(S, 0, -1):
            j = arg[k][j]
            idx.append(j)
        idx = list(reversed(idx))
        cuts = [units[i][0] if i < U else nb - 1 - L_ for i in idx]
        return SpatialPlan(S, tuple(cuts), tuple(range(S)), L_).validate(depth)
    raise ValueError(f"no row-split plan of {S} stages for a {h}x{w} image and depth {depth}")
