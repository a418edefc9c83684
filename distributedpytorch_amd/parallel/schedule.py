"""GPipe schedule model with per-link transfer queues, and the placement search.

The pipeline engine (:class:`.pipeline.GPipeDist`, reference ``model/unet_model.py:24-53`` generalised
to S stages x M microbatches over a :class:`.placement.Placement`) runs ALL forwards, then ALL
backwards: the loss is the reference's global Dice over the whole batch, so no microbatch's backward
can start before every microbatch's forward has reached the head.  Its step time is a fill / drain
schedule whose best stage boundaries depend on measured per-block TIME (the full-resolution levels run
at ~0.6 PF on MI355X, the deep GEMMs at 1.3-1.5 PF) AND on the bytes each boundary puts on an xGMI link.

:func:`simulate_placement` runs that schedule op by op:

* ops: forward (j, m) and backward (j, m) of every segment j and microbatch m; segment j's microbatches
  run in order (0..M-1 forward, M-1..0 backward); a stage runs one op at a time, in a static order
  (``orders``) or, with ``orders=None``, by list scheduling (the earliest-startable op; ties by
  ``policy``) -- the order it picks is returned and is what the engine issues;
* dependencies: forward (j, m) after every producer segment's forward (j-1 for x, the encoder segment
  for a skip); backward (j, m) after every consumer segment's backward, the head segment's after the
  loss (all forwards of the head segment);
* transfers: the tensors one op sends to one other stage are one message (one grouped RCCL launch:
  latency once, bytes add) on the DIRECTED peer link (src stage, dst stage); a link carries one message
  at a time, FIFO in the order the sender's ops finish, so a message starts at max(producer end, link
  free) and arrives ``latency + bytes / bandwidth`` later.  Segments of one stage hand over locally;
* the stage ends after its last op plus its deferred weight gradients (the engine merges every
  microbatch's weight gradient of a layer into one launch in the drain) and its optimizer step.

:func:`search` finds the best contiguous or mirrored (V) placement for a measured table: an exact
min-max DP over stage busy times gives the start, then a local search over single-cut moves with the
simulator (including half-block cuts) and every microbatch count the table supports.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

from .placement import Placement, remote_groups, seg_io

DEFAULT_LINK_GBS = 100.0
DEFAULT_LINK_LATENCY_MS = 0.015


@dataclass
class SegCost:
    fwd: float                   # ms per microbatch forward
    bwd: float                   # ms per microbatch backward (dgrads + weight gradients not deferred)


@dataclass
class Timeline:
    step_ms: float
    fwd: List[List[Tuple[float, float]]]     # [segment][microbatch] -> (start, end)
    bwd: List[List[Tuple[float, float]]]
    stage_end: List[float]
    busy_ms: List[float]                     # compute time per stage
    orders: List[Dict[str, List[int]]]       # per stage: segment sequence of its fwd / bwd ops
    link_busy: Dict[Tuple[int, int], float] = field(default_factory=dict)   # ms of transfer per directed link
    link_bytes: Dict[Tuple[int, int], int] = field(default_factory=dict)    # bytes per step per directed link

    def efficiency(self) -> float:
        """Mean stage utilisation: sum of stage busy time / (stages x step)."""
        return sum(self.busy_ms) / (len(self.busy_ms) * self.step_ms)


def edge_bytes(pl: Placement, depth: int, widths: Sequence[int], mid_width: int, mb: int, h: int, w: int,
               dtype_bytes: int = 2) -> Dict[Tuple[int, int], int]:
    """Bytes per microbatch of every segment edge (producer segment, consumer segment) -- the x along
    the chain, the skips, and a DoubleConv's inner activation at a half-block cut."""
    out: Dict[Tuple[int, int], int] = {}
    for _, (pu, cu, nbytes) in unit_boundary_bytes(depth, widths, mid_width, mb, h, w, dtype_bytes).items():
        p, c = pl.seg_of(pu / 2), pl.seg_of(cu / 2)
        if p != c:
            out[(p, c)] = out.get((p, c), 0) + nbytes
    return out


def simulate_placement(pl: Placement, depth: int, M: int, costs: Sequence[SegCost],
                       ebytes: Optional[Dict[Tuple[int, int], int]] = None, wgrad: Sequence[float] = None,
                       opt: Sequence[float] = None, loss_ms: float = 0.0, link_gbs: float = DEFAULT_LINK_GBS,
                       link_latency_ms: float = DEFAULT_LINK_LATENCY_MS,
                       orders: Optional[List[Dict[str, List[int]]]] = None, policy: str = "further") -> Timeline:
    """Simulate one all-forward / all-backward step of placement ``pl`` (see the module docstring).

    ``costs[j]``: per-microbatch forward / backward ms of segment j; ``ebytes[(p, c)]``: bytes per
    microbatch from segment p to segment c (forward activations; the backward sends gradients of the
    same size the other way); ``wgrad`` / ``opt``: per-stage deferred weight-gradient and optimizer ms."""
    K, S = pl.K, pl.S
    ins, outs = seg_io(pl, depth)
    ebytes = ebytes or {}
    wgrad = list(wgrad) if wgrad is not None else [0.0] * S
    opt = list(opt) if opt is not None else [0.0] * S
    segs = [pl.segments(s) for s in range(S)]
    owner = pl.owner
    fwd = [[None] * M for _ in range(K)]
    bwd = [[None] * M for _ in range(K)]
    # arrival of the message op (kind, j, m) sends to stage d: arrive[(kind, j, m, d)]
    arrive: Dict[Tuple[str, int, int, int], float] = {}
    link_free: Dict[Tuple[int, int], float] = {}
    link_busy: Dict[Tuple[int, int], float] = {}
    link_bytes: Dict[Tuple[int, int], int] = {}
    free = [0.0] * S
    fnext = [0] * K
    bnext = [M - 1] * K
    done_f = [0] * S
    nf = [len(segs[s]) * M for s in range(S)]
    done_b = [0] * S
    got = [{"fwd": [], "bwd": []} for _ in range(S)]
    pos = [{"fwd": 0, "bwd": 0} for _ in range(S)]
    head = pl.head_seg
    loss_t = None

    # messages: per op, the edges grouped by destination stage
    fwd_msgs = [remote_groups(pl, outs[j], owner[j]) for j in range(K)]
    bwd_msgs = [remote_groups(pl, ins[j], owner[j]) for j in range(K)]

    def msg_bytes(j, edges, kind):
        if kind == "fwd":
            return sum(ebytes.get((j, c), 0) for c in {c for _, c in edges})
        return sum(ebytes.get((p, j), 0) for p in {p for _, p in edges})

    def ready(kind, j, m):
        """Time all inputs of op (kind, j, m) are on its stage, or None if a producer is unscheduled."""
        me = owner[j]
        t = 0.0
        if kind == "fwd":
            for _, p in ins[j]:
                if fwd[p][m] is None:
                    return None
                t = max(t, fwd[p][m][1] if owner[p] == me else arrive[("fwd", p, m, me)])
            return t
        if j == head:
            if loss_t is None:
                return None
            t = loss_t
        for _, c in outs[j]:
            if bwd[c][m] is None:
                return None
            t = max(t, bwd[c][m][1] if owner[c] == me else arrive[("bwd", c, m, me)])
        return t

    def send(kind, j, m, end):
        src = owner[j]
        for d, edges in (fwd_msgs[j] if kind == "fwd" else bwd_msgs[j]).items():
            nbytes = msg_bytes(j, edges, kind)
            dur = nbytes / (link_gbs * 1e6)
            st = max(end, link_free.get((src, d), 0.0))
            link_free[(src, d)] = st + dur
            link_busy[(src, d)] = link_busy.get((src, d), 0.0) + dur
            link_bytes[(src, d)] = link_bytes.get((src, d), 0) + nbytes
            arrive[(kind, j, m, d)] = st + dur + link_latency_ms

    def candidates(s):
        kind = "fwd" if done_f[s] < nf[s] else "bwd"
        if kind == "bwd" and done_b[s] >= nf[s]:
            return kind, []
        if orders is not None:
            seq = orders[s][kind]
            j = seq[pos[s][kind]]
            return kind, [j]
        if kind == "fwd":
            return kind, [j for j in segs[s] if fnext[j] < M]
        return kind, [j for j in segs[s] if bnext[j] >= 0]

    def prio(kind, j):
        further = -j if kind == "fwd" else j         # closer to the end of its phase's chain first
        return further if policy == "further" else -further

    total = 2 * K * M
    n = 0
    while n < total:
        best = None
        for s in range(S):
            kind, cands = candidates(s)
            for j in cands:
                m = fnext[j] if kind == "fwd" else bnext[j]
                r = ready(kind, j, m)
                if r is None:
                    continue
                key = (max(free[s], r), prio(kind, j), s)
                if best is None or key < best[0]:
                    best = (key, s, kind, j, m)
        if best is None:
            raise RuntimeError(f"schedule deadlock: placement {pl}, orders {orders}")
        (start, _, _), s, kind, j, m = best
        dur = costs[j].fwd if kind == "fwd" else costs[j].bwd
        end = start + dur
        free[s] = end
        if kind == "fwd":
            fwd[j][m] = (start, end)
            fnext[j] += 1
            done_f[s] += 1
            if j == head and fnext[j] == M:
                loss_t = end + loss_ms
        else:
            bwd[j][m] = (start, end)
            bnext[j] -= 1
            done_b[s] += 1
        got[s][kind].append(j)
        if orders is not None:
            pos[s][kind] += 1
        send(kind, j, m, end)
        n += 1
    stage_end = [free[s] + wgrad[s] + opt[s] for s in range(S)]
    busy = [M * sum(costs[j].fwd + costs[j].bwd for j in segs[s]) + wgrad[s] + opt[s] for s in range(S)]
    return Timeline(max(stage_end), fwd, bwd, stage_end, busy, got, link_busy, link_bytes)


# ------------------------------------------------------------------------------------ cost model
def boundary_bytes(depth: int, widths: Sequence[int], mid_width: int, mb: int, h: int, w: int,
                   dtype_bytes: int = 2) -> Dict[str, Tuple[int, int, int]]:
    """(producer block, consumer block, bytes per microbatch) of every tensor that can cross a cut:
    the x between consecutive blocks and the skip of each encoder level."""
    out = {}
    H, W = h, w
    for lvl, wd in enumerate(widths):
        out[f"skip{lvl}"] = (lvl, depth + 1 + (depth - 1 - lvl), mb * wd * H * W * dtype_bytes)
        H, W = H // 2, W // 2
        out[f"x{lvl}"] = (lvl, lvl + 1, mb * wd * H * W * dtype_bytes)      # pooled -> next block
    out[f"x{depth}"] = (depth, depth + 1, mb * mid_width * H * W * dtype_bytes)   # mid -> dec0
    for i, wd in enumerate(reversed(widths)):
        H, W = H * 2, W * 2
        out[f"x{depth + 1 + i}"] = (depth + 1 + i, depth + 2 + i, mb * wd * H * W * dtype_bytes)
    return out


def unit_boundary_bytes(depth: int, widths: Sequence[int], mid_width: int, mb: int, h: int, w: int,
                        dtype_bytes: int = 2) -> Dict[str, Tuple[int, int, int]]:
    """:func:`boundary_bytes` in half-block UNIT space (unit 2b = part a of block b, 2b+1 = part b, the
    head is the last unit): x leaves a block from its part b and enters the next block's part a, a skip
    leaves its encoder block's part b and enters its decoder block's part a, and inside every block the
    first conv's output goes from part a to part b."""
    nb = 2 * depth + 2
    out = {}
    for name, (p, c, nbytes) in boundary_bytes(depth, widths, mid_width, mb, h, w, dtype_bytes).items():
        out[name] = (2 * p + 1, 2 * c, nbytes)
    H, W = h, w
    for lvl, wd in enumerate(widths):                       # encoder first-conv outputs
        out[f"a{lvl}"] = (2 * lvl, 2 * lvl + 1, mb * wd * H * W * dtype_bytes)
        H, W = H // 2, W // 2
    out[f"a{depth}"] = (2 * depth, 2 * depth + 1, mb * mid_width * H * W * dtype_bytes)
    for i, wd in enumerate(reversed(widths)):               # decoder first-conv outputs
        H, W = H * 2, W * 2
        b = depth + 1 + i
        out[f"a{b}"] = (2 * b, 2 * b + 1, mb * wd * H * W * dtype_bytes)
    assert all(c <= 2 * (nb - 1) for _, c, _ in out.values())
    return out


def unit_table(table: dict) -> dict:
    """The half-block UNIT view of a block-time table (``per_mb[..]["units"]``, tools/block_times.py):
    every block but the head becomes two units (part a / part b of its DoubleConv), so placements may
    cut between the two convs."""
    t = dict(table)
    t["per_mb"] = {mb: row["units"] for mb, row in table["per_mb"].items() if "units" in row}
    if not t["per_mb"]:
        raise ValueError("table has no half-block unit times (tools/block_times.py round 4+)")
    nbk = len(next(iter(table["per_mb"].values()))["fwd"])
    opt = table.get("opt_ms", [0.0] * nbk)
    t["opt_ms"] = [v / 2 for v in opt[:-1] for _ in (0, 1)] + [opt[-1]]
    t["unit_space"] = True
    t["block_table"] = table            # the single-GPU step (efficiency basis) stays the whole-block one
    return t


def block_to_unit(pos: float, nblocks: int) -> int:
    """Cut position in blocks (``b + 0.5`` = inside block b; ``nblocks`` = the end) -> unit index."""
    return 2 * nblocks - 1 if pos == nblocks else int(round(2 * pos))


def unit_to_block(u: int, nblocks: int):
    return nblocks if u == 2 * nblocks - 1 else (u // 2 if u % 2 == 0 else u / 2)


class CostTable:
    """Per-microbatch cost of any unit range [a, b) of a block-time table (tools/block_times.py).

    In unit space a block whose two halves fall in one range costs its measured whole-block time; only a
    block a cut splits is priced from its half-block units (the halves lose the block's fusions)."""

    def __init__(self, table: dict, mb: int, M: int, defer: bool = True):
        self.table = table
        self.unit_space = bool(table.get("unit_space"))
        self.row = table["per_mb"][str(mb)]
        self.big = table["per_mb"].get(str(mb * M))
        if self.unit_space:
            bt = table["block_table"]
            self.brow, self.bbig = bt["per_mb"][str(mb)], bt["per_mb"].get(str(mb * M))
            self.nbk = len(self.brow["fwd"])
        else:
            self.nbk = len(self.row["fwd"])
        self.U = len(self.row["fwd"])           # units (or blocks) in this table's index space
        self.M, self.defer = M, defer
        self.opt = table.get("opt_ms", [0.0] * self.U)
        self._memo: Dict[Tuple[int, int], Tuple[float, float, float, float]] = {}

    def pos(self, u: int):
        """Index -> block position."""
        return unit_to_block(u, self.nbk) if self.unit_space else u

    def idx(self, p) -> int:
        return block_to_unit(p, self.nbk) if self.unit_space else int(p)

    def range(self, a: int, b: int) -> Tuple[float, float, float, float]:
        """(fwd, bwd, deferred wgrad, opt) ms of index range [a, b)."""
        key = (a, b)
        if key in self._memo:
            return self._memo[key]
        items, u = [], a
        while u < b:
            if self.unit_space and u % 2 == 0 and u + 1 < b and u // 2 < self.nbk - 1:
                items.append((self.brow, self.bbig, u // 2))
                u += 2
            else:
                items.append((self.row, self.big, u))
                u += 1
        f = sum(r["fwd"][i] for r, _, i in items)
        if self.defer:
            bw = sum(r["bwd_nowgrad"][i] for r, _, i in items)
            wg = sum((bg["bwd"][i] - bg["bwd_nowgrad"][i]) if bg is not None
                     else self.M * (r["bwd"][i] - r["bwd_nowgrad"][i]) for r, bg, i in items)
        else:
            bw = sum(r["bwd"][i] for r, _, i in items)
            wg = 0.0
        op = sum(self.opt[i] for i in range(a, b))
        out = (f, bw, max(wg, 0.0), op)
        self._memo[key] = out
        return out


def placement_costs(table: dict, pl: Placement, mb: int, M: int, defer: bool = True):
    """(segment costs, per-stage deferred weight-gradient ms, per-stage optimizer ms, edge bytes)."""
    ct = CostTable(table, mb, M, defer)
    costs, wg, op = [], [0.0] * pl.S, [0.0] * pl.S
    for j in range(pl.K):
        a, b = pl.seg_range(j)
        f, bw, w_, o_ = ct.range(ct.idx(a), ct.idx(b))
        costs.append(SegCost(f, bw))
        wg[pl.owner[j]] += w_
        op[pl.owner[j]] += o_
    h, w = table["img"]
    eb = edge_bytes(pl, table["depth"], table["widths"], table["mid_width"], mb, h, w)
    return costs, wg, op, eb


def simulate_table(table: dict, pl: Placement, mb: int, M: int, defer: bool = True, orders=None,
                   policy: str = "further", **link) -> Timeline:
    costs, wg, op, eb = placement_costs(table, pl, mb, M, defer)
    return simulate_placement(pl, table["depth"], M, costs, eb, wg, op, orders=orders, policy=policy, **link)


def single_device_ms(table: dict, batch: int) -> Optional[float]:
    """Measured single-stage step of the whole batch (sum of blocks + optimizer), if the table has it."""
    if "block_table" in table:
        table = table["block_table"]
    row = table["per_mb"].get(str(batch))
    if row is not None:
        return sum(row["fwd"]) + sum(row["bwd"]) + sum(table.get("opt_ms", []))
    big = max(int(k) for k in table["per_mb"])
    if batch > big and batch % big == 0:
        # beyond the largest measured batch the single-GPU rate is flat (b256 vs b512 within 1 %):
        # scale the largest measured step per image
        r = table["per_mb"][str(big)]
        return (sum(r["fwd"]) + sum(r["bwd"])) * batch / big + sum(table.get("opt_ms", []))
    return None


# ------------------------------------------------------------------------------------ search
def _minmax_dp(ct: CostTable, S: int, M: int, kind: str) -> List[int]:
    """Index cuts minimising the largest stage busy time M (f + b) + wgrad + opt (no transfers):
    contiguous (S segments) or mirrored (2S-1 segments, stage s = segments s and 2S-2-s)."""
    U = ct.U
    T = [[0.0] * (U + 1) for _ in range(U + 1)]
    for a in range(U):
        for b in range(a + 1, U + 1):
            f, bw, wg, op = ct.range(a, b)
            T[a][b] = M * (f + bw) + wg + op
    INF = float("inf")
    if kind == "contiguous":
        best = [[INF] * (U + 1) for _ in range(S + 1)]
        arg = [[0] * (U + 1) for _ in range(S + 1)]
        best[0][0] = 0.0
        for s in range(1, S + 1):
            for j in range(s, U + 1):
                for i in range(s - 1, j):
                    v = max(best[s - 1][i], T[i][j])
                    if v < best[s][j]:
                        best[s][j], arg[s][j] = v, i
        cuts, j = [U], U
        for s in range(S, 0, -1):
            j = arg[s][j]
            cuts.append(j)
        return list(reversed(cuts))
    # mirrored: F[k][(i, j)] = best max over stages k.. given left boundary i, right boundary j
    from functools import lru_cache

    @lru_cache(maxsize=None)
    def F(k, i, j):
        if k == S - 1:
            return (T[i][j], ())
        best = (INF, ())
        rem = S - 1 - k            # stages still to place inside (i', j')
        for i2 in range(i + 1, j):
            for j2 in range(j - 1, i2, -1):
                if j2 - i2 < 1 or i2 - i < 1 or j - j2 < 1:
                    continue
                if j2 - i2 < rem:   # each inner stage needs >= 1 unit (the bottom one), the others 2
                    continue
                c = T[i][i2] + T[j2][j]
                if c >= best[0]:
                    continue
                sub = F(k + 1, i2, j2)
                v = max(c, sub[0])
                if v < best[0]:
                    best = (v, ((i2, j2),) + sub[1])
        return best

    v, path = F(0, 0, U)
    if v == INF:
        raise ValueError(f"no mirrored placement of {S} stages over {U} units")
    left = [0] + [p[0] for p in path]
    right = [p[1] for p in reversed(path)] + [U]
    return left + right


def _to_placement(ct: CostTable, idx_cuts: Sequence[int], kind: str) -> Placement:
    cuts = [ct.pos(u) for u in idx_cuts]
    return Placement.mirrored(cuts) if kind == "v" else Placement.contiguous(cuts)


def mirrored_starts(depth: int, S: int, half: bool = True):
    """Skip-local V placements: stage s owns encoder range [L_s, L_{s+1}) and the decoder blocks of the
    SAME levels, so no skip leaves its GPU.  A left cut at block position p (a half position = inside
    the encoder block) mirrors to 2D+1-p on the decoder side (encoder level l <-> decoder block 2D-l; a
    cut inside enc_l after its first conv keeps enc_l's skip with the lower stage, whose decoder part a
    then also stays there).  Yields cut lists in block positions."""
    import itertools
    step = 0.5 if half else 1.0
    left = [p * step for p in range(1, int((depth + 1) / step))]       # (0, D+1): encoder + mid side
    for inner in itertools.combinations(left, S - 1):
        right = [2 * depth + 1 - p for p in reversed(inner)]
        cuts = [0, *inner, *right, 2 * depth + 2]
        if all(b > a for a, b in zip(cuts, cuts[1:])):
            yield cuts


def _local_search(table, ct: CostTable, idx_cuts: List[int], kind: str, mb: int, M: int, sim_kw,
                  tl0: Optional[Timeline] = None) -> Tuple[List[int], Timeline]:
    def evaluate(c):
        try:
            pl = _to_placement(ct, c, kind)
            pl.validate(table["depth"])
        except ValueError:
            return None
        return simulate_table(table, pl, mb, M, **sim_kw)

    cur = list(idx_cuts)
    tl = tl0 or evaluate(cur)
    improved = True
    while improved and tl is not None:
        improved = False
        for k in range(1, len(cur) - 1):
            for d in (-2, -1, 1, 2):
                c = list(cur)
                c[k] += d
                if not (c[k - 1] < c[k] < c[k + 1]):
                    continue
                t2 = evaluate(c)
                if t2 is not None and t2.step_ms < tl.step_ms - 1e-9:
                    cur, tl, improved = c, t2, True
    return cur, tl


def search(table: dict, S: int, batch: int, kind: str = "v", Ms: Optional[Sequence[int]] = None,
           policies: Sequence[str] = ("feed", "further"), top: int = 3, **link) -> List[dict]:
    """Best placement of ``kind`` (``contiguous`` | ``v``) for every microbatch count M (from ``Ms`` or
    every count the table's microbatch sizes allow).  Starts: the min-max DP over stage busy times and,
    for ``v``, every skip-local mirrored placement (:func:`mirrored_starts`), each simulated with both
    op-order policies; the ``top`` best starts are refined by a local search over single-cut moves."""
    t1 = single_device_ms(table, batch)
    out = []
    sizes = sorted(int(k) for k in table["per_mb"])
    depth = table["depth"]
    for M in (Ms or sorted({batch // k for k in sizes if batch % k == 0})):
        mb = batch // M
        if str(mb) not in table["per_mb"]:
            continue
        ct = CostTable(table, mb, M)
        starts = [_minmax_dp(ct, S, M, kind)]
        if kind == "v":
            starts += [[ct.idx(p) for p in c] for c in mirrored_starts(depth, S, half=bool(table.get("unit_space")))]
        scored = []
        seen = set()
        for c in starts:
            if tuple(c) in seen:
                continue
            seen.add(tuple(c))
            try:
                pl = _to_placement(ct, c, kind).validate(depth)
            except ValueError:
                continue
            for policy in policies:
                tl = simulate_table(table, pl, mb, M, policy=policy, **link)
                scored.append((tl.step_ms, c, policy, tl))
        scored.sort(key=lambda r: r[0])
        best = None
        for _, c, policy, tl in scored[:top]:
            cuts, tl2 = _local_search(table, ct, c, kind, mb, M, dict(link, policy=policy), tl)
            if best is None or tl2.step_ms < best[2].step_ms:
                best = (cuts, policy, tl2)
        if best is None:
            continue
        cuts, policy, tl = best
        out.append(plan_row(_to_placement(ct, cuts, kind), tl, batch, M, t1, policy))
    return out


def plan_row(pl: Placement, tl: Timeline, batch: int, M: int, t1: Optional[float], policy: str) -> dict:
    r = {"stages": pl.S, "microbatches": M, "mb": batch // M, "placement": pl.kind, "cuts": list(pl.cuts),
         "owner": list(pl.owner), "policy": policy, "step_ms": round(tl.step_ms, 3),
         "img_s": round(batch * 1000.0 / tl.step_ms, 1), "utilisation": round(tl.efficiency(), 3),
         "max_link_busy_ms": round(max(tl.link_busy.values()), 3) if tl.link_busy else 0.0,
         "max_link_gb": round(max(tl.link_bytes.values()) / 1e9, 3) if tl.link_bytes else 0.0}
    if t1 is not None:
        r["speedup_vs_1gpu"] = round(t1 / tl.step_ms, 3)
        r["scaling_efficiency"] = round(t1 / tl.step_ms / pl.S, 3)
    return r


def evaluate_placement(table: dict, pl: Placement, batch: int, Ms: Optional[Sequence[int]] = None,
                       policy: str = "further", **link) -> List[dict]:
    """Simulated rows of a FIXED placement (e.g. the reference cut) at every microbatch count."""
    t1 = single_device_ms(table, batch)
    out = []
    sizes = sorted(int(k) for k in table["per_mb"])
    for M in (Ms or sorted({batch // k for k in sizes if batch % k == 0})):
        mb = batch // M
        if str(mb) not in table["per_mb"]:
            continue
        tl = simulate_table(table, pl, mb, M, policy=policy, **link)
        out.append(plan_row(pl, tl, batch, M, t1, policy))
    return out


def load_table(path: str) -> dict:
    with open(path) as f:
        return json.load(f)


# ------------------------------------------------------------------------------------ chosen plans
PLANS_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "plans.json")


def plan_key(model: str, h: int, w: int, stages: int, batch: int) -> str:
    return f"{model}:{h}x{w}:{stages}:{batch}"


def load_plan(model: str, h: int, w: int, stages: int, batch: int, path: str = None,
              depth: Optional[int] = None) -> Optional[dict]:
    """The plan tools/pipeline_plan.py chose for this (model, image, stages, global batch):
    {"placement": Placement, "microbatches", "policy", "predicted_img_s", ...}, or None.  The placement
    is validated against the model (``depth``; looked up from the preset when not given): its stage
    count, last cut == the head's end, no cut inside the head, microbatches dividing the batch."""
    path = path or PLANS_PATH
    if not os.path.exists(path):
        return None
    with open(path) as f:
        plans = json.load(f)
    key = plan_key(model, h, w, stages, batch)
    p = plans.get(key)
    if p is None:
        return None
    if depth is None:
        from ..models.unet import PRESETS
        depth = PRESETS[model].depth if model in PRESETS else None
    try:
        if p.get("spatial"):                     # row-split top levels (parallel/spatial.py)
            from .spatial import SpatialPlan
            pl = SpatialPlan.from_plan(p)
        else:
            pl = Placement.from_plan(p)
        if depth is not None:
            pl.validate(depth)
        M = int(p["microbatches"])
        if pl.S != stages or M < 1 or batch % M:
            raise ValueError(f"{pl.S} stages / {M} microbatches")
    except (ValueError, KeyError, TypeError) as e:
        raise ValueError(f"malformed pipeline plan {key}: {p} ({e})") from e
    cuts = list(pl.cuts) if hasattr(pl, "cuts") else list(pl.inner_cuts)
    return dict(p, placement=pl, cuts=cuts, microbatches=M)
