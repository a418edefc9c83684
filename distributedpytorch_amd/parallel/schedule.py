"""GPipe schedule model and time-balanced stage partitioner.

The pipeline engine (:class:`.pipeline.GPipeDist`, reference ``model/unet_model.py:24-53`` generalised
to S stages x M microbatches) runs ALL forwards, then ALL backwards: the loss is the reference's
global Dice over the whole batch, so no microbatch's backward can start before every microbatch's
forward has reached the head.  Its step time is therefore not the ideal ``M (F + B)`` of the slowest
stage but a fill / drain schedule, and the stage boundaries that minimise it depend on measured
per-block TIME, not FLOPs (the full-resolution levels run at ~0.6 PF on MI355X, the deep GEMMs at
1.3-1.5 PF).  This module

* simulates that schedule (:func:`simulate`) from per-stage costs: forward / backward per microbatch,
  the deferred weight gradients (:class:`..models.hip_unet.HipBlocks` merges every microbatch's
  weight gradient of a layer into one launch after the layer's last microbatch -- work that runs in
  the drain, after the stage's last backward), and point-to-point transfer times of the boundary
  tensors (x and the UNet skips go straight from producer to consumer stage over xGMI);
* builds stage costs from a measured per-block time table (``tools/block_times.py`` on one GPU,
  JSON in ``profiles/``) and a transfer model (:func:`stage_costs`);
* searches every contiguous partition for the one with the smallest simulated step
  (:func:`best_partition`) and the microbatch count that maximises throughput (:func:`plan`).

Dependencies modelled (they are exactly GPipeDist.train_step's):
  forward  (s, m): after (s, m-1) and after every producer stage p of s has finished (p, m) and its
                   tensors arrived (x from s-1, each skip from the stage that ran its encoder level);
  backward (s, m), m = M-1 .. 0: after (s, m+1) [for m = M-1: after the stage's last forward; the
                   last stage also after the loss], and after every consumer stage c has finished
                   backward (c, m) and its gradient arrived;
  the stage ends after its last backward plus its deferred weight gradients (work-conserving: they
  share the CUs with the last microbatch's dgrads, so they extend the stage by their own time);
  the step ends when every stage has run its optimizer step.
Communication is asynchronous (RCCL on its own streams) and does not delay the sender's compute.
"""
from __future__ import annotations

import itertools
import json
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple


@dataclass
class StageCost:
    fwd: float                  # ms per microbatch forward
    bwd: float                  # ms per microbatch backward (dgrads + weight gradients not deferred)
    wgrad: float = 0.0          # ms of the deferred (merged over all microbatches) weight gradients
    opt: float = 0.0            # ms of the stage's optimizer step
    # transfer ms per microbatch: forward activations / skips to consumer stage c, gradients to producer p
    xfer_fwd: Dict[int, float] = field(default_factory=dict)
    xfer_bwd: Dict[int, float] = field(default_factory=dict)


@dataclass
class Timeline:
    step_ms: float
    fwd: List[List[Tuple[float, float]]]     # [stage][microbatch] -> (start, end)
    bwd: List[List[Tuple[float, float]]]
    stage_end: List[float]
    busy_ms: List[float]                     # compute time per stage

    def efficiency(self) -> float:
        """Mean stage utilisation: sum of stage busy time / (stages x step)."""
        return sum(self.busy_ms) / (len(self.busy_ms) * self.step_ms)


def simulate(costs: Sequence[StageCost], M: int, loss_ms: float = 0.0) -> Timeline:
    """Simulate one all-forward / all-backward GPipe step (see the module docstring)."""
    S = len(costs)
    producers = [sorted(p for p in range(S) if s in costs[p].xfer_fwd) for s in range(S)]
    consumers = [sorted(costs[s].xfer_fwd) for s in range(S)]
    fwd = [[(0.0, 0.0)] * M for _ in range(S)]
    bwd = [[(0.0, 0.0)] * M for _ in range(S)]
    # forward: producers always have lower stage indices, so stage order is a topological order
    for s in range(S):
        t = 0.0
        for m in range(M):
            start = t
            for p in producers[s]:
                start = max(start, fwd[p][m][1] + costs[p].xfer_fwd[s])
            end = start + costs[s].fwd
            fwd[s][m] = (start, end)
            t = end
    # backward: consumers have higher indices -> reverse stage order
    for s in reversed(range(S)):
        t = fwd[s][M - 1][1] + (loss_ms if s == S - 1 else 0.0)
        for m in reversed(range(M)):
            start = t
            for c in consumers[s]:
                start = max(start, bwd[c][m][1] + costs[c].xfer_bwd[s])
            end = start + costs[s].bwd
            bwd[s][m] = (start, end)
            t = end
    stage_end = [bwd[s][0][1] + costs[s].wgrad + costs[s].opt for s in range(S)]
    busy = [M * (c.fwd + c.bwd) + c.wgrad + c.opt for c in costs]
    return Timeline(max(stage_end), fwd, bwd, stage_end, busy)


# ------------------------------------------------------------------------------------ cost model
def _stage_of(idx: int, cuts: Sequence[int]) -> int:
    for s in range(len(cuts) - 1):
        if cuts[s] <= idx < cuts[s + 1]:
            return s
    raise ValueError(idx)


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
    every block but the head becomes two units (part a / part b of its DoubleConv), so partitions may
    cut between the two convs.  Cuts found on it are unit indices; :func:`plan` reports them as block
    positions (unit u -> u / 2: ``b + 0.5`` = inside block b)."""
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


def stage_costs(table: dict, mb: int, M: int, cuts: Sequence[int], link_gbs: float = 100.0,
                link_latency_ms: float = 0.015, defer: bool = True) -> List[StageCost]:
    """Stage costs of partition ``cuts`` at microbatch ``mb`` (M microbatches) from a block time table.

    ``table``: {"depth", "widths", "mid_width", "img": [h, w], "per_mb": {str(mb): {"fwd": [...],
    "bwd": [...], "bwd_nowgrad": [...]}}, "opt_ms": [...]} (ms per block, tools/block_times.py).
    With ``defer`` the stage's weight gradients are merged over the M microbatches (one launch per
    layer, measured at the full step's image count M*mb when the table has it, else scaled)."""
    depth, widths, mid_width = table["depth"], table["widths"], table["mid_width"]
    h, w = table["img"]
    row = table["per_mb"][str(mb)]
    big = table["per_mb"].get(str(mb * M))
    S = len(cuts) - 1
    unit_space = bool(table.get("unit_space"))
    if unit_space:       # a block whose two halves share a stage costs its measured whole-block time
        bt = table["block_table"]
        brow, bbig = bt["per_mb"][str(mb)], bt["per_mb"].get(str(mb * M))
        nbk = len(brow["fwd"])
    costs = []
    for s in range(S):
        items, u = [], cuts[s]
        while u < cuts[s + 1]:
            if unit_space and u % 2 == 0 and u + 1 < cuts[s + 1] and u // 2 < nbk - 1:
                items.append((brow, bbig, u // 2))
                u += 2
            else:
                items.append((row, big, u))
                u += 1
        f = sum(r["fwd"][i] for r, _, i in items)
        if defer:
            b = sum(r["bwd_nowgrad"][i] for r, _, i in items)
            wg = sum((bg["bwd"][i] - bg["bwd_nowgrad"][i]) if bg is not None else M * (r["bwd"][i] - r["bwd_nowgrad"][i])
                     for r, bg, i in items)
        else:
            b = sum(r["bwd"][i] for r, _, i in items)
            wg = 0.0
        opt = sum(table.get("opt_ms", [0.0] * len(row["fwd"]))[i] for i in range(cuts[s], cuts[s + 1]))
        costs.append(StageCost(f, b, max(wg, 0.0), opt))
    bfun = unit_boundary_bytes if table.get("unit_space") else boundary_bytes
    for name, (pb, cb, nbytes) in bfun(depth, widths, mid_width, mb, h, w).items():
        if pb >= len(table["per_mb"][str(mb)]["fwd"]) or cb >= len(table["per_mb"][str(mb)]["fwd"]):
            continue
        ps, cs = _stage_of(pb, cuts), _stage_of(cb, cuts)
        if ps == cs:
            continue
        ms = link_latency_ms + nbytes / (link_gbs * 1e6)
        # several tensors to the same peer travel in one grouped launch: bytes add, latency once
        costs[ps].xfer_fwd[cs] = costs[ps].xfer_fwd.get(cs, link_latency_ms) + ms - link_latency_ms
        costs[cs].xfer_bwd[ps] = costs[cs].xfer_bwd.get(ps, link_latency_ms) + ms - link_latency_ms
    return costs


def single_device_ms(table: dict, batch: int) -> Optional[float]:
    """Measured single-stage step of the whole batch (sum of blocks + optimizer), if the table has it."""
    if "block_table" in table:
        table = table["block_table"]
    row = table["per_mb"].get(str(batch))
    if row is None:
        return None
    return sum(row["fwd"]) + sum(row["bwd"]) + sum(table.get("opt_ms", []))


def partitions(nblocks: int, S: int):
    """Every contiguous split of ``nblocks`` blocks into S non-empty stages (cut lists)."""
    for inner in itertools.combinations(range(1, nblocks), S - 1):
        yield [0, *inner, nblocks]


def best_partition(table: dict, S: int, mb: int, M: int, **kw) -> Tuple[List[int], Timeline]:
    nb = len(table["per_mb"][str(mb)]["fwd"])
    best = None
    for cuts in partitions(nb, S):
        tl = simulate(stage_costs(table, mb, M, cuts, **kw), M)
        if best is None or tl.step_ms < best[1].step_ms:
            best = (cuts, tl)
    return best


def plan(table: dict, S: int, batch: int, cuts: Optional[Sequence[int]] = None, **kw) -> List[dict]:
    """For every microbatch count M whose microbatch size the table has: the best (or the given)
    partition, its simulated step, img/s and efficiency against the measured single-stage step."""
    out = []
    t1 = single_device_ms(table, batch)
    units = bool(table.get("unit_space"))
    nbk = len(next(iter(table["block_table"]["per_mb"].values()))["fwd"]) if units else None
    for M in sorted({batch // int(k) for k in table["per_mb"] if batch % int(k) == 0 and batch // int(k) >= 1}):
        mb = batch // M
        if cuts is None:
            c, tl = best_partition(table, S, mb, M, **kw)
        else:
            uc = [block_to_unit(p, nbk) for p in cuts] if units else list(cuts)
            c, tl = list(cuts), simulate(stage_costs(table, mb, M, uc, **kw), M)
        if units and cuts is None:
            c = [unit_to_block(u, nbk) for u in c]          # unit index -> block position (b + 0.5: inside block b)
        r = {"stages": S, "microbatches": M, "mb": mb, "cuts": c, "step_ms": round(tl.step_ms, 3),
             "img_s": round(batch * 1000.0 / tl.step_ms, 1), "utilisation": round(tl.efficiency(), 3)}
        if t1 is not None:
            r["speedup_vs_1gpu"] = round(t1 / tl.step_ms, 3)
            r["scaling_efficiency"] = round(t1 / tl.step_ms / S, 3)
        out.append(r)
    return out


def load_table(path: str) -> dict:
    with open(path) as f:
        return json.load(f)


# ------------------------------------------------------------------------------------ chosen plans
PLANS_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "plans.json")


def plan_key(model: str, h: int, w: int, stages: int, batch: int) -> str:
    return f"{model}:{h}x{w}:{stages}:{batch}"


def load_plan(model: str, h: int, w: int, stages: int, batch: int, path: str = None) -> Optional[dict]:
    """The time-balanced plan tools/pipeline_plan.py chose from measured block times for this
    (model, image, stages, global batch): {"cuts", "microbatches", "predicted_img_s", ...}, or None."""
    path = path or PLANS_PATH
    if not os.path.exists(path):
        return None
    with open(path) as f:
        plans = json.load(f)
    p = plans.get(plan_key(model, h, w, stages, batch))
    if p is None:
        return None
    cuts = [int(c) if float(c) == int(c) else float(c) for c in p["cuts"]]     # b + 0.5: a cut inside block b
    M = int(p["microbatches"])
    if (len(cuts) != stages + 1 or cuts[0] != 0 or any(b <= a for a, b in zip(cuts, cuts[1:])) or batch % M
            or any(c * 2 != int(c * 2) for c in cuts)):
        raise ValueError(f"malformed pipeline plan {plan_key(model, h, w, stages, batch)}: {p}")
    return dict(p, cuts=cuts, microbatches=M)
