"""GPipe schedule model (parallel/schedule.py) against hand-computed timelines, and the
time-balanced partitioner on a synthetic block-time table (CPU only)."""
import os

import pytest

from distributedpytorch_amd.parallel.schedule import (StageCost, best_partition, boundary_bytes, partitions,
                                                      plan, simulate, stage_costs)


def test_two_stage_hand_computed():
    # F = (1, 2), B = (2, 3), M = 2, no transfers:
    #   s0 fwd m0 [0,1] m1 [1,2]; s1 fwd m0 [1,3] m1 [3,5]
    #   s1 bwd m1 [5,8] m0 [8,11]; s0 bwd m1 [max(2,8)=8,10] m0 [max(10,11)=11,13]
    c = [StageCost(1, 2, xfer_fwd={1: 0.0}), StageCost(2, 3, xfer_bwd={0: 0.0})]
    tl = simulate(c, 2)
    assert tl.fwd == [[(0, 1), (1, 2)], [(1, 3), (3, 5)]]
    assert tl.bwd == [[(11, 13), (8, 10)], [(8, 11), (5, 8)]]
    assert tl.step_ms == 13
    # the first stage's deferred weight gradients run in its drain: 13 + 1
    c[0].wgrad = 1.0
    assert simulate(c, 2).step_ms == 14
    # transfers delay the consumer: x arrives 0.5 after the producer's forward ends
    c = [StageCost(1, 2, xfer_fwd={1: 0.5}), StageCost(2, 3, xfer_bwd={0: 0.5})]
    tl = simulate(c, 2)
    assert tl.fwd[1] == [(1.5, 3.5), (3.5, 5.5)]
    assert tl.bwd[0] == [(12.0, 14.0), (9.0, 11.0)]      # s1 bwd m1 [5.5,8.5] m0 [8.5,11.5]


def test_four_stage_uniform_matches_gpipe_formula():
    # F = 1, B = 2 everywhere, M = 2: (M + S - 1)(F + B) = 15; stage 0 also feeds stage 3 (a skip)
    c = [StageCost(1, 2, xfer_fwd={1: 0.0, 3: 0.0}), StageCost(1, 2, xfer_fwd={2: 0.0}, xfer_bwd={0: 0.0}),
         StageCost(1, 2, xfer_fwd={3: 0.0}, xfer_bwd={1: 0.0}), StageCost(1, 2, xfer_bwd={2: 0.0, 0: 0.0})]
    tl = simulate(c, 2)
    assert tl.step_ms == 15
    assert tl.bwd[0] == [(13, 15), (11, 13)]
    assert abs(tl.efficiency() - 2 / 5) < 1e-12
    for M in (1, 4, 8, 32):
        assert abs(simulate(c, M).efficiency() - M / (M + 3)) < 1e-12


def _table():
    # depth 2 UNet (6 blocks); uneven block times; per_mb 1, 2, 4
    depth, widths, mid = 2, [8, 16], 32
    base_f = [4.0, 2.0, 1.0, 2.0, 4.0, 0.5]
    per = {}
    for mb in (1, 2, 4):
        f = [v * mb for v in base_f]
        per[str(mb)] = {"fwd": f, "bwd": [2 * v for v in f], "bwd_nowgrad": [1.5 * v for v in f]}
    return {"depth": depth, "widths": widths, "mid_width": mid, "img": [32, 32], "per_mb": per,
            "opt_ms": [0.0] * 6}


def test_boundary_bytes_shapes():
    b = boundary_bytes(2, [8, 16], 32, 1, 32, 32)
    assert b["skip0"] == (0, 4, 8 * 32 * 32 * 2) and b["skip1"] == (1, 3, 16 * 16 * 16 * 2)
    assert b["x0"] == (0, 1, 8 * 16 * 16 * 2) and b["x2"] == (2, 3, 32 * 8 * 8 * 2)
    assert b["x4"] == (4, 5, 8 * 32 * 32 * 2)


def test_time_partition_beats_flop_like_cut():
    t = _table()
    assert sum(1 for _ in partitions(6, 3)) == 10
    cuts, tl = best_partition(t, 2, 1, 4, link_gbs=1e9)
    # brute force over the simulator: no other 2-stage cut is faster
    for c in partitions(6, 2):
        assert simulate(stage_costs(t, 1, 4, c, link_gbs=1e9), 4).step_ms >= tl.step_ms - 1e-9
    assert cuts == [0, 3, 6]            # 7 | 6.5 forward ms: the balanced-by-time cut
    rows = plan(t, 2, 4, link_gbs=1e9)
    assert [r["microbatches"] for r in rows] == [1, 2, 4]
    assert rows[-1]["step_ms"] < rows[0]["step_ms"]   # more microbatches: smaller bubble
    assert all(0 < r["scaling_efficiency"] <= 1 for r in rows)


def test_deferred_wgrad_accounting():
    t = _table()
    a = stage_costs(t, 1, 4, [0, 3, 6], defer=True)
    b = stage_costs(t, 1, 4, [0, 3, 6], defer=False)
    # same total backward work, split into per-microbatch dgrads + one merged weight-gradient tail
    for x, y in zip(a, b):
        assert x.bwd * 4 + x.wgrad == pytest.approx(y.bwd * 4)


def test_plan_lookup_drives_mp_defaults(tmp_path, monkeypatch):
    """parallel/plans.json (tools/pipeline_plan.py output) sets the MP cut and microbatch count for the
    configurations it covers; others fall back to the reference / FLOP-balanced cut; an explicit
    --microbatches wins; a malformed plan is an error, not a silent default."""
    import json
    from distributedpytorch_amd.config import TrainConfig, mp_plan
    from distributedpytorch_amd.parallel import schedule as sch
    path = tmp_path / "plans.json"
    path.write_text(json.dumps({"unet:512x512:2:256": {"cuts": [0, 4, 10], "microbatches": 8,
                                                       "predicted_img_s": 5000.0}}))
    monkeypatch.setattr(sch, "PLANS_PATH", str(path))
    cfg = TrainConfig(model="unet", img_size=(512, 512), batch_size=256)
    assert mp_plan(cfg, 2) == ("time", [0, 4, 10], 8)
    cfg.microbatches = 4
    assert mp_plan(cfg, 2) == ("time", [0, 4, 10], 4)
    cfg.mp_cut = "reference"
    assert mp_plan(cfg, 2) == ("reference", None, 4)
    cfg = TrainConfig(model="unet", img_size=(512, 512), batch_size=128)        # no plan for this batch
    assert mp_plan(cfg, 2) == ("reference", None, 2)
    assert mp_plan(cfg, 4, default_microbatches=8) == ("balanced", None, 8)
    cfg.mp_cut = "time"
    assert mp_plan(cfg, 2)[0] == "balanced"
    path.write_text(json.dumps({"unet:512x512:2:256": {"cuts": [0, 10, 4], "microbatches": 8}}))
    with pytest.raises(ValueError):
        sch.load_plan("unet", 512, 512, 2, 256)


def test_shipped_plans_are_well_formed():
    import json
    from distributedpytorch_amd.models.blocks import n_blocks
    from distributedpytorch_amd.models.unet import PRESETS
    from distributedpytorch_amd.parallel import schedule as sch
    if not os.path.exists(sch.PLANS_PATH):
        pytest.skip("no plans shipped")
    with open(sch.PLANS_PATH) as f:
        plans = json.load(f)
    for key in plans:
        model, hw, S, batch = key.split(":")
        h, w = map(int, hw.split("x"))
        p = sch.load_plan(model, h, w, int(S), int(batch))
        assert p["cuts"][-1] == n_blocks(PRESETS[model].depth)


def test_unit_space_cuts_inside_doubleconv():
    """Half-block units: unit 2b / 2b+1 = part a / b of block b, the head the last unit; a partition
    found on units is reported in block positions (b + 0.5 = a cut between block b's convs) and
    evaluates to the same step when passed back as cuts; the boundary tensors follow the parts."""
    from distributedpytorch_amd.parallel.schedule import (block_to_unit, unit_boundary_bytes, unit_table,
                                                          unit_to_block)
    nb = 6
    for p in (0, 0.5, 1, 2.5, 5, 6):
        assert unit_to_block(block_to_unit(p, nb), nb) == p
    b = unit_boundary_bytes(2, [8, 16], 32, 1, 32, 32)
    assert b["skip0"] == (1, 8, 8 * 32 * 32 * 2)          # enc0 part b -> dec1 (block 4) part a
    assert b["x2"] == (5, 6, 32 * 8 * 8 * 2)               # mid part b -> dec0 part a
    assert b["a2"] == (4, 5, 32 * 8 * 8 * 2)               # mid's first conv output
    assert b["a4"] == (8, 9, 8 * 32 * 32 * 2)              # dec1's first conv output (full resolution)
    t = _table()
    for row in t["per_mb"].values():
        row["units"] = {k: [v / 2 for v in row[k][:-1] for _ in (0, 1)] + [row[k][-1]] for k in ("fwd", "bwd", "bwd_nowgrad")}
    ut = unit_table(t)
    best = max(plan(ut, 2, 4, link_gbs=1e9), key=lambda r: r["img_s"])
    again = plan(ut, 2, 4, cuts=best["cuts"], link_gbs=1e9)
    assert [r["step_ms"] for r in again if r["microbatches"] == best["microbatches"]] == [best["step_ms"]]
    whole = max(plan(t, 2, 4, link_gbs=1e9), key=lambda r: r["img_s"])
    assert best["step_ms"] <= whole["step_ms"] + 1e-9     # finer cuts can only help the balance


def test_unit_space_prices_uncut_blocks_whole():
    """A block whose two halves share a stage costs its measured whole-block time; only a block that a
    cut splits is priced from its half-block units (the halves lose the block's fusions, so their sum
    is larger than the whole)."""
    from distributedpytorch_amd.parallel.schedule import unit_table
    t = _table()
    for row in t["per_mb"].values():       # halves 30 % dearer than the whole block
        row["units"] = {k: [0.65 * v for v in row[k][:-1] for _ in (0, 1)] + [row[k][-1]]
                        for k in ("fwd", "bwd", "bwd_nowgrad")}
    ut = unit_table(t)
    whole = stage_costs(t, 1, 4, [0, 3, 6], defer=False)
    units = stage_costs(ut, 1, 4, [0, 6, 11], defer=False)           # the same partition in unit space
    assert [c.fwd for c in units] == pytest.approx([c.fwd for c in whole])
    assert [c.bwd for c in units] == pytest.approx([c.bwd for c in whole])
    split = stage_costs(ut, 1, 4, [0, 5, 11], defer=False)           # cut inside block 2 (2.5)
    f = t["per_mb"]["1"]["fwd"]
    assert split[0].fwd == pytest.approx(f[0] + f[1] + 0.65 * f[2])
    assert split[1].fwd == pytest.approx(0.65 * f[2] + f[3] + f[4] + f[5])
