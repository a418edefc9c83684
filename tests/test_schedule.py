"""GPipe schedule model (parallel/schedule.py) against hand-computed timelines -- including FIFO
queueing of transfers on a directed peer link when a transfer outlasts the compute -- the V placement
(parallel/placement.py), and the placement search on block-time tables (CPU only)."""
import json
import os

import pytest

from distributedpytorch_amd.parallel.placement import (Placement, channel_members, describe, parse_placement,
                                                       seg_io, stage_io, v_partition)
from distributedpytorch_amd.parallel.schedule import (CostTable, SegCost, boundary_bytes, edge_bytes,
                                                      evaluate_placement, mirrored_starts, placement_costs,
                                                      search, simulate_placement, unit_table)

NOLAT = dict(link_latency_ms=0.0)


def test_two_stage_hand_computed():
    # F = (1, 2), B = (2, 3), M = 2, no transfer bytes:
    #   s0 fwd m0 [0,1] m1 [1,2]; s1 fwd m0 [1,3] m1 [3,5]
    #   s1 bwd m1 [5,8] m0 [8,11]; s0 bwd m1 [max(2,8)=8,10] m0 [max(10,11)=11,13]
    pl = Placement.contiguous([0, 5, 10])
    tl = simulate_placement(pl, 4, 2, [SegCost(1, 2), SegCost(2, 3)], **NOLAT)
    assert tl.fwd == [[(0, 1), (1, 2)], [(1, 3), (3, 5)]]
    assert tl.bwd == [[(11, 13), (8, 10)], [(8, 11), (5, 8)]]
    assert tl.step_ms == 13
    # the first stage's deferred weight gradients run in its drain: 13 + 1
    assert simulate_placement(pl, 4, 2, [SegCost(1, 2), SegCost(2, 3)], wgrad=[1.0, 0.0], **NOLAT).step_ms == 14


def test_link_queue_fifo_when_transfer_outlasts_compute():
    """2 ms transfers after 1 ms stages (the old model let every transfer start at its
    producer's end, i.e. overlapped messages that physically queue on one link).
      fwd s0: m0 [0,1] m1 [1,2] m2 [2,3]; link 0->1: m0 [1,3] m1 [3,5] m2 [5,7] (queued, not [2,4] / [3,5])
      fwd s1: m0 [3,4] m1 [5,6] m2 [7,8]; loss at 8
      bwd s1: m2 [8,9] m1 [9,10] m0 [10,11]; link 1->0: m2 [9,11] m1 [11,13] m0 [13,15]
      bwd s0: m2 [11,12] m1 [13,14] m0 [15,16]"""
    pl = Placement.contiguous([0, 5, 10])
    eb = {(0, 1): 2_000_000}                        # 2 ms at 1 GB/s
    tl = simulate_placement(pl, 4, 3, [SegCost(1, 1), SegCost(1, 1)], eb, link_gbs=1.0, **NOLAT)
    assert tl.fwd[1] == [(3, 4), (5, 6), (7, 8)]
    assert tl.bwd[1] == [(10, 11), (9, 10), (8, 9)]
    assert tl.bwd[0] == [(15, 16), (13, 14), (11, 12)]
    assert tl.step_ms == 16
    assert tl.link_busy[(0, 1)] == pytest.approx(6.0) and tl.link_busy[(1, 0)] == pytest.approx(6.0)
    # the same transfers, each shorter than the compute, never queue: s1 runs back to back
    tl2 = simulate_placement(pl, 4, 3, [SegCost(1, 1), SegCost(1, 1)], {(0, 1): 500_000}, link_gbs=1.0, **NOLAT)
    assert tl2.fwd[1] == [(1.5, 2.5), (2.5, 3.5), (3.5, 4.5)]


def test_v_placement_hand_computed():
    """V over 2 stages (segments 0 / 1 / 2 on stages 0 / 1 / 0), unit costs, M = 2, 'feed' order
    (forward: the segment that feeds others first; backward: likewise):
      s0 fwd seg0 m0 [0,1] seg0 m1 [1,2] seg2 m0 [2,3] seg2 m1 [3,4]; s1 seg1 m0 [1,2] m1 [2,3]; loss 4
      s0 bwd seg2 m1 [4,5] seg2 m0 [5,6] seg0 m1 [6,7] seg0 m0 [7,8]; s1 seg1 m1 [5,6] m0 [6,7]"""
    pl = Placement.mirrored([0, 2, 7, 10])
    assert pl.owner == (0, 1, 0) and pl.kind == "v" and pl.S == 2
    c = [SegCost(1, 1)] * 3
    tl = simulate_placement(pl, 4, 2, c, policy="feed", **NOLAT)
    assert tl.fwd == [[(0, 1), (1, 2)], [(1, 2), (2, 3)], [(2, 3), (3, 4)]]
    assert tl.bwd == [[(7, 8), (6, 7)], [(6, 7), (5, 6)], [(5, 6), (4, 5)]]
    assert tl.step_ms == 8 and tl.efficiency() == pytest.approx(12 / 16)
    assert tl.orders[0] == {"fwd": [0, 0, 2, 2], "bwd": [2, 2, 0, 0]}
    assert tl.orders[1] == {"fwd": [1, 1], "bwd": [1, 1]}
    # replaying the recorded order reproduces the timeline exactly (the engine issues this order)
    again = simulate_placement(pl, 4, 2, c, orders=tl.orders, **NOLAT)
    assert again.fwd == tl.fwd and again.bwd == tl.bwd
    # an order that waits on its own later op deadlocks, and the model says so
    with pytest.raises(RuntimeError):
        simulate_placement(pl, 4, 2, c, orders=[{"fwd": [2, 2, 0, 0], "bwd": [2, 2, 0, 0]},
                                                {"fwd": [1, 1], "bwd": [1, 1]}], **NOLAT)


def test_v_keeps_skips_local_and_cuts_link_bytes():
    """UNet 512^2 bf16: the reference cut moves all four skips + the bottleneck (31 MiB per image), the
    two-stage V moves the pooled enc1 output down (2 MiB) and the dec1 output up (4 MiB)."""
    MiB = 1 << 20
    ref = Placement.contiguous([0, 5, 10])
    eb = edge_bytes(ref, 4, [32, 64, 128, 256], 512, 1, 512, 512)
    assert eb == {(0, 1): 31 * MiB}
    v = Placement.mirrored([0, 2, 7, 10])
    eb = edge_bytes(v, 4, [32, 64, 128, 256], 512, 1, 512, 512)
    assert {k: b for k, b in eb.items() if v.owner[k[0]] != v.owner[k[1]]} == {(0, 1): 2 * MiB, (1, 2): 4 * MiB}
    assert eb[(0, 2)] == 24 * MiB                       # skips 0 and 1: segment 0 -> 2, both on stage 0
    ins, outs = seg_io(v, 4)
    # skips 0 / 1 are handed from segment 0 to segment 2 on stage 0; 2 / 3 stay inside segment 1
    assert ins[1] == [("x", 0)] and sorted(ins[2]) == [("skip0", 0), ("skip1", 0), ("x", 1)]
    recv, send = stage_io(v, 4)
    assert recv == [[("x", 1)], [("x", 0)]] and send == [[("x", 1)], [("x", 0)]]
    assert describe(v, 4) == ["stage 0: enc0 enc1 dec2 dec3 head", "stage 1: enc2 enc3 mid dec0 dec1"]
    for S in (2, 3, 4):
        for cuts in mirrored_starts(4, S):                # every mirrored start is skip-local
            _, send = stage_io(Placement.mirrored(cuts), 4)
            assert all(n == "x" for o in send for n, _ in o), cuts


def test_channels_have_one_sender():
    v = Placement.mirrored([0, 1, 2, 3, 6, 7, 8, 10])
    mem = channel_members(v, 4)
    ins, outs = seg_io(v, 4)
    for j in range(v.K):
        assert v.owner[j] in mem[j]
        assert {v.owner[c] for _, c in outs[j]} <= set(mem[j]) and {v.owner[p] for _, p in ins[j]} <= set(mem[j])


def test_placement_parse_and_validate():
    assert parse_placement("v:0,2,7,10") == Placement.mirrored([0, 2, 7, 10])
    assert parse_placement("0,5,10@0,1") == Placement.contiguous([0, 5, 10])
    with pytest.raises(ValueError):
        Placement((0, 3, 5, 10), (0, 0, 1))               # adjacent segments on one stage
    with pytest.raises(ValueError):
        Placement.mirrored([0, 2, 7, 9.5, 10])            # even segment count
    with pytest.raises(ValueError):
        Placement.mirrored([0, 2, 7, 9.5]).validate(4)    # ends inside the chain
    with pytest.raises(ValueError):
        Placement.mirrored([0, 2, 7, 10]).validate(3)     # wrong depth


def _table():
    # depth 2 UNet (6 blocks); uneven block times; per_mb 1, 2, 4; units for half-block cuts
    depth, widths, mid = 2, [8, 16], 32
    base_f = [4.0, 2.0, 1.0, 2.0, 4.0, 0.5]
    per = {}
    for mb in (1, 2, 4):
        f = [v * mb for v in base_f]
        row = {"fwd": f, "bwd": [2 * v for v in f], "bwd_nowgrad": [1.5 * v for v in f]}
        row["units"] = {k: [v / 2 for v in row[k][:-1] for _ in (0, 1)] + [row[k][-1]] for k in row}
        per[str(mb)] = row
    return {"model": "unet-tiny", "depth": depth, "widths": widths, "mid_width": mid, "img": [32, 32],
            "per_mb": per, "opt_ms": [0.0] * 6}


def test_search_beats_reference_cut_when_links_are_slow():
    t = _table()
    ref = evaluate_placement(t, Placement.contiguous([0, 3, 6]), 4, link_gbs=1e-4)
    best_v = search(unit_table(t), 2, 4, "v", link_gbs=1e-4)
    r = {x["microbatches"]: x for x in ref}
    for row in best_v:
        assert row["step_ms"] < r[row["microbatches"]]["step_ms"]
        assert row["placement"] == "v"
    # the search result is reproducible by simulating its placement with its policy
    b = min(best_v, key=lambda x: x["step_ms"])
    again = evaluate_placement(unit_table(t), Placement(b["cuts"], b["owner"]), 4, Ms=[b["microbatches"]],
                               policy=b["policy"], link_gbs=1e-4)
    assert again[0]["step_ms"] == b["step_ms"]


def test_contiguous_search_matches_brute_force():
    import itertools
    t = _table()
    for M in (2, 4):
        best = [r for r in search(t, 3, 4, "contiguous", Ms=[M], link_gbs=1e9)][0]
        brute = min(evaluate_placement(t, Placement.contiguous([0, *inner, 6]), 4, Ms=[M], policy=pol,
                                       link_gbs=1e9)[0]["step_ms"]
                    for inner in itertools.combinations(range(1, 6), 2) for pol in ("feed", "further"))
        assert best["step_ms"] == pytest.approx(brute)


def test_deferred_wgrad_accounting():
    t = _table()
    pl = Placement.contiguous([0, 3, 6])
    a, wa, _, _ = placement_costs(t, pl, 1, 4, defer=True)
    b, wb, _, _ = placement_costs(t, pl, 1, 4, defer=False)
    # same total backward work, split into per-microbatch dgrads + one merged weight-gradient tail
    for x, y, w_, w0 in zip(a, b, wa, wb):
        assert x.bwd * 4 + w_ == pytest.approx(y.bwd * 4) and w0 == 0


def test_unit_space_prices_uncut_blocks_whole():
    """A block whose two halves share a segment costs its measured whole-block time; only a block that a
    cut splits is priced from its half-block units (the halves lose the block's fusions)."""
    t = _table()
    for row in t["per_mb"].values():       # halves 30 % dearer than the whole block
        row["units"] = {k: [0.65 * v for v in row[k][:-1] for _ in (0, 1)] + [row[k][-1]]
                        for k in ("fwd", "bwd", "bwd_nowgrad")}
    ut = unit_table(t)
    whole, _, _, _ = placement_costs(t, Placement.contiguous([0, 3, 6]), 1, 4, defer=False)
    units, _, _, _ = placement_costs(ut, Placement.contiguous([0, 3, 6]), 1, 4, defer=False)
    assert [c.fwd for c in units] == pytest.approx([c.fwd for c in whole])
    split, _, _, _ = placement_costs(ut, Placement.contiguous([0, 2.5, 6]), 1, 4, defer=False)
    f = t["per_mb"]["1"]["fwd"]
    assert split[0].fwd == pytest.approx(f[0] + f[1] + 0.65 * f[2])
    assert split[1].fwd == pytest.approx(0.65 * f[2] + f[3] + f[4] + f[5])
    ct = CostTable(ut, 1, 4)
    assert ct.idx(2.5) == 5 and ct.pos(5) == 2.5 and ct.pos(11) == 6


def test_boundary_bytes_shapes():
    b = boundary_bytes(2, [8, 16], 32, 1, 32, 32)
    assert b["skip0"] == (0, 4, 8 * 32 * 32 * 2) and b["skip1"] == (1, 3, 16 * 16 * 16 * 2)
    assert b["x0"] == (0, 1, 8 * 16 * 16 * 2) and b["x2"] == (2, 3, 32 * 8 * 8 * 2)
    assert b["x4"] == (4, 5, 8 * 32 * 32 * 2)


def test_v_partition_is_skip_local_and_covers_all_blocks():
    from distributedpytorch_amd.models.unet import build_model
    for name, S in (("unet", 2), ("unet", 4), ("unet-xl", 8), ("unet-tiny4", 8)):
        cfg = build_model(name).cfg
        pl = v_partition(cfg, S, 512, 512)
        assert pl.S == S and pl.kind == "v"
        _, send = stage_io(pl, cfg.depth)
        assert all(n == "x" for o in send for n, _ in o)


def test_plan_lookup_drives_mp_defaults(tmp_path, monkeypatch):
    """parallel/plans.json (tools/pipeline_plan.py output) sets the MP placement, microbatch count and op
    order for the configurations it covers; others fall back to the skip-local V placement (auto) or the
    reference cut (``--mp-cut reference``, M = 2 as the reference); an explicit --microbatches wins; a
    malformed plan is an error, not a silent default."""
    from distributedpytorch_amd.config import TrainConfig, mp_plan
    from distributedpytorch_amd.parallel import schedule as sch
    path = tmp_path / "plans.json"
    orders = [{"fwd": [0] * 8 + [2] * 8, "bwd": [2] * 8 + [0] * 8}, {"fwd": [1] * 8, "bwd": [1] * 8}]
    path.write_text(json.dumps({"unet:512x512:2:256": {"cuts": [0, 2, 7, 10], "owner": [0, 1, 0], "microbatches": 8,
                                                       "policy": "feed", "orders": orders,
                                                       "predicted_img_s": 5000.0}}))
    monkeypatch.setattr(sch, "PLANS_PATH", str(path))
    cfg = TrainConfig(model="unet", img_size=(512, 512), batch_size=256)
    p = mp_plan(cfg, 2)
    assert (p.mode, p.placement, p.microbatches, p.orders) == ("time", Placement.mirrored([0, 2, 7, 10]), 8, orders)
    cfg.microbatches = 4
    p = mp_plan(cfg, 2)
    assert p.microbatches == 4 and p.orders is None        # the stored order is for M = 8
    cfg.mp_cut = "reference"
    assert mp_plan(cfg, 2).placement == Placement.contiguous([0, 5, 10])
    cfg = TrainConfig(model="unet", img_size=(512, 512), batch_size=128)        # no plan for this batch
    p = mp_plan(cfg, 2)
    assert p.mode == "v" and p.placement == Placement.mirrored([0, 2, 7, 10]) and p.microbatches == 8
    cfg.mp_cut = "reference"
    assert mp_plan(cfg, 2).microbatches == 2
    path.write_text(json.dumps({"unet:512x512:2:256": {"cuts": [0, 10, 4], "microbatches": 8}}))
    with pytest.raises(ValueError):
        sch.load_plan("unet", 512, 512, 2, 256)
    path.write_text(json.dumps({"unet:512x512:2:256": {"cuts": [0, 2, 7, 9.5], "owner": [0, 1, 0],
                                                       "microbatches": 8}}))
    with pytest.raises(ValueError):                       # does not end at the head
        sch.load_plan("unet", 512, 512, 2, 256)


def test_shipped_plans_are_well_formed():
    from distributedpytorch_amd.models.unet import PRESETS
    from distributedpytorch_amd.parallel import schedule as sch
    if not os.path.exists(sch.PLANS_PATH):
        pytest.skip("no plans shipped")
    with open(sch.PLANS_PATH) as f:
        plans = json.load(f)
    for key in plans:
        model, hw, S, batch = key.split(":")
        h, w = map(int, hw.split("x"))
        p = sch.load_plan(model, h, w, int(S), int(batch), depth=PRESETS[model].depth)
        pl = p["placement"]
        assert pl.S == int(S)
        if p.get("orders"):                                # the stored order replays without deadlock
            assert len(p["orders"]) == pl.S
            c = [SegCost(1.0, 2.0)] * pl.K
            simulate_placement(pl, PRESETS[model].depth, p["microbatches"], c, orders=p["orders"])


def _unet_table():
    from distributedpytorch_amd.parallel.schedule import load_table, unit_table
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    return unit_table(load_table(os.path.join(root, "profiles", "block_times_unetxl_1024_r04.json")))


def test_graph_simulator_reproduces_placement_simulator():
    """The op-graph scheduler of the row-split model (parallel/spatial.py simulate_graph) is the placement
    scheduler on a general graph: a whole-level placement expressed as a graph, with the deferred weight
    gradients after the last op as in simulate_placement, gives the identical timeline."""
    from distributedpytorch_amd.parallel.schedule import placement_costs, simulate_placement
    from distributedpytorch_amd.parallel.spatial import GNode, placement_graph, simulate_graph
    t = _unet_table()
    for pl, M in ((Placement.mirrored([0, 1, 2, 3, 3.5, 4, 4.5, 5, 6, 6.5, 7, 7.5, 8, 9, 10, 12]), 8),
                  (Placement.contiguous([0, 2, 4, 5.5, 6.5, 8, 9, 10, 12]), 4)):
        costs, wg, op, eb = placement_costs(t, pl, 16 // M, M)
        a = simulate_placement(pl, t["depth"], M, costs, eb, wg, op)
        nodes, opt = placement_graph(t, pl, 16, M)
        nodes = [GNode(n.name, n.stage, n.fwd, n.bwd, n.ins, n.head) for n in nodes]    # wgrad at the end
        b = simulate_graph(nodes, pl.S, M, wg, opt)
        assert abs(a.step_ms - b.step_ms) < 1e-9 and a.stage_end == pytest.approx(b.stage_end)
        assert a.orders == b.orders


def test_row_split_geometry_is_exact_and_covering():
    """parallel/spatial.py row_plan: own rows partition the image; every split level runs on rows whose
    two 3x3 convs are exact (two rows inside each non-border edge) on what its consumers read; decoder rows
    even-aligned so the transposed conv's output rows map exactly."""
    from distributedpytorch_amd.parallel.spatial import row_plan
    for H, S, L, bounds in ((1024, 8, 1, None), (1024, 8, 2, None), (64, 4, 2, None), (64, 2, 1, (0, 24, 64)),
                            (1024, 8, 2, (0, 132 - 4, 332, 512, 664, 788, 864, 948, 1024))):
        rp = row_plan(H, S, L, bounds)
        assert rp[0].own[0] == 0 and rp[-1].own[1] == H
        assert all(a.own[1] == b.own[0] for a, b in zip(rp, rp[1:]))
        for sl in rp:
            for l in range(L):
                Hl = H >> l
                ex = lambda r: (r[0] + (2 if r[0] > 0 else 0), r[1] - (2 if r[1] < Hl else 0))   # noqa: E731
                e = ex(sl.enc_in[l])
                assert e[0] <= sl.dec_in[l][0] and sl.dec_in[l][1] <= e[1]          # the skip rows are exact
                d = ex(sl.dec_in[l])
                need = sl.own if l == 0 else sl.up_src(l - 1)
                assert d[0] <= need[0] and need[1] <= d[1]                          # consumer's rows exact
                assert sl.dec_in[l][0] % 2 == 0 and (sl.dec_in[l][1] % 2 == 0 or sl.dec_in[l][1] == Hl)
                assert sl.enc_in[l][0] % 2 == 0
                if l + 1 < L:
                    nxt = sl.enc_in[l + 1]
                    assert e[0] <= 2 * nxt[0] and 2 * nxt[1] <= e[1]
            assert ex(sl.enc_in[L - 1])[0] <= 2 * sl.send[0] and 2 * sl.send[1] <= ex(sl.enc_in[L - 1])[1]
            assert sl.up_src(L - 1) == sl.recv


def test_shipped_row_split_plan_predicts_half_efficiency():
    """Config 5 (UNet-XL 1024^2, 8 stages, b16): the plan tools/pipeline_plan.py ships re-simulates to its
    recorded prediction, >= 0.5 scaling efficiency with the link queues on, and beats the
    best whole-level V placement on the same model."""
    from distributedpytorch_amd.parallel.schedule import PLANS_PATH, single_device_ms
    from distributedpytorch_amd.parallel.spatial import SpatialPlan, simulate_placement_graph, simulate_spatial
    with open(PLANS_PATH) as f:
        p = json.load(f)["unet-xl:1024x1024:8:16"]
    assert p.get("spatial"), p
    t = _unet_table()
    plan = SpatialPlan.from_plan(p).validate(5)
    tl = simulate_spatial(t, plan, 16, p["microbatches"], policy=p["policy"])
    eff = single_device_ms(t, 16) / tl.step_ms / 8
    assert abs(16000.0 / tl.step_ms - p["predicted_img_s"]) < 0.5 and eff >= 0.5
    v = p["v_alternative"]
    tv = simulate_placement_graph(t, Placement(tuple(v["cuts"]), tuple(v["owner"])), 16, v["microbatches"])
    assert tv.step_ms > tl.step_ms
