#!/usr/bin/env python3
"""Pipeline plans from measured per-block times (tools/block_times.py) and the link-queueing GPipe
schedule model (distributedpytorch_amd/parallel/schedule.py).

For BASELINE config 4 (UNet 512^2, 2 stages) and config 5 (UNet-XL 1024^2, 8 stages), at every
microbatch count the table supports and at two effective xGMI rates per directed peer link (100 and
64 GB/s), the simulated step, img/s, efficiency and busiest-link load of

  * the reference cut (encoder+mid | decoder+head, 2 stages) and the FLOP-balanced contiguous cut,
  * the best contiguous placement the search finds (half-block cuts allowed),
  * the best mirrored V placement (stage s owns encoder level(s) s and the same decoder level(s)),

then writes a text table and the chosen plans (distributedpytorch_amd/parallel/plans.json, read by
``--mp-cut auto|time``): placement, microbatch count, op-order policy and the per-stage op order the
simulation used (the engine issues exactly that order).

    python tools/pipeline_plan.py profiles/block_times_unet_512_r04.json profiles/block_times_unetxl_1024_r04.json
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributedpytorch_amd.models.blocks import partition          # noqa: E402
from distributedpytorch_amd.models.unet import PRESETS              # noqa: E402
from distributedpytorch_amd.parallel.placement import Placement, describe, v_partition  # noqa: E402
from distributedpytorch_amd.parallel.schedule import (evaluate_placement, load_table, search,  # noqa: E402
                                                      simulate_table, single_device_ms, unit_table)
from distributedpytorch_amd.parallel.spatial import (SpatialPlan, search_spatial,  # noqa: E402
                                                     simulate_placement_graph, simulate_spatial)


def fmt(r, label):
    return (f"{label:16s} {r['microbatches']:3d} {r['mb']:4d} {str(r['cuts']):52s} {r['policy']:7s} "
            f"{r['step_ms']:9.2f} {r['img_s']:8.1f} {r.get('scaling_efficiency', float('nan')):6.3f} "
            f"{r['max_link_gb']:7.2f} {r['max_link_busy_ms']:8.1f}")


def hybrid_tables(paths, link_gbs):
    """--mp-replicas: R pipelines of S stages on G = R x S GPUs at a fixed global batch B (each pipeline
    B / R images).  Step = the best V pipeline of S stages at B / R (simulated, links queued) + the
    data-parallel all-reduce of the largest stage's fp32 gradients over R GPUs, not overlapped (ring:
    2 (R-1)/R x bytes at the link rate); S = 1 is plain data parallelism."""
    from distributedpytorch_amd.models.unet import build_model
    from distributedpytorch_amd.parallel.pipeline import placement_param_names
    out = []
    for path in paths:
        t = load_table(path)
        ut = unit_table(t) if any("units" in row for row in t["per_mb"].values()) else t
        model_name, (h, w) = t["model"], t["img"]
        model = build_model(model_name)
        numel = {n: p.numel() for n, p in model.named_parameters()}
        G, batches = (2, [256]) if model_name == "unet" else (8, [16, 32, 64])
        for B in batches:
            t1 = single_device_ms(t, B)
            out.append(f"## {model_name} {h}x{w}: {G} GPUs as R pipelines x S stages, global batch {B}, "
                       f"{link_gbs:g} GB/s links (single GPU: {t1:.1f} ms)")
            out.append(f"{'S':>2s} {'R':>2s} {'b/pipe':>6s} {'M':>3s} {'pipe ms':>8s} {'ar ms':>6s} {'step ms':>8s} "
                       f"{'img/s':>8s} {'eff':>6s}  placement")
            for S in [d for d in range(1, G + 1) if G % d == 0]:
                R = G // S
                if B % R:
                    continue
                b = B // R
                if S == 1:
                    tp, M, pl_s, stage_bytes = single_device_ms(t, b), 1, "whole model", 4 * sum(numel.values())
                    if tp is None:
                        continue
                else:
                    rows = search(ut, S, b, "v", link_gbs=link_gbs)
                    if not rows:
                        continue
                    best = max(rows, key=lambda r: r["img_s"])
                    pl = Placement(best["cuts"], best["owner"])
                    tp, M, pl_s = 1000.0 * b / best["img_s"], best["microbatches"], str(pl)
                    stage_bytes = max(4 * sum(numel[n] for n in placement_param_names(model, pl, s)) for s in range(S))
                tar = 2 * (R - 1) / R * stage_bytes / (link_gbs * 1e6) if R > 1 else 0.0
                step = tp + tar
                out.append(f"{S:2d} {R:2d} {b:6d} {M:3d} {tp:8.2f} {tar:6.2f} {step:8.2f} {1000 * B / step:8.1f} "
                           f"{t1 / (G * step):6.3f}  {pl_s}")
            out.append("")
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tables", nargs="+")
    ap.add_argument("--links", default="100,64", help="effective GB/s per directed xGMI peer link (first: the plan's)")
    ap.add_argument("--out", default="profiles/pipeline_plan_r06.txt")
    ap.add_argument("--plans", default="distributedpytorch_amd/parallel/plans.json")
    a = ap.parse_args()
    links = [float(v) for v in a.links.split(",")]
    lines, plans = [], {}
    for path in a.tables:
        t = load_table(path)
        ut = unit_table(t) if any("units" in row for row in t["per_mb"].values()) else t
        model, (h, w) = t["model"], t["img"]
        cfg = PRESETS[model]
        mbs = sorted(int(k) for k in t["per_mb"])
        configs = [(2, max(mbs)), (4, max(mbs))] if model == "unet" else [(8, 16), (8, 32), (8, 64)]
        for S, batch in configs:
            t1 = single_device_ms(t, batch)
            best_v = None
            for gbs in links:
                kw = dict(link_gbs=gbs)
                lines.append(f"## {model} {h}x{w}, {S} stages, global batch {batch}, xGMI {gbs:g} GB/s per directed link "
                             f"(single-GPU step {'%.1f ms' % t1 if t1 else 'n/a'})")
                lines.append(f"{'placement':16s} {'M':>3s} {'mb':>4s} {'cuts':52s} {'policy':7s} {'step ms':>9s} "
                             f"{'img/s':>8s} {'eff':>6s} {'link GB':>7s} {'link ms':>8s}")
                fixed = []
                if S == 2:
                    fixed.append(("reference", Placement.contiguous(partition(cfg, S, h, w, mode="reference"))))
                fixed.append(("flop-contig", Placement.contiguous(partition(cfg, S, h, w, mode="balanced"))))
                fixed.append(("flop-v", v_partition(cfg, S, h, w)))
                for label, pl in fixed:
                    for pol in ("feed", "further"):
                        for r in evaluate_placement(ut, pl, batch, policy=pol, **kw):
                            lines.append(fmt(r, label))
                cont = search(ut, S, batch, "contiguous", **kw)
                for r in cont:
                    lines.append(fmt(r, "search-contig"))
                vv = search(ut, S, batch, "v", **kw)
                for r in vv:
                    lines.append(fmt(r, "search-v"))
                bc = max(cont, key=lambda r: r["img_s"])
                bv = max(vv, key=lambda r: r["img_s"])
                lines.append(f"-> best contiguous {bc['cuts']} M={bc['microbatches']}: {bc['img_s']} img/s "
                             f"(eff {bc.get('scaling_efficiency')}); best V {bv['cuts']} M={bv['microbatches']}: "
                             f"{bv['img_s']} img/s (eff {bv.get('scaling_efficiency')})")
                lines.append("")
                if gbs == links[0]:
                    best_v = bv
                else:          # the chosen plan re-simulated at the slower link
                    pl = Placement(best_v["cuts"], best_v["owner"])
                    r = evaluate_placement(ut, pl, batch, Ms=[best_v["microbatches"]], policy=best_v["policy"], **kw)[0]
                    best_v.setdefault("at_slow_link", {})[f"{gbs:g}"] = {
                        "img_s": r["img_s"], "efficiency": r.get("scaling_efficiency")}
            pl = Placement(best_v["cuts"], best_v["owner"])
            M = best_v["microbatches"]
            tl = simulate_table(ut, pl, batch // M, M, policy=best_v["policy"], link_gbs=links[0])
            row = {
                "cuts": best_v["cuts"], "owner": best_v["owner"], "placement": pl.kind, "microbatches": M,
                "policy": best_v["policy"], "orders": tl.orders,
                "predicted_img_s": best_v["img_s"], "predicted_efficiency": best_v.get("scaling_efficiency"),
                "link_gbs": links[0], "at_slow_link": best_v.get("at_slow_link", {}),
                "source": os.path.basename(path)}
            chosen = f"{pl} M={M} policy {best_v['policy']}: {best_v['img_s']} img/s predicted at {links[0]:g} GB/s; " \
                + "; ".join(describe(pl, cfg.depth))
            if model != "unet" and not cfg.batchnorm and S >= 4:
                # row-split top levels (parallel/spatial.py) against the best whole-level V, both on the op-graph
                # model (deferred weight gradients in the drain's idle time)
                tv = simulate_placement_graph(ut, pl, batch, M, policy=best_v["policy"], link_gbs=links[0])
                v_img = round(batch * 1000.0 / tv.step_ms, 1)
                lines.append(f"## {model} {h}x{w}, {S} stages, b{batch}: row-split top levels vs the V above "
                             f"(op-graph model; V {pl} M={M}: {v_img} img/s, eff {t1 / tv.step_ms / S:.3f})")
                sp = search_spatial(ut, S, batch, link_gbs=links[0], top=6)
                for r in sp:
                    lines.append(f"spatial L={r['split_levels']} M={r['microbatches']:3d} mb={r['mb']:3d} inner "
                                 f"{r['inner_cuts']}@{r['inner_owner']} rows {r['row_bounds']} {r['policy']:7s} "
                                 f"{r['step_ms']:8.2f} ms {r['img_s']:8.1f} img/s eff {r.get('scaling_efficiency')} "
                                 f"link {r['max_link_gb']:.2f} GB / {r['max_link_busy_ms']:.1f} ms")
                bs = max(sp, key=lambda r: r["img_s"]) if sp else None
                if bs is not None and bs["img_s"] > v_img:
                    sp_pl = SpatialPlan.from_plan(bs)
                    for gbs in links[1:]:
                        t2 = simulate_spatial(ut, sp_pl, batch, bs["microbatches"], policy=bs["policy"], link_gbs=gbs)
                        bs.setdefault("at_slow_link", {})[f"{gbs:g}"] = {
                            "img_s": round(batch * 1000.0 / t2.step_ms, 1),
                            "efficiency": round(t1 / t2.step_ms / S, 3)}
                    row = {**sp_pl.to_plan(), "placement": "spatial", "microbatches": bs["microbatches"],
                           "policy": bs["policy"], "predicted_img_s": bs["img_s"],
                           "predicted_efficiency": bs.get("scaling_efficiency"), "link_gbs": links[0],
                           "at_slow_link": bs.get("at_slow_link", {}), "source": os.path.basename(path),
                           "v_alternative": {"cuts": best_v["cuts"], "owner": best_v["owner"], "microbatches": M,
                                             "img_s_graph_model": v_img}}
                    chosen = f"{sp_pl} M={bs['microbatches']} policy {bs['policy']}: {bs['img_s']} img/s predicted " \
                             f"(eff {bs.get('scaling_efficiency')}) at {links[0]:g} GB/s (V: {v_img})"
                lines.append("")
            lines.append(f"-> chosen for {model} {S} stages b{batch}: {chosen}")
            lines.append("")
            plans[f"{model}:{h}x{w}:{S}:{batch}"] = row
    lines += hybrid_tables(a.tables, links[0])
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n")
    if a.plans:
        old = {}
        if os.path.exists(a.plans):
            with open(a.plans) as f:
                old = json.load(f)
        for key, row in plans.items():      # measured rehearsals stay with a plan whose placement is unchanged
            prev = old.get(key, {})
            if "measured" in prev and prev.get("cuts") == row.get("cuts") and prev.get("owner") == row.get("owner") \
                    and prev.get("inner_cuts") == row.get("inner_cuts") and prev.get("microbatches") == row["microbatches"]:
                row["measured"] = prev["measured"]
        with open(a.plans, "w") as f:
            json.dump(plans, f, indent=1)


if __name__ == "__main__":
    main()
