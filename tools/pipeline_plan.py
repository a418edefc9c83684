#!/usr/bin/env python3
"""Pipeline plan from measured per-block times (tools/block_times.py) and the GPipe schedule model
(distributedpytorch_amd/parallel/schedule.py): for BASELINE configs 4 (UNet 512^2, 2 stages) and 5
(UNet-XL 1024^2, 8 stages) the simulated step, img/s and efficiency of

  * the reference cut (encoder+mid | decoder+head) / the FLOP-balanced cut the engine used so far, and
  * the time-balanced cut the simulator finds,

at every microbatch count the table supports; writes a text table and the chosen defaults
(distributedpytorch_amd/parallel/plans.json, read by bench.py / the trainer for ``--mp-cut auto``).

    python tools/pipeline_plan.py profiles/block_times_unet_512_r04.json profiles/block_times_unetxl_1024_r04.json
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributedpytorch_amd.models.blocks import partition          # noqa: E402
from distributedpytorch_amd.models.unet import PRESETS              # noqa: E402
from distributedpytorch_amd.parallel.schedule import load_table, plan, single_device_ms, unit_table  # noqa: E402


def rows_for(table, S, batch, cuts, label, **kw):
    out = []
    for r in plan(table, S, batch, cuts=cuts, **kw):
        r["partition"] = label
        out.append(r)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tables", nargs="+")
    ap.add_argument("--link-gbs", type=float, default=100.0, help="effective xGMI GB/s per peer pair")
    ap.add_argument("--out", default="profiles/pipeline_plan_r04.txt")
    ap.add_argument("--plans", default="distributedpytorch_amd/parallel/plans.json")
    a = ap.parse_args()
    lines, plans = [], {}
    for path in a.tables:
        t = load_table(path)
        model, (h, w) = t["model"], t["img"]
        cfg = PRESETS[model]
        mbs = sorted(int(k) for k in t["per_mb"])
        # config 4: UNet 512^2 on 2 stages at the bench batch; config 5: UNet-XL 1024^2 on 8 stages at the
        # single-GPU bench batch (16) and at the larger global batches the HBM allows (more microbatches:
        # a smaller fill / drain bubble)
        configs = [(2, max(mbs))] if model == "unet" else [(8, 16), (8, 32), (8, 64)]
        for S, batch in configs:
            kw = dict(link_gbs=a.link_gbs)
            t1 = single_device_ms(t, batch)
            lines.append(f"## {model} {h}x{w}, {S} stages, global batch {batch} "
                         f"(single-GPU step {'%.1f ms' % t1 if t1 else 'n/a'})")
            ref = partition(cfg, S, h, w, mode="reference") if S == 2 else None
            flop = partition(cfg, S, h, w, mode="balanced")
            allr = []
            if ref is not None:
                allr += rows_for(t, S, batch, ref, "reference", **kw)
            allr += rows_for(t, S, batch, flop, "flop-balanced", **kw)
            allr += rows_for(t, S, batch, None, "time-balanced", **kw)
            if any("units" in row for row in t["per_mb"].values()):
                # conv-level stage boundaries: cuts between the two convs of a DoubleConv (b + 0.5)
                allr += rows_for(unit_table(t), S, batch, None, "time+conv-cut", **kw)
            lines.append(f"{'partition':14s} {'M':>3s} {'mb':>4s} {'cuts':40s} {'step ms':>9s} {'img/s':>8s} "
                         f"{'util':>6s} {'eff':>6s}")
            for r in allr:
                lines.append(f"{r['partition']:14s} {r['microbatches']:3d} {r['mb']:4d} {str(r['cuts']):40s} "
                             f"{r['step_ms']:9.2f} {r['img_s']:8.1f} {r['utilisation']:6.3f} "
                             f"{r.get('scaling_efficiency', float('nan')):6.3f}")
            best = max((r for r in allr if r["partition"] in ("time-balanced", "time+conv-cut")), key=lambda r: r["img_s"])
            lines.append(f"-> chosen: {best['partition']} cut {best['cuts']}, {best['microbatches']} microbatches "
                         f"({best['img_s']} img/s predicted)")
            lines.append("")
            plans[f"{model}:{h}x{w}:{S}:{batch}"] = {"cuts": best["cuts"], "microbatches": best["microbatches"],
                                                     "predicted_img_s": best["img_s"],
                                                     "predicted_efficiency": best.get("scaling_efficiency")}
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n")
    if a.plans:
        with open(a.plans, "w") as f:
            json.dump(plans, f, indent=1)


if __name__ == "__main__":
    main()
