#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats CSV run: per-kernel totals and one training step's
dispatch timeline (between the last two Adam launches).  Usage: prof_summary.py <dir> [--steps N]"""
import argparse
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--timeline", action="store_true")
    a = ap.parse_args()
    stats = glob.glob(os.path.join(a.dir, "**", "*kernel_stats.csv"), recursive=True)[0]
    trace = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    adam = [i for i, r in enumerate(rows) if "adam" in r["Kernel_Name"]]
    steps = len(adam)
    print(f"# kernel totals over {steps} traced steps ({os.path.basename(stats)})")
    st = list(csv.DictReader(open(stats)))
    tot = sum(float(r["TotalDurationNs"]) for r in st)
    print(f"{'ms/step':>9} {'calls/step':>10} {'%':>6}  kernel")
    for r in sorted(st, key=lambda r: -float(r["TotalDurationNs"]))[:30]:
        name = r["Name"]
        if "at::native" in name:
            name = "torch:" + name.split("at::native::")[1][:50]
        print(f"{float(r['TotalDurationNs']) / 1e6 / steps:9.3f} {int(r['Calls']) / steps:10.1f} "
              f"{float(r['Percentage']):6.2f}  {name[:100]}")
    print(f"total kernel time per step: {tot / 1e6 / steps:.3f} ms")
    if len(adam) >= 2:
        a0, a1 = adam[-2], adam[-1]
        step = rows[a0 + 1:a1 + 1]
        t0 = int(step[0]["Start_Timestamp"])
        wall = (int(step[-1]["End_Timestamp"]) - t0) / 1e3
        busy = sum((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in step)
        print(f"last step: wall {wall:.1f} us, kernels busy {busy:.1f} us ({100 * busy / wall:.1f}%), "
              f"{len(step)} dispatches")
        # the GPU idle time: wall not covered by any kernel (launch gaps, host syncs), and the largest gaps
        ivs = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in step)
        cov, gaps, end = 0, [], ivs[0][0]
        for s0, e0 in ivs:
            if s0 > end:
                gaps.append(((s0 - end) / 1e3, (end - t0) / 1e3))
            cov += max(0, e0 - max(s0, end))
            end = max(end, e0)
        idle = sum(g for g, _ in gaps)
        print(f"idle (no kernel running): {idle:.1f} us ({100 * idle / wall:.1f}% of the step) in {len(gaps)} gaps; "
              "largest: " + ", ".join(f"{g:.0f} us at {t:.0f}" for g, t in sorted(gaps, reverse=True)[:5]))
        if a.timeline:
            for r in step:
                d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
                n = r["Kernel_Name"]
                if "at::native" in n:
                    n = "torch:" + n.split("at::native::")[1][:40]
                print(f"{(int(r['Start_Timestamp']) - t0) / 1e3:9.1f} {d:8.1f}us grid={r['Grid_Size_X']:>9} "
                      f"lds={r['LDS_Block_Size']:>6} vgpr={r['VGPR_Count']:>3} {n[:70]}")


if __name__ == "__main__":
    main()
