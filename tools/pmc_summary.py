#!/usr/bin/env python3
"""Average rocprofv3 PMC counters per kernel (``rocprofv3 --pmc ... --output-format csv``).

    python tools/pmc_summary.py gpurun_out/pmc
"""
import collections
import csv
import glob
import os
import sys


def main(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        print("no counter_collection.csv under", d)
        return
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in files:
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "?").split("(")[0][:60]
            agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for name, ctrs in agg.items():
        print(name)
        n = max(len(v) for v in ctrs.values())
        for c, v in sorted(ctrs.items()):
            print(f"   {c:28s} mean {sum(v) / len(v):16.1f}  (n={len(v)})")
        w = ctrs.get("SQ_WAVE_CYCLES")
        if w:
            wc = sum(w) / len(w)
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if c in ctrs:
                    print(f"   {c:28s} = {100 * (sum(ctrs[c]) / len(ctrs[c])) / wc:5.1f}% of wave cycles")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc")
