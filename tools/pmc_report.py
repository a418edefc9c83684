#!/usr/bin/env python3
"""Per-kernel hardware-counter report from rocprofv3 --pmc passes of one training step.

Passes (each its own rocprofv3 run, --kernel-trace only; tools/gpu_pmc.sh runs them):
  sq   : SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
         SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE + GRBM_GUI_ACTIVE
  fetch: FETCH_SIZE       write: WRITE_SIZE

Derived per kernel (summed over its dispatches), following MI355X_MICROARCH.md:
  MFMA util  = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs * GRBM_GUI_ACTIVE / 8)    (GRBM sums 8 XCDs)
  LDS confl  = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE  (extra cycles per LDS-array cycle)
  waits      = SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY as % of SQ_WAVE_CYCLES
  HBM bytes  = (2 * FETCH_SIZE + WRITE_SIZE) * 1024   (gfx950 FETCH_SIZE counts half a wide read)
  HBM TB/s   = HBM bytes / kernel time (kernel trace of the fetch pass)

    python tools/pmc_report.py gpurun_out/pmc_sq gpurun_out/pmc_fetch gpurun_out/pmc_write
"""
import collections
import csv
import glob
import os
import sys


def _short(name):
    name = name.split("(")[0]
    if "at::native" in name:
        return "torch:" + name.split("at::native::")[1][:40]
    return name.replace("void ", "")[:60]


def counters(d):
    """{kernel: {counter: total}}, {kernel: dispatches}, {kernel: total ns}"""
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = _short(r.get("Kernel_Name", "?"))
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    dur = collections.defaultdict(float)
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            dur[_short(r["Kernel_Name"])] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return tot, {k: len(v) for k, v in disp.items()}, dur


def main(sq_dir, fetch_dir=None, write_dir=None):
    sq, nd, dur_sq = counters(sq_dir)
    fe, _, dur_fe = counters(fetch_dir) if fetch_dir else ({}, {}, {})
    wr, _, _ = counters(write_dir) if write_dir else ({}, {}, {})
    dur = dur_fe or dur_sq
    rows = sorted(sq, key=lambda k: -dur.get(k, 0.0))
    total_t = sum(dur.values())
    print(f"{'kernel':60s} {'time%':>6} {'MFMA%':>6} {'LDScf':>6} {'wait%':>6} {'stall%':>6} {'act%':>5} "
          f"{'HBM GB':>7} {'TB/s':>6}")
    for k in rows[:40]:
        c = sq[k]
        t = dur.get(k, 0.0)
        grbm = c.get("GRBM_GUI_ACTIVE", 0.0)
        mfma = 100.0 * c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (1024.0 * grbm / 8.0) if grbm else 0.0
        idx = c.get("SQ_LDS_IDX_ACTIVE", 0.0)
        conf = c.get("SQ_LDS_BANK_CONFLICT", 0.0) / idx if idx else 0.0
        wc = c.get("SQ_WAVE_CYCLES", 0.0)
        pct = (lambda n: 100.0 * c.get(n, 0.0) / wc if wc else 0.0)
        gb = ((2.0 * fe.get(k, {}).get("FETCH_SIZE", 0.0) + wr.get(k, {}).get("WRITE_SIZE", 0.0)) * 1024.0 / 1e9
              if fe else 0.0)
        tbs = gb / (t / 1e9) / 1e3 if t and gb else 0.0
        print(f"{k:60s} {100 * t / total_t if total_t else 0:6.1f} {mfma:6.1f} {conf:6.3f} {pct('SQ_WAIT_ANY'):6.1f} "
              f"{pct('SQ_WAIT_INST_ANY'):6.1f} {pct('SQ_ACTIVE_INST_ANY'):5.1f} {gb:7.2f} {tbs:6.2f}")
    print(f"# {len(rows)} kernels; time% of the traced kernel time; MFMA% of the chip's MFMA issue capacity "
          f"over the kernel's own cycles; LDScf = bank-conflict cycles per LDS-array cycle")


if __name__ == "__main__":
    main(*sys.argv[1:4])
