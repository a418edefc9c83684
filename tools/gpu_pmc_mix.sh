#!/bin/bash
# Instruction mix of the full-resolution streaming kernels (one counter pass, kernel-trace only):
# VALU / MFMA / LDS / VMEM / SALU instructions and wave / busy cycles per dispatch.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
R=$PWD
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
rm -rf gpurun_out/pmc_mix
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
   --kernel-include-regex "${KRE:-bwd_stream|igemm_stream|igemm_halo|glds|wgrad_stream}" --kernel-trace --output-format csv -d $R/gpurun_out/pmc_mix -o run \
   -- python3 $R/bench.py --batch 64 --steps 2 --warmup 1 > $R/gpurun_out/pmc_mix.log 2>&1) || { echo "pmc rc=$?"; tail -5 gpurun_out/pmc_mix.log; exit 1; }
python tools/pmc_summary.py gpurun_out/pmc_mix > gpurun_out/pmc_mix_summary.txt 2>&1
python - <<'PY'
import csv, glob, collections
files = glob.glob("gpurun_out/pmc_mix/**/*counter_collection.csv", recursive=True)
agg = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
for f in files:
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][:58]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
print(f"{'kernel':58s} {'VALU/w':>8s} {'MFMA/w':>8s} {'LDS/w':>7s} {'VMRD/w':>7s} {'VMWR/w':>7s} {'SALU/w':>7s} {'cyc/w':>9s}")
for k, c in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_BUSY_CYCLES", 0)):
    w = c.get("SQ_WAVE_CYCLES", 1)
    # per 1000 wave-cycles
    f = 1000.0 / max(w, 1)
    print(f"{k:58s} {c['SQ_INSTS_VALU']*f:8.1f} {c['SQ_INSTS_MFMA']*f:8.1f} {c['SQ_INSTS_LDS']*f:7.1f} {c['SQ_INSTS_VMEM_RD']*f:7.1f} {c['SQ_INSTS_VMEM_WR']*f:7.1f} {c['SQ_INSTS_SALU']*f:7.1f} {w:9.3g}")
PY
