#!/bin/bash
# PMC table of the fp32 step after the round-5 kernels (halo conv, split halo wgrad, first-layer wgrad)
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/r05pmc
bash tools/gpu_pmc.sh --dtype fp32 --batch 16 --steps 2 --warmup 1 > /dev/null 2>&1 || { echo "fp32 pmc failed"; exit 1; }
cp gpurun_out/pmc_report.txt gpurun_out/r05pmc/pmc_fp32_b16_halo.txt; head -24 gpurun_out/r05pmc/pmc_fp32_b16_halo.txt
