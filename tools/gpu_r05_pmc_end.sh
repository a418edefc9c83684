#!/bin/bash
# end-of-round PMC tables: plain UNet b128 and BN UNet b128 (three counter passes each, tools/gpu_pmc.sh)
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/pmcend
O=gpurun_out/pmcend
bash tools/gpu_pmc.sh --batch 128 --steps 2 --warmup 1 > /dev/null 2>&1 || { echo "bf16 pmc failed"; exit 1; }
cp gpurun_out/pmc_report.txt $O/pmc_b128_512.txt; head -20 $O/pmc_b128_512.txt | cut -c1-120
bash tools/gpu_pmc.sh --model unet-bn --batch 128 --steps 2 --warmup 1 > /dev/null 2>&1 || { echo "bn pmc failed"; exit 1; }
cp gpurun_out/pmc_report.txt $O/pmc_bn_b128_512.txt; head -20 $O/pmc_bn_b128_512.txt | cut -c1-120
