#!/bin/bash
# Round 5: PMC tables (fp32 b16 and bf16 b128 steps) and one-GPU rehearsals of the shipped pipeline plans.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/r05pmc
O=gpurun_out/r05pmc
bash tools/gpu_pmc.sh --dtype fp32 --batch 16 --steps 2 --warmup 1 > /dev/null 2>&1 || { echo "fp32 pmc failed"; exit 1; }
cp gpurun_out/pmc_report.txt $O/pmc_fp32_b16.txt; head -24 $O/pmc_fp32_b16.txt
bash tools/gpu_pmc.sh --batch 128 --steps 2 --warmup 1 > /dev/null 2>&1 || { echo "bf16 pmc failed"; exit 1; }
cp gpurun_out/pmc_report.txt $O/pmc_b128_512.txt; head -24 $O/pmc_b128_512.txt
timeout -k 10 300 python bench.py --model unet-xl --img 1024 --batch 16 --steps 6 --warmup 2 > $O/xl_1stage.log 2>&1 || { echo "xl failed"; exit 1; }
echo "xl 1 stage: $(tail -1 $O/xl_1stage.log | cut -c80-140)"
timeout -k 10 400 python bench.py --model unet-xl --img 1024 --batch 16 --parallelism mp --stages 8 --steps 6 --warmup 2 > $O/xl_mp8.log 2>&1 || { echo "xl mp failed"; tail -3 $O/xl_mp8.log; exit 1; }
echo "xl mp8 (plan): $(tail -1 $O/xl_mp8.log | cut -c80-140)"
timeout -k 10 300 python bench.py --parallelism mp --stages 2 --steps 10 --warmup 3 > $O/mp2.log 2>&1 || { echo "mp2 failed"; exit 1; }
echo "unet mp2 (plan): $(tail -1 $O/mp2.log | cut -c80-140)"
