#!/bin/bash
# documentation artifacts of the final tree: BN and plain kernel summaries, BN peak-memory breakdown
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/doc
R=$PWD; O=gpurun_out/doc
rm -rf $O/bn $O/unet
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/bn -o run -- python3 $R/bench.py --model unet-bn --steps 5 --warmup 2 > $R/$O/bn.log 2>&1) || { echo "bn prof failed"; exit 1; }
python tools/prof_summary.py $O/bn --timeline > $O/sum_bn.txt 2>&1; head -4 $O/sum_bn.txt
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/unet -o run -- python3 $R/bench.py --steps 5 --warmup 2 > $R/$O/unet.log 2>&1) || { echo "unet prof failed"; exit 1; }
python tools/prof_summary.py $O/unet --timeline > $O/sum_unet.txt 2>&1; head -4 $O/sum_unet.txt
timeout -k 10 300 python tools/mem_peak.py --model unet-bn --batch 256 > $O/mem_peak_bn.txt 2>&1 || { echo "mem_peak failed"; exit 1; }
head -16 $O/mem_peak_bn.txt
