#!/bin/bash
# kernel-trace summary of the BN UNet step (b256, 512^2)
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/bnprof
R=$PWD; O=gpurun_out/bnprof
rm -rf $O/prof
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- python3 $R/bench.py --model unet-bn --steps 5 --warmup 2 > $R/$O/prof.log 2>&1) || { echo "prof failed"; tail $O/prof.log; exit 1; }
python tools/prof_summary.py $O/prof --timeline > $O/prof_summary_bn.txt 2>&1; head -45 $O/prof_summary_bn.txt | cut -c1-150
