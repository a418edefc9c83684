#!/bin/bash
# BN step kernel traces: BN mode 1 loader transforms early (default build) vs late (libdpa_hip_late.so)
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/lateprof
R=$PWD; O=gpurun_out/lateprof; L=$R/distributedpytorch_amd/_C/libdpa_hip_late.so
rm -rf $O/early $O/late
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/early -o run -- python3 $R/bench.py --model unet-bn --steps 5 --warmup 2 > $R/$O/early.log 2>&1) || { echo "early prof failed"; exit 1; }
(cd /tmp && DPA_LIB_PATH=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/late -o run -- python3 $R/bench.py --model unet-bn --steps 5 --warmup 2 > $R/$O/late.log 2>&1) || { echo "late prof failed"; exit 1; }
for v in early late; do python tools/prof_summary.py $O/$v > $O/sum_$v.txt 2>&1; echo "== $v"; grep "bwd_stream" $O/sum_$v.txt | head -8 | cut -c1-110; done
