#!/bin/bash
# Kernel-trace profiles of bench.py from the current tree and from build/ab/oldtree (same box),
# summaries side by side (first NTOP lines each).
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
R=$PWD
for v in old new; do
  d=$R; [ $v = old ] && d=$R/build/ab/oldtree
  rm -rf gpurun_out/abprof_$v
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/abprof_$v -o run -- python3 $d/bench.py --steps 4 --warmup 2 ${AB_ARGS:-} > $R/gpurun_out/abprof_$v.log 2>&1) || { echo "prof $v rc=$?"; exit 1; }
  python tools/prof_summary.py gpurun_out/abprof_$v > gpurun_out/abprof_${v}_summary.txt 2>&1
  echo "== $v"; head -${NTOP:-16} gpurun_out/abprof_${v}_summary.txt
done
