#!/bin/bash
# Two kernel-trace profiles of the bench under different env settings (PA / PB), summaries side by side.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
R=$PWD
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
for v in A B; do
  E=$([ $v = A ] && echo "${PA:-X=1}" || echo "${PB:-X=1}")
  ARGS=$([ $v = A ] && echo "${PARGS_A:-$PARGS}" || echo "${PARGS_B:-$PARGS}")
  rm -rf gpurun_out/prof$v
  (cd /tmp && env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof$v -o run -- python3 $R/bench.py --steps 4 --warmup 2 $ARGS > $R/gpurun_out/prof$v.log 2>&1) || { echo "prof $v rc=$?"; exit 1; }
  python tools/prof_summary.py gpurun_out/prof$v > gpurun_out/prof${v}_summary.txt 2>&1
  echo "== $v ($E)"; head -${NTOP:-25} gpurun_out/prof${v}_summary.txt
done
