#!/bin/bash
# Same-box interleaved A/B of launch-geometry knobs (env settings in KNOBS, ';'-separated).
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
[ -n "$KNOB_BUILD" ] && { python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1; }
IFS=';' read -ra ARR <<< "${KNOBS:-X=0}"
for i in 1 2; do for j in "${!ARR[@]}"; do
  E="${ARR[$j]}"
  env $E timeout -k 10 200 python bench.py --steps 12 --warmup 4 ${KARGS:-} > gpurun_out/knob_$j$i.log 2>&1 || { echo "[$E] failed"; tail -3 gpurun_out/knob_$j$i.log; exit 1; }
  echo "[$E] $(tail -1 gpurun_out/knob_$j$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
