#!/bin/bash
# Timing ablation (numerics intentionally wrong): the bench with each kernel family's launches
# skipped (bench.py --timing-ablation, ops/kernels.py set_timing_ablation) -> the end-to-end step time
# that family costs.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
for v in none wgrad_deep wgrad halo glds bwd stream deconv "halo,glds" none; do
  E=$v; [ $v = none ] && E=
  timeout -k 10 200 python bench.py --steps 12 --warmup 4 --timing-ablation "$E" ${ABL_ARGS:-} > gpurun_out/abl_$v.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/abl_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/abl_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
