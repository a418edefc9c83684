#!/bin/bash
# Same-box A/B of an environment switch: bench.py with and without $AB_ENV (e.g.
# AB_ENV="DPA_NO_FUSED_HALVES=1"), interleaved twice.  AB_ARGS: extra bench arguments.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
for i in 1 2; do for v in base env; do
  if [ $v = env ]; then E="$AB_ENV"; else E=""; fi
  env $E timeout -k 10 300 python bench.py --steps ${AB_STEPS:-12} --warmup 4 ${AB_ARGS:-} > gpurun_out/abenv_$v$i.log 2>&1 || exit 1
  echo "$v($E) $(tail -1 gpurun_out/abenv_$v$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
