#!/bin/bash
# Same-box A/B of two library builds (build/ab/old.so, build/ab/new.so) on the row-streaming weight
# gradient at the UNet shapes (tools/kbench.py wgrad lines), then the whole step.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
for v in old new; do
  DPA_LIB_PATH=$PWD/build/ab/$v.so timeout -k 10 300 python tools/kbench.py --batch ${BATCH:-256} --reps 5 --paths "" \
    --only "L0 32->32,L1 64->64,L2 128->128,L3 256->256,L3 512->256" > gpurun_out/kbw_$v.log 2>&1 || exit 1
  echo "== $v"; grep "wgrad stream" gpurun_out/kbw_$v.log
done
for i in 1 2; do for v in old new; do
  DPA_LIB_PATH=$PWD/build/ab/$v.so timeout -k 10 200 python bench.py --steps 12 --warmup 4 > gpurun_out/abw_$v$i.log 2>&1 || exit 1
  echo "$v $(tail -1 gpurun_out/abw_$v$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
