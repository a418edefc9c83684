#!/bin/bash
# Same-box A/B of two library builds (build/ab/old.so, build/ab/new.so): row-streaming forward convs
# per layer (tools/kbench.py --paths stream), then the whole step, interleaved.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
for v in old new; do
  DPA_LIB_PATH=$PWD/build/ab/$v.so timeout -k 10 300 python tools/kbench.py --batch ${KB_BATCH:-256} --paths stream \
    --only "L0,L1 32->64,L1 64->64" --no-wgrad > gpurun_out/kbs_$v.log 2>&1 || exit 1
  echo "== $v"; grep -v amdgpu gpurun_out/kbs_$v.log
done
for i in 1 2; do for v in old new; do
  DPA_LIB_PATH=$PWD/build/ab/$v.so timeout -k 10 200 python bench.py --steps 12 --warmup 4 > gpurun_out/abs_$v$i.log 2>&1 || exit 1
  echo "$v $(tail -1 gpurun_out/abs_$v$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
