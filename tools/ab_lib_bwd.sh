#!/bin/bash
# Same-box A/B of two library builds (build/ab/old.so, build/ab/new.so): fused conv backward per layer
# (tools/kbench_bwd.py --only-fused), then the whole step, interleaved.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
for v in old new; do
  DPA_LIB_PATH=$PWD/build/ab/$v.so timeout -k 10 300 python tools/kbench_bwd.py --only-fused > gpurun_out/kbb_$v.log 2>&1 || exit 1
  echo "== $v"; grep -v amdgpu gpurun_out/kbb_$v.log | tail -12
done
for i in 1 2; do for v in old new; do
  DPA_LIB_PATH=$PWD/build/ab/$v.so timeout -k 10 200 python bench.py --steps 12 --warmup 4 > gpurun_out/abb_$v$i.log 2>&1 || exit 1
  echo "$v $(tail -1 gpurun_out/abb_$v$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
