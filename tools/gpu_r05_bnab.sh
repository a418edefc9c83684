#!/bin/bash
# BN UNet same-box A/B of the round-5 BN partial-sum hand-overs (pool backward, deconv backward)
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/bnab
O=gpurun_out/bnab
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --model unet-bn --steps 10 --warmup 3 > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -3 $O/$tag.log; exit 1; }
  echo "$tag $(tail -1 $O/$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["peak_mem_gb"])')"
}
run all DPA_X=0
run nopool DPA_NO_BN_SUMS_POOL=1
run nodeconv DPA_NO_BN_SUMS_DECONV=1
run none DPA_NO_BN_SUMS_POOL=1 DPA_NO_BN_SUMS_DECONV=1
run all2 DPA_X=0
run nopool2 DPA_NO_BN_SUMS_POOL=1
run nodeconv2 DPA_NO_BN_SUMS_DECONV=1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/unet.log 2>&1 || exit 1
echo "unet $(tail -1 $O/unet.log | cut -c80-140)"
