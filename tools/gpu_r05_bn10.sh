#!/bin/bash
# BN UNet: head backward folded into the last decoder conv's fused backward -- tests, same-box A/B
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/bn10
O=gpurun_out/bn10
timeout -k 10 600 python -u -m pytest -x -q -rP --timeout 300 --timeout-method thread -m gpu tests/test_bn_on_load.py \
  tests/test_hip_kernels.py tests/test_bwd_fused.py > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
run() {
  local tag=$1 model=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --model $model --steps 10 --warmup 3 > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -3 $O/$tag.log; exit 1; }
  echo "$tag $(tail -1 $O/$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["peak_mem_gb"])')"
}
run on unet-bn DPA_X=0
run off unet-bn DPA_NO_BN_HEAD_FOLD=1
run on2 unet-bn DPA_X=0
run off2 unet-bn DPA_NO_BN_HEAD_FOLD=1
