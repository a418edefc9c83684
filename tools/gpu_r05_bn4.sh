#!/bin/bash
# BN UNet: head backward deferred into the decoder + fixed-chunk BN apply; wgrad reduce presum (plain UNet) --
# kernel tests, same-box A/B of the knobs, peak-memory breakdown
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/bn4
O=gpurun_out/bn4
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_bn_on_load.py \
  tests/test_hip_kernels.py tests/test_hip_variants.py tests/test_fp32_engine.py > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
run() {
  local tag=$1 model=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --model $model --steps 10 --warmup 3 > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -3 $O/$tag.log; exit 1; }
  echo "$tag $(tail -1 $O/$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["peak_mem_gb"])')"
}
run bn_all unet-bn DPA_X=0
run bn_nocc unet-bn DPA_NO_BN_CC_APPLY=1
run bn_nodefer unet-bn DPA_NO_BN_HEAD_DEFER=1
run bn_all2 unet-bn DPA_X=0
run bn_nocc2 unet-bn DPA_NO_BN_CC_APPLY=1
run unet_all unet DPA_X=0
run unet_nopresum unet DPA_NO_WGRAD_PRESUM=1
run unet_all2 unet DPA_X=0
run unet_nopresum2 unet DPA_NO_WGRAD_PRESUM=1
timeout -k 10 300 python tools/mem_peak.py --model unet-bn --batch 256 > $O/mem_peak_bn.txt 2>&1 || { echo "mem_peak failed"; tail -5 $O/mem_peak_bn.txt; exit 1; }
head -24 $O/mem_peak_bn.txt
