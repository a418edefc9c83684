#!/bin/bash
# BN UNet: head on load + z-based pool sums -- kernel tests, same-box A/B of the BN knobs, peak-memory breakdown
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/bn3
O=gpurun_out/bn3
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_bn_on_load.py \
  tests/test_hip_kernels.py tests/test_hip_variants.py > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --model unet-bn --steps 10 --warmup 3 > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -3 $O/$tag.log; exit 1; }
  echo "$tag $(tail -1 $O/$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["peak_mem_gb"])')"
}
run all DPA_X=0
run nohead DPA_NO_BN_HEAD_ON_LOAD=1
run nopoolz DPA_NO_BN_SUMS_POOL_Z=1
run nopool DPA_NO_BN_SUMS_POOL=1
run nodeconv DPA_NO_BN_SUMS_DECONV=1
run all2 DPA_X=0
run nohead2 DPA_NO_BN_HEAD_ON_LOAD=1
run nopool2 DPA_NO_BN_SUMS_POOL=1
timeout -k 10 300 python tools/mem_peak.py --model unet-bn --batch 256 > $O/mem_peak_bn.txt 2>&1 || { echo "mem_peak failed"; tail -5 $O/mem_peak_bn.txt; exit 1; }
head -30 $O/mem_peak_bn.txt
