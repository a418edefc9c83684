#!/bin/bash
# BN UNet: dual-input full-resolution decoder level, its skip kept as z, fused two-pass backward of the 256^2 concat conv --
# tests, same-box A/B of both knobs
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/bn9
O=gpurun_out/bn9
timeout -k 10 600 python -u -m pytest -x -q -rP --timeout 300 --timeout-method thread -m gpu tests/test_bn_on_load.py \
  tests/test_dual_input.py tests/test_split_blocks.py tests/test_half_cuts.py tests/test_bwd_fused.py > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
run() {
  local tag=$1 model=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --model $model --steps 10 --warmup 3 > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -3 $O/$tag.log; exit 1; }
  echo "$tag $(tail -1 $O/$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["peak_mem_gb"])')"
}
grep "flat gradient on vs off" $O/pytest.log
run all unet-bn DPA_X=0
run noskipz unet-bn DPA_NO_BN_SKIP_Z=1
run nodual unet-bn DPA_NO_BN_DUAL=1
run nohalves unet-bn DPA_NO_BN_HALVES=1
run all2 unet-bn DPA_X=0
run noskipz2 unet-bn DPA_NO_BN_SKIP_Z=1
run nodual2 unet-bn DPA_NO_BN_DUAL=1
run nohalves2 unet-bn DPA_NO_BN_HALVES=1
