#!/bin/bash
# BN mode 1 at 64 input channels: loader transforms right after the dx MFMAs (libdpa_hip_early.so, built with
# -DDPA_EARLY_BNM1=1) vs next to the ring store (default build) -- BN tests on the early build, same-box A/B
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/early
O=gpurun_out/early
E=$PWD/distributedpytorch_amd/_C/libdpa_hip_early.so
DPA_LIB_PATH=$E timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_bn_on_load.py \
  tests/test_dual_input.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --model unet-bn --steps 10 --warmup 3 > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -3 $O/$tag.log; exit 1; }
  echo "$tag $(tail -1 $O/$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
run base DPA_X=0
run early DPA_LIB_PATH=$E
run base2 DPA_X=0
run early2 DPA_LIB_PATH=$E
