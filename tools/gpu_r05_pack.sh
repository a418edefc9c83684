#!/bin/bash
# one-instruction bf16 pair packing (default build) vs the two-cast form (libdpa_hip_old.so): whole GPU suite on
# the new build, then same-box benches and kernel-trace totals
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/pack
R=$PWD; O=gpurun_out/pack; OLD=$R/distributedpytorch_amd/_C/libdpa_hip_old.so
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
run() {
  local tag=$1 model=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --model $model --steps 10 --warmup 3 > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -3 $O/$tag.log; exit 1; }
  echo "$tag $(tail -1 $O/$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
for r in 1 2; do
  run unet_new$r unet DPA_X=0
  run unet_old$r unet DPA_LIB_PATH=$OLD
  run bn_new$r unet-bn DPA_X=0
  run bn_old$r unet-bn DPA_LIB_PATH=$OLD
done
prof() {
  local tag=$1 model=$2; shift 2
  rm -rf $O/$tag
  (cd /tmp && env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/$tag -o run -- python3 $R/bench.py --model $model --steps 5 --warmup 2 > $R/$O/$tag.log 2>&1) || { echo "$tag prof failed"; exit 1; }
  python tools/prof_summary.py $O/$tag > $O/sum_$tag.txt 2>&1
  echo "== $tag: $(grep 'total kernel time' $O/sum_$tag.txt) | $(grep 'last step' $O/sum_$tag.txt | cut -c1-40)"
}
prof tr_unet_new unet DPA_X=0
prof tr_unet_old unet DPA_LIB_PATH=$OLD
prof tr_bn_new unet-bn DPA_X=0
prof tr_bn_old unet-bn DPA_LIB_PATH=$OLD
