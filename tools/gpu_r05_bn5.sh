#!/bin/bash
# whole GPU suite after the BN memory changes; BN + plain bench twice; BN peak-memory breakdown
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/bn5
O=gpurun_out/bn5
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
run() {
  local tag=$1 model=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --model $model --steps 10 --warmup 3 > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -3 $O/$tag.log; exit 1; }
  echo "$tag $(tail -1 $O/$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["peak_mem_gb"])')"
}
run bn unet-bn DPA_X=0
run unet unet DPA_X=0
run bn2 unet-bn DPA_X=0
run unet2 unet DPA_X=0
timeout -k 10 300 python tools/mem_peak.py --model unet-bn --batch 256 > $O/mem_peak_bn.txt 2>&1 || { echo "mem_peak failed"; tail -5 $O/mem_peak_bn.txt; exit 1; }
head -20 $O/mem_peak_bn.txt
