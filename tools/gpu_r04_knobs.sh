#!/bin/bash
# Round-4: launch-geometry knobs re-checked after this round's kernel changes (interleaved A/B, default first and last).
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/knobs
O=gpurun_out/knobs
run() {  # $1 tag, rest = env assignments
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 15 --warmup 4 > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -3 $O/$tag.log; exit 1; }
  echo "$tag $(tail -1 $O/$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
run base0 DPA_X=0
run wgg512 DPA_WGRAD_GEMM_BLOCKS=512
run wgg1024 DPA_WGRAD_GEMM_BLOCKS=1024
run wgs1024 DPA_WGRAD_STREAM_BLOCKS=1024
run wgs4096 DPA_WGRAD_STREAM_BLOCKS=4096
run bwd2048 DPA_BWD_BLOCKS=2048
run prio DPA_SIDE_PRIORITY=-1
run base1 DPA_X=0
# fp32: the hand-written fp32 engine vs stock PyTorch fp32 (MIOpen) at the same batch
timeout -k 10 600 python bench.py --dtype fp32 --batch 16 --steps 5 --warmup 2 > $O/fp32_hip.log 2>&1 || { echo "fp32 hip failed"; exit 1; }
echo "fp32_hip $(tail -1 $O/fp32_hip.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
timeout -k 10 900 python bench.py --dtype fp32 --backend torch --batch 16 --steps 5 --warmup 2 > $O/fp32_torch.log 2>&1 || { echo "fp32 torch failed"; tail -3 $O/fp32_torch.log; exit 1; }
echo "fp32_torch $(tail -1 $O/fp32_torch.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
