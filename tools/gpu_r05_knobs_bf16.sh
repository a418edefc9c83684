#!/bin/bash
# headline bench (bf16 b256) under launch-geometry knob settings, same box, two rounds
set -o pipefail
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/knobs
O=gpurun_out/knobs
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -3 $O/$tag.log; exit 1; }
  echo "$tag $(tail -1 $O/$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
for r in 1 2; do
  run base$r DPA_X=0
  run chunks2_$r DPA_ENC0_CHUNKS=2
  run chunks8_$r DPA_ENC0_CHUNKS=8
  run wsb4096_$r DPA_WGRAD_STREAM_BLOCKS=4096
  run bwdb2048_$r DPA_BWD_BLOCKS=2048
done
