#!/bin/bash
# Round-4: fp32 engines at a larger batch (hand-written fp32 vs stock PyTorch fp32).
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/f32b
O=gpurun_out/f32b
for B in 32 64; do
  timeout -k 10 300 python bench.py --dtype fp32 --batch $B --steps 6 --warmup 2 > $O/hip_b$B.log 2>&1 || { echo "hip b$B failed"; tail -3 $O/hip_b$B.log; exit 1; }
  echo "hip b$B $(tail -1 $O/hip_b$B.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
timeout -k 10 600 python bench.py --dtype fp32 --backend torch --batch 64 --steps 6 --warmup 2 > $O/torch_b64.log 2>&1 || { echo "torch b64 failed"; tail -3 $O/torch_b64.log; exit 1; }
echo "torch b64 $(tail -1 $O/torch_b64.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
