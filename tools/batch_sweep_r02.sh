#!/bin/bash
# Per-GPU batch sweep of bench.py on one box (batch 32 = the stock baseline's batch; 256 = default).
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
for b in 32 256 512 256 512; do
  timeout -k 10 200 python bench.py --batch $b --steps 12 --warmup 3 --out gpurun_out/bsweep.jsonl > gpurun_out/bsweep_$b.log 2>&1 || exit 1
  tail -1 gpurun_out/bsweep_$b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["config"]["per_gpu_batch"], d["value"], d["ms_per_step"], d["peak_mem_gb"])'
done
