#!/bin/bash
# per-GPU batch sweep of the headline bench (same box)
set -o pipefail
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/bsweep
O=gpurun_out/bsweep
for b in 256 384 512 256; do
  timeout -k 10 400 python bench.py --batch $b --steps 10 --warmup 3 > $O/b$b.log 2>&1 || { echo "b$b failed"; tail -3 $O/b$b.log; exit 1; }
  echo "b$b $(tail -1 $O/b$b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["peak_mem_gb"])')"
done
