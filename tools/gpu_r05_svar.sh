#!/bin/bash
# streaming-conv strip variants at b256 (auto vs 1: BP128x4w, 2: BP64x4w, 3: BP128x8w, 4: BP64x8w)
set -o pipefail
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/svar
timeout -k 10 500 python tools/kbench.py --batch 256 --only "L0 64->32,L0 32->32,L1 64->64,L1 32->64" --paths stream \
  --svar 1 2 3 4 --no-wgrad --reps 5 > gpurun_out/svar/kbench.txt 2>&1; rc=$?
cat gpurun_out/svar/kbench.txt | grep -v amdgpu.ids; exit $rc
