#!/bin/bash
# Same-box A/B of the fused backward's row staging: registers (DPA_BWD_DMA=0) vs LDS-DMA rings of 4 or
# 5 slots -- tests first, then per-layer kbench_bwd and the whole step.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
for d in 4 5; do
  DPA_BWD_DMA=$d timeout -k 10 200 python -u -m pytest tests/test_bwd_fused.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_dma$d.log 2>&1 || { tail -20 gpurun_out/pytest_dma$d.log; exit 1; }
  echo "dma=$d tests: $(tail -1 gpurun_out/pytest_dma$d.log)"
done
for d in 0 4 5; do
  DPA_BWD_DMA=$d timeout -k 10 300 python tools/kbench_bwd.py --only-fused > gpurun_out/kbd_$d.log 2>&1 || exit 1
  echo "== dma=$d"; grep "fused" gpurun_out/kbd_$d.log | cut -c1-70
done
for i in 1 2; do for d in 0 4 5; do
  DPA_BWD_DMA=$d timeout -k 10 200 python bench.py --steps 12 --warmup 4 > gpurun_out/abd_$d$i.log 2>&1 || exit 1
  echo "dma=$d $(tail -1 gpurun_out/abd_$d$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
