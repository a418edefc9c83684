#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/px
O=gpurun_out/px
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_fp32_engine.py > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/f32_kbench.py --batch 16 --img 512 --wgrad-px both > $O/kbench.txt 2>&1 || { echo kbench failed; tail $O/kbench.txt; exit 1; }
grep -v amdgpu.ids $O/kbench.txt
for px in 0 1 0 1; do
  DPA_NO_F32_WGRAD_PX=$((1-px)) timeout -k 10 300 python bench.py --dtype fp32 --batch 16 --steps 10 --warmup 3 > $O/bench_px$px.log 2>&1 || { echo bench failed; exit 1; }
  echo "px=$px $(tail -1 $O/bench_px$px.log | cut -c80-140)"
done
