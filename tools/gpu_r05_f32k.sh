#!/bin/bash
# Round 5: fp32 kernel A/B -- the 256 x 256 weight-gradient tile vs 128 x 128 per layer, its test, and the
# fp32 bench with and without it.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/f32k
O=gpurun_out/f32k
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_fp32_engine.py > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/f32_kbench.py --batch 16 --img 512 --wgrad-big both > $O/kbench.txt 2>&1 || { echo kbench failed; tail $O/kbench.txt; exit 1; }
cat $O/kbench.txt
for big in 0 1; do
  DPA_F32_WGRAD_BIG=$big timeout -k 10 300 python bench.py --dtype fp32 --batch 16 --steps 10 --warmup 3 > $O/bench_big$big.log 2>&1 || { echo bench failed; tail $O/bench_big$big.log; exit 1; }
  echo "big=$big $(tail -1 $O/bench_big$big.log | cut -c80-140)"
done
