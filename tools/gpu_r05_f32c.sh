#!/bin/bash
# fp32 engine confirmation: engine + multirank fp32 tests, bench.py --dtype fp32 b16 x2, rocprof kernel summary
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/f32c
O=gpurun_out/f32c
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_fp32_engine.py \
  tests/test_hip_multirank.py -k "fp32 or f32 or engine" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --dtype fp32 --batch 16 --steps 20 --warmup 3 > $O/bench_$i.log 2>&1 || { echo bench failed; tail -5 $O/bench_$i.log; exit 1; }
  echo "run $i $(tail -1 $O/bench_$i.log | cut -c80-140)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --dtype fp32 --batch 16 --steps 5 --warmup 2 > $O/prof.log 2>&1 || { echo prof failed; tail -5 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/kernel_stats.csv
head -25 $O/kernel_stats.csv | cut -c1-150
