#!/bin/bash
# wgrad_rows: kernel tests, then same-box A/B of the bench with the deep weight gradients on the new
# kernel (default) vs the row-streaming kernel (DPA_NO_WGRAD_ROWS=1), and pipeline depths.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_hip_kernels.py -k "wgrad" > gpurun_out/pytest_wrows.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_wrows.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_hip_model.py > gpurun_out/pytest_wrows_model.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_wrows_model.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do for v in base rows d2 d1; do
  case $v in base) E="DPA_WGRAD_ROWS=0";; rows) E="DPA_WGRAD_ROWS=1 DPA_WGRAD_ROWS_DEPTH=3";; d2) E="DPA_WGRAD_ROWS=1 DPA_WGRAD_ROWS_DEPTH=2";; d1) E="DPA_WGRAD_ROWS=1 DPA_WGRAD_ROWS_DEPTH=1";; esac
  env $E timeout -k 10 200 python bench.py --steps 12 --warmup 4 > gpurun_out/wrows_$v$i.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/wrows_$v$i.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/wrows_$v$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
