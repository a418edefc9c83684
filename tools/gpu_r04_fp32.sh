#!/bin/bash
# Round-4: fp32 hand-written path -- op / whole-step tests against torch fp32, train.py --dtype fp32, timing.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/fp32
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_fp32_engine.py tests/test_fp32_backend.py > gpurun_out/fp32/pytest.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error" gpurun_out/fp32/pytest.log | tail -20; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --dtype fp32 --batch 16 --steps 5 --warmup 2 > gpurun_out/fp32/bench.log 2>&1 || { echo "bench fp32 failed"; tail -5 gpurun_out/fp32/bench.log; exit 1; }
tail -1 gpurun_out/fp32/bench.log | cut -c1-250
