#!/bin/bash
# Slice-staged GEMMs (cfg 18/19): fp32-anchored tests, per-layer timing against pp2h (14/15).
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/sl
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_rowblock.py > gpurun_out/sl/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/sl/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/kbench.py --batch 256 --paths "" --no-wgrad --gvar 14 15 262144 524288 --reps 7 --only "L2,L3,mid" > gpurun_out/sl/kbench.log 2>&1 || { echo kbench failed; tail gpurun_out/sl/kbench.log; exit 1; }
grep -v "n/a" gpurun_out/sl/kbench.log
