#!/bin/bash
# Build + GPU tests + smoke + benches (one gpurun call). Every GPU step has its own timeout.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo build failed; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 400 python -m pytest tests -m gpu -x -q -k "${PYTEST_K:-}" > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -40 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
[ -n "$SKIP_BENCH" ] && exit 0
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --backend hip --steps 10 --warmup 3 --batch ${BATCH:-16} > gpurun_out/bench_hip.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench_hip.log
exit $rc
