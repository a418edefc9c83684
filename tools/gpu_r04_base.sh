#!/bin/bash
# Round-4 starting point on one MI355X: GPU tests, smoke, default bench, kernel-trace profile.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/base
R=$PWD
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > gpurun_out/base/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/base/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/base/smoke.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/base/smoke.log; exit 1; }
tail -1 gpurun_out/base/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/base/bench.log 2>&1 || { echo "bench failed"; tail gpurun_out/base/bench.log; exit 1; }
tail -1 gpurun_out/base/bench.log
rm -rf gpurun_out/base/prof
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/base/prof -o run -- python3 $R/bench.py --steps 5 --warmup 2 > $R/gpurun_out/base/prof.log 2>&1) || { echo "prof failed"; exit 1; }
python tools/prof_summary.py gpurun_out/base/prof > gpurun_out/base/prof_summary.txt 2>&1; head -40 gpurun_out/base/prof_summary.txt
