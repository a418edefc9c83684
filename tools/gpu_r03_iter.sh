#!/bin/bash
# Round-3 iteration: selected GPU tests (TESTS, default the kernel/model/strategy files), then the
# default bench and the 640x960 bench (BENCH_ARGS / BENCH640_ARGS), optional profile (PROF_ARGS).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
R=$PWD
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { tail gpurun_out/build.log; exit 1; }
TESTS=${TESTS:-"tests/test_hip_kernels.py tests/test_hip_model.py"}
if [ "$TESTS" != "none" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu $TESTS > gpurun_out/pytest_iter.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_iter.log; [ $rc -ne 0 ] && exit $rc
fi
if [ "${BENCH_ARGS}" != "none" ]; then
  timeout -k 10 300 python bench.py ${BENCH_ARGS} > gpurun_out/bench_iter.log 2>&1 || { echo "bench rc=$?"; tail -5 gpurun_out/bench_iter.log; exit 1; }
  tail -1 gpurun_out/bench_iter.log
fi
if [ -n "${BENCH640_ARGS}" ]; then
  timeout -k 10 300 python bench.py ${BENCH640_ARGS} > gpurun_out/bench640_iter.log 2>&1 || { echo "bench640 rc=$?"; tail -5 gpurun_out/bench640_iter.log; exit 1; }
  tail -1 gpurun_out/bench640_iter.log
fi
if [ -n "${PROF_ARGS}" ]; then
  rm -rf gpurun_out/prof_iter
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_iter -o run -- python3 $R/bench.py ${PROF_ARGS} > $R/gpurun_out/prof_iter.log 2>&1) || { echo "prof rc=$?"; exit 1; }
  python tools/prof_summary.py gpurun_out/prof_iter > gpurun_out/prof_iter_summary.txt 2>&1; head -40 gpurun_out/prof_iter_summary.txt
fi
exit 0
