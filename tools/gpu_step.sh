#!/bin/bash
# One gpurun call, no rebuild (the in-tree .so travels with the snapshot).  Steps chosen by env:
#   GEMM="<glds_variant_check args>"  SKEL="<gemm_skeleton args>"  TESTS=1 (pytest -m gpu + smoke)
#   BENCH="<bench args>" (repeatable via BENCH2)  PROF="<bench args>" (rocprofv3 kernel trace)
# Every GPU step has its own timeout; the script stops at the first failing step.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$PWD
if [ -n "$GEMM" ]; then timeout -k 10 300 python tools/glds_variant_check.py $GEMM > gpurun_out/gemm_check.log 2>&1; rc=$?; echo "gemm check rc=$rc"; grep -v amdgpu.ids gpurun_out/gemm_check.log | tail -20; [ $rc -ne 0 ] && exit $rc; fi
if [ -n "$SKEL" ]; then timeout -k 10 300 python tools/gemm_skeleton.py $SKEL > gpurun_out/gemm_skel.log 2>&1; rc=$?; echo "skeleton rc=$rc"; grep -v amdgpu.ids gpurun_out/gemm_skel.log; [ $rc -ne 0 ] && exit $rc; fi
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log; [ $rc -ne 0 ] && exit $rc
fi
for b in BENCH BENCH2 BENCH3; do
  v="${!b}"; [ -z "$v" ] && continue
  [ "$v" = "default" ] && v=""
  timeout -k 10 300 python bench.py $v > gpurun_out/$b.log 2>&1; rc=$?; echo "$b rc=$rc"; tail -1 gpurun_out/$b.log; [ $rc -ne 0 ] && exit $rc
done
if [ -n "$PROF" ]; then
  rm -rf gpurun_out/prof
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py $PROF > $R/gpurun_out/prof.log 2>&1); rc=$?; echo "prof rc=$rc"; [ $rc -ne 0 ] && exit $rc
  python tools/prof_summary.py gpurun_out/prof > gpurun_out/prof_summary.txt 2>&1; head -40 gpurun_out/prof_summary.txt
fi
exit 0
