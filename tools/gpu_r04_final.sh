#!/bin/bash
# Round-4 end: every GPU test, smoke, the default bench (x2), a kernel-trace profile of the step.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/final
R=$PWD; O=gpurun_out/final
timeout -k 10 1100 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for i in 1 2; do
  timeout -k 10 300 python bench.py > $O/bench_$i.log 2>&1 || { echo "bench failed"; tail -3 $O/bench_$i.log; exit 1; }
  tail -1 $O/bench_$i.log | cut -c80-200
done
rm -rf $O/prof
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- python3 $R/bench.py --steps 5 --warmup 2 > $R/$O/prof.log 2>&1) || { echo "prof failed"; exit 1; }
python tools/prof_summary.py $O/prof > $O/prof_summary.txt 2>&1; head -12 $O/prof_summary.txt
