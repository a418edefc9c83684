#!/bin/bash
# Round-5 starting point on one MI355X: GPU tests, smoke, default bench, kernel-trace profile, and the
# one-GPU pipeline rehearsal of the reference cut vs the mirrored V placement (2 stages on cuda:0).
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/base
R=$PWD; O=gpurun_out/base
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.log 2>&1
rc=$?; tail -4 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-400
for cut in reference v; do
  timeout -k 10 300 python bench.py --parallelism mp --stages 2 --mp-cut $cut --microbatches 8 --steps 10 --warmup 3 > $O/mp_$cut.log 2>&1 || { echo "mp $cut failed"; tail $O/mp_$cut.log; exit 1; }
  tail -1 $O/mp_$cut.log | cut -c1-300
done
rm -rf $O/prof
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- python3 $R/bench.py --steps 5 --warmup 2 > $R/$O/prof.log 2>&1) || { echo "prof failed"; exit 1; }
python tools/prof_summary.py $O/prof > $O/prof_summary.txt 2>&1; head -40 $O/prof_summary.txt
