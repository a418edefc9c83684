#!/bin/bash
# Round-4 iteration: the named test files, two default benches, one kernel-trace profile.
# usage: bash tools/gpu_r04_quick.sh <out-subdir> <test files...>
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp
R=$PWD; O=gpurun_out/$1; shift; mkdir -p $O
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread "$@" > $O/pytest.log 2>&1
  rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
fi
for i in 1 2; do
  timeout -k 10 300 python bench.py > $O/bench_$i.log 2>&1 || { echo "bench failed"; tail -3 $O/bench_$i.log; exit 1; }
  tail -1 $O/bench_$i.log | cut -c80-200
done
rm -rf $O/prof
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- python3 $R/bench.py --steps 5 --warmup 2 > $R/$O/prof.log 2>&1) || { echo "prof failed"; exit 1; }
python tools/prof_summary.py $O/prof > $O/prof_summary.txt 2>&1; head -24 $O/prof_summary.txt
