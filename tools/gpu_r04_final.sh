#!/bin/bash
# Round-4 end.  PART=tests: every GPU test + smoke.  PART=bench: the default bench (x2), the BN and fp32
# benches, a kernel-trace profile of the default step.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/final
R=$PWD; O=gpurun_out/final
if [ "${PART:-tests}" = tests ]; then
  timeout -k 10 1000 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.log 2>&1
  rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
  exit 0
fi
for i in 1 2; do
  timeout -k 10 300 python bench.py > $O/bench_$i.log 2>&1 || { echo "bench failed"; tail -3 $O/bench_$i.log; exit 1; }
  tail -1 $O/bench_$i.log | cut -c80-200
done
timeout -k 10 300 python bench.py --model unet-bn > $O/bench_bn.log 2>&1 || { echo "bn bench failed"; tail -3 $O/bench_bn.log; exit 1; }
tail -1 $O/bench_bn.log | cut -c80-200
timeout -k 10 300 python bench.py --dtype fp32 --batch 16 --steps 8 --warmup 2 > $O/bench_fp32.log 2>&1 || { echo "fp32 bench failed"; tail -3 $O/bench_fp32.log; exit 1; }
tail -1 $O/bench_fp32.log | cut -c80-200
rm -rf $O/prof
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- python3 $R/bench.py --steps 5 --warmup 2 > $R/$O/prof.log 2>&1) || { echo "prof failed"; exit 1; }
python tools/prof_summary.py $O/prof > $O/prof_summary.txt 2>&1; head -12 $O/prof_summary.txt
