#!/bin/bash
# Round 5 end validation: whole GPU suite, smoke(), bf16 / BN / fp32 benches, kernel-trace summaries of the
# bf16 and BN steps (rocprofv3, one run each) for profiles/.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/final
R=$PWD; O=gpurun_out/final
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for i in 1 2; do
  timeout -k 10 300 python bench.py > $O/bench_$i.log 2>&1 || { echo "bench failed"; tail $O/bench_$i.log; exit 1; }
  echo "bf16 $i: $(tail -1 $O/bench_$i.log | cut -c80-140)"
done
timeout -k 10 300 python bench.py --model unet-bn --steps 10 --warmup 3 > $O/bench_bn.log 2>&1 || { echo "bn bench failed"; tail $O/bench_bn.log; exit 1; }
echo "bn: $(tail -1 $O/bench_bn.log | cut -c80-140)"
timeout -k 10 300 python bench.py --dtype fp32 --batch 16 --steps 20 --warmup 3 > $O/bench_fp32.log 2>&1 || { echo "fp32 bench failed"; tail $O/bench_fp32.log; exit 1; }
echo "fp32: $(tail -1 $O/bench_fp32.log | cut -c80-140)"
rm -rf $O/prof $O/profbn
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- python3 $R/bench.py --steps 5 --warmup 2 > $R/$O/prof.log 2>&1) || { echo "prof failed"; exit 1; }
python tools/prof_summary.py $O/prof --timeline > $O/prof_summary_bf16.txt 2>&1; head -8 $O/prof_summary_bf16.txt | cut -c1-120
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/profbn -o run -- python3 $R/bench.py --model unet-bn --steps 5 --warmup 2 > $R/$O/profbn.log 2>&1) || { echo "profbn failed"; exit 1; }
python tools/prof_summary.py $O/profbn --timeline > $O/prof_summary_bn.txt 2>&1; head -8 $O/prof_summary_bn.txt | cut -c1-120
