#!/bin/bash
# Round 5 iteration: the whole GPU suite, the bf16 bench, the fp32 bench and an fp32 kernel-trace summary.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/iter
R=$PWD; O=gpurun_out/iter
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail $O/bench.log; exit 1; }
echo "bf16: $(tail -1 $O/bench.log | cut -c80-140)"
timeout -k 10 300 python bench.py --dtype fp32 --batch 16 --steps 10 --warmup 3 > $O/bench_fp32.log 2>&1 || { echo "fp32 bench failed"; tail $O/bench_fp32.log; exit 1; }
echo "fp32: $(tail -1 $O/bench_fp32.log | cut -c80-140)"
rm -rf $O/prof
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- python3 $R/bench.py --dtype fp32 --batch 16 --steps 4 --warmup 2 > $R/$O/prof.log 2>&1) || { echo "prof failed"; exit 1; }
python tools/prof_summary.py $O/prof --timeline > $O/prof_summary_fp32.txt 2>&1; grep -c "torch:" $O/prof_summary_fp32.txt; head -30 $O/prof_summary_fp32.txt
timeout -k 10 300 python tools/f32_kbench.py --batch 16 --img 512 --igemm-wide both > $O/f32_kbench_wide.txt 2>&1 || { echo "kbench failed"; tail $O/f32_kbench_wide.txt; exit 1; }
grep -v amdgpu.ids $O/f32_kbench_wide.txt
for w in 0 1; do
  DPA_F32_IGEMM_WIDE=$w timeout -k 10 300 python bench.py --dtype fp32 --batch 16 --steps 10 --warmup 3 > $O/bench_fp32_wide$w.log 2>&1 || { echo "fp32 bench failed"; exit 1; }
  echo "fp32 wide=$w: $(tail -1 $O/bench_fp32_wide$w.log | cut -c80-140)"
done
for c in 1 2 4 1 2 4; do
  DPA_ENC0_CHUNKS=$c timeout -k 10 300 python bench.py --steps 15 --warmup 3 > $O/bench_chunks$c.log 2>&1 || { echo "bench chunks failed"; exit 1; }
  echo "enc0 chunks=$c: $(tail -1 $O/bench_chunks$c.log | cut -c80-140)"
done
