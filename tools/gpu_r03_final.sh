#!/bin/bash
# End-of-round validation on one MI355X: every GPU test, smoke(), the default bench, the reference's
# default shape (640x960) at batch 4 through bench.py and train.py (peak HBM vs the reference's 7.8 GB),
# and a kernel-trace profile of the default bench.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/final
R=$PWD
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/final/build.log 2>&1 || { tail gpurun_out/final/build.log; exit 1; }
timeout -k 10 1500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/final/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/final/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/final/bench.log 2>&1 || { echo "bench failed"; exit 1; }
tail -1 gpurun_out/final/bench.log
timeout -k 10 300 python bench.py --img 640x960 --batch 4 --steps 50 --warmup 10 > gpurun_out/final/bench_640x960_b4.log 2>&1 || exit 1
tail -1 gpurun_out/final/bench_640x960_b4.log
timeout -k 10 300 python train.py --synthetic --synthetic-len 512 -e 2 -b 4 --out-dir /tmp/tr640 > gpurun_out/final/train_640x960_b4.log 2>&1 || { echo "train failed"; tail -5 gpurun_out/final/train_640x960_b4.log; exit 1; }
cp /tmp/tr640/logs/singleGPU.jsonl gpurun_out/final/train_640x960_b4.jsonl
grep '"epoch"' gpurun_out/final/train_640x960_b4.jsonl | tail -1
rm -rf gpurun_out/final/prof
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/final/prof -o run -- python3 $R/bench.py --steps 5 --warmup 2 > $R/gpurun_out/final/prof.log 2>&1) || { echo "prof failed"; exit 1; }
python tools/prof_summary.py gpurun_out/final/prof > gpurun_out/final/prof_summary.txt 2>&1; head -12 gpurun_out/final/prof_summary.txt
