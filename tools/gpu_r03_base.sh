#!/bin/bash
# Round-3 baseline on a fresh box: default bench (b256 512^2), the reference's default shape
# 640x960 at batch 4 and a large batch, and a kernel-trace profile at 640x960.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
R=$PWD
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { tail gpurun_out/build.log; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/bench_b256.log 2>&1 || { echo "bench rc=$?"; tail -5 gpurun_out/bench_b256.log; exit 1; }
tail -1 gpurun_out/bench_b256.log
timeout -k 10 300 python bench.py --img 640x960 --batch 4 --steps 20 --warmup 5 > gpurun_out/bench_640x960_b4.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/bench_640x960_b4.log; exit 1; }
tail -1 gpurun_out/bench_640x960_b4.log
timeout -k 10 300 python bench.py --img 640x960 --batch 128 --steps 10 --warmup 3 > gpurun_out/bench_640x960_b128.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/bench_640x960_b128.log; exit 1; }
tail -1 gpurun_out/bench_640x960_b128.log
rm -rf gpurun_out/prof640
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof640 -o run -- python3 $R/bench.py --img 640x960 --batch 128 --steps 5 --warmup 2 > $R/gpurun_out/prof640.log 2>&1) || { echo "prof rc=$?"; exit 1; }
python tools/prof_summary.py gpurun_out/prof640 > gpurun_out/prof640_summary.txt 2>&1; head -45 gpurun_out/prof640_summary.txt
