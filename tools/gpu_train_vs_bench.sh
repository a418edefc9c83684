#!/bin/bash
# train.py (HBM-resident synthetic data, full trainer loop) vs bench.py at the headline config.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
B=${BATCH:-256}
timeout -k 10 400 python train.py --synthetic --img-size 512 -b $B -e 1 --max-steps ${STEPS:-30} --log-every 10 \
  --out-dir /tmp/trainrun > gpurun_out/train_512_b$B.log 2>&1; rc=$?; echo "train rc=$rc"; grep -v amdgpu gpurun_out/train_512_b$B.log | tail -4
[ $rc -ne 0 ] && exit $rc
cp /tmp/trainrun/logs/singleGPU.jsonl gpurun_out/train_512_b$B.jsonl 2>/dev/null
timeout -k 10 300 python bench.py --batch $B --steps 20 --warmup 5 > gpurun_out/bench_b$B.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_b$B.log
exit $rc
