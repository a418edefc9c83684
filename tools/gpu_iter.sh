#!/bin/bash
# One iteration: build, GPU tests, bench (batch $BATCH), rocprofv3 kernel stats of the bench.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
R=$PWD
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { tail gpurun_out/build.log; exit 1; }
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --batch ${BATCH:-32} > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log
[ $rc -ne 0 ] && exit $rc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python3 $R/bench.py --steps 5 --warmup 2 --batch ${BATCH:-32} > $R/gpurun_out/prof.log 2>&1; echo "prof rc=$?"; cd $R
if [ -n "$KBENCH" ]; then timeout -k 10 300 python tools/kbench.py $KBENCH > gpurun_out/kbench.log 2>&1; echo "kbench rc=$?"; cat gpurun_out/kbench.log | grep -v amdgpu; fi
if [ -n "$DDP_REHEARSAL" ]; then
  DPA_SAME_DEVICE=1 DPA_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 2 --batch 4 > gpurun_out/ddp_rehearsal.log 2>&1; echo "ddp rehearsal rc=$?"; grep -v amdgpu.ids gpurun_out/ddp_rehearsal.log | tail -3
  DPA_SAME_DEVICE=1 DPA_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 train.py -t DDP --synthetic --synthetic-len 16 --img-size 128 -e 1 -b 2 --out-dir /tmp/ddp_train > gpurun_out/ddp_train.log 2>&1; echo "ddp train rc=$?"; grep -v amdgpu.ids gpurun_out/ddp_train.log | tail -3
fi
