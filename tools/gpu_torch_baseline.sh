#!/bin/bash
# Stock PyTorch-ROCm (MIOpen) baseline of the same training step (reference architecture, bf16 autocast,
# channels_last), at per-GPU batch $TB_BATCH.  MIOpen's compiled kernels and find results go to
# gpurun_out/miopen (merged back by gpurun); copy that directory to ./.miopen before the next call and
# it is reused (first-iteration compilation took minutes per batch size on a cold box).
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/miopen
if [ -d .miopen ]; then cp -r .miopen/. gpurun_out/miopen/; fi
export MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen
export MIOPEN_CUSTOM_CACHE_DIR=$PWD/gpurun_out/miopen
export MIOPEN_FIND_MODE=${MIOPEN_FIND_MODE:-FAST}
B=${TB_BATCH:-32}
timeout -k 10 ${TB_TIMEOUT:-1000} python bench.py --backend torch --steps ${TB_STEPS:-10} --warmup ${TB_WARMUP:-3} \
  --batch $B > gpurun_out/bench_torch_b$B.log 2>&1; rc=$?
echo "torch bench b$B rc=$rc"; grep -v amdgpu.ids gpurun_out/bench_torch_b$B.log | tail -3; du -sh gpurun_out/miopen
exit $rc
