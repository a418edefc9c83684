#!/bin/bash
# Stock PyTorch-ROCm (MIOpen) baseline of the same training step (reference architecture, bf16 autocast).
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
export MIOPEN_FIND_MODE=${MIOPEN_FIND_MODE:-FAST}
export MIOPEN_LOG_LEVEL=${MIOPEN_LOG_LEVEL:-3}
timeout -k 10 ${TB_TIMEOUT:-1000} python bench.py --backend torch --steps ${TB_STEPS:-10} --warmup ${TB_WARMUP:-3} --batch ${TB_BATCH:-8} 2>&1 > gpurun_out/bench_torch.log 2>&1; echo "torch bench rc=$?"; grep -v amdgpu.ids gpurun_out/bench_torch.log | tail -3
