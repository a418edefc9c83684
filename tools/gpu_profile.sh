#!/bin/bash
# rocprofv3 kernel-trace stats of the HIP bench + the stock-PyTorch (MIOpen) baseline.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
R=$PWD
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --backend hip --steps 20 --warmup 5 --batch ${BATCH:-32} > gpurun_out/bench_hip_b${BATCH:-32}.log 2>&1; echo "bench rc=$?"; tail -1 gpurun_out/bench_hip_b${BATCH:-32}.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_hip -o run -- python3 $R/bench.py --backend hip --steps 5 --warmup 2 --batch ${BATCH:-32} > $R/gpurun_out/prof_hip.log 2>&1; echo "prof rc=$?"
cd $R
if [ -n "$TORCH_BASE" ]; then
  MIOPEN_FIND_MODE=FAST timeout -k 10 500 python bench.py --backend torch --steps 10 --warmup 3 --batch ${BATCH:-32} > gpurun_out/bench_torch.log 2>&1; echo "torch bench rc=$?"; tail -2 gpurun_out/bench_torch.log
fi
