#!/bin/bash
# Stock-PyTorch (MIOpen) baseline on one MI355X: tests, bench, rocprof kernel stats.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo build failed; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 400 python bench.py --backend torch --steps 20 --warmup 5 --batch 32 > gpurun_out/bench_torch_b32.log 2>&1 || { echo bench failed; tail -30 gpurun_out/bench_torch_b32.log; exit 1; }
tail -2 gpurun_out/bench_torch_b32.log
timeout -k 10 300 python bench.py --backend torch --steps 10 --warmup 3 --batch 8 > gpurun_out/bench_torch_b8.log 2>&1 && tail -1 gpurun_out/bench_torch_b8.log
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_torch -o run -- python3 $GRAFT_REPO_ROOT/bench.py --backend torch --steps 5 --warmup 3 --batch 32 > $GRAFT_REPO_ROOT/gpurun_out/prof_torch.log 2>&1; echo "prof rc=$?"
find $GRAFT_REPO_ROOT/gpurun_out/prof_torch -name '*stats*' | head
