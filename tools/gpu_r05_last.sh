#!/bin/bash
# last check of the round's final tree: whole GPU suite, smoke, bf16 + BN bench
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/last
O=gpurun_out/last
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail $O/bench.log; exit 1; }
echo "bf16: $(tail -1 $O/bench.log | cut -c80-140)"
timeout -k 10 300 python bench.py --model unet-bn --steps 10 --warmup 3 > $O/bench_bn.log 2>&1 || { echo "bn bench failed"; exit 1; }
echo "bn: $(tail -1 $O/bench_bn.log | cut -c80-140)"
