#!/bin/bash
# Round-4: dual-input level 1 + BN-on-load validation, UNet / BN-UNet bench, BN-UNet kernel-trace profile.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/bn
R=$PWD
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_dual_input.py tests/test_bn_on_load.py tests/ > gpurun_out/bn/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/bn/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bn/bench_unet.log 2>&1 || { echo "bench unet failed"; tail -3 gpurun_out/bn/bench_unet.log; exit 1; }
tail -1 gpurun_out/bn/bench_unet.log | cut -c1-220
timeout -k 10 300 python bench.py --model unet-bn > gpurun_out/bn/bench_bn.log 2>&1 || { echo "bench bn failed"; tail -3 gpurun_out/bn/bench_bn.log; exit 1; }
tail -1 gpurun_out/bn/bench_bn.log | cut -c1-300
rm -rf gpurun_out/bn/prof
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/bn/prof -o run -- python3 $R/bench.py --model unet-bn --steps 5 --warmup 2 > $R/gpurun_out/bn/prof.log 2>&1) || { echo "prof failed"; exit 1; }
python tools/prof_summary.py gpurun_out/bn/prof > gpurun_out/bn/prof_summary.txt 2>&1; head -30 gpurun_out/bn/prof_summary.txt
