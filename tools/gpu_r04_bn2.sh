#!/bin/bash
# Round-4: BN-on-load / loader transforms moved into the MFMA region -- tests, benches, BN profile.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/bn2
R=$PWD
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bn_on_load.py tests/test_bwd_fused.py tests/test_dual_input.py tests/test_hip_variants.py > gpurun_out/bn2/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/bn2/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bn2/bench_unet.log 2>&1 || { echo "bench unet failed"; tail -3 gpurun_out/bn2/bench_unet.log; exit 1; }
tail -1 gpurun_out/bn2/bench_unet.log | cut -c1-200
timeout -k 10 300 python bench.py --model unet-bn > gpurun_out/bn2/bench_bn.log 2>&1 || { echo "bench bn failed"; tail -3 gpurun_out/bn2/bench_bn.log; exit 1; }
tail -1 gpurun_out/bn2/bench_bn.log | cut -c1-200
rm -rf gpurun_out/bn2/prof gpurun_out/bn2/profu
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/bn2/prof -o run -- python3 $R/bench.py --model unet-bn --steps 5 --warmup 2 > $R/gpurun_out/bn2/prof.log 2>&1) || { echo "prof failed"; exit 1; }
python tools/prof_summary.py gpurun_out/bn2/prof > gpurun_out/bn2/prof_summary.txt 2>&1; head -24 gpurun_out/bn2/prof_summary.txt
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/bn2/profu -o run -- python3 $R/bench.py --steps 5 --warmup 2 > $R/gpurun_out/bn2/profu.log 2>&1) || { echo "prof unet failed"; exit 1; }
python tools/prof_summary.py gpurun_out/bn2/profu > gpurun_out/bn2/profu_summary.txt 2>&1; head -24 gpurun_out/bn2/profu_summary.txt
