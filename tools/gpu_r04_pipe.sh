#!/bin/bash
# Round-4 iteration: tests of the changed kernels, slice-staged GEMM timing, bench, per-block time tables.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/sl gpurun_out/pipe
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bn_on_load.py tests/test_bwd_fused.py > gpurun_out/sl/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/sl/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > gpurun_out/sl/bench.log 2>&1 || { echo bench failed; tail -3 gpurun_out/sl/bench.log; exit 1; }
tail -1 gpurun_out/sl/bench.log | cut -c1-200
timeout -k 10 300 python tools/kbench.py --batch 256 --paths "" --no-wgrad --gvar 14 15 262144 524288 --reps 7 --only "L2,L3,mid" > gpurun_out/sl/kbench.log 2>&1 || { echo kbench failed; tail gpurun_out/sl/kbench.log; exit 1; }
grep -v "n/a" gpurun_out/sl/kbench.log
timeout -k 10 400 python -u tools/block_times.py --model unet --img 512 --mbs 8 16 32 64 128 256 --out gpurun_out/pipe/block_times_unet_512.json > gpurun_out/pipe/bt_unet.log 2>&1 || { echo bt unet failed; tail gpurun_out/pipe/bt_unet.log; exit 1; }
tail -2 gpurun_out/pipe/bt_unet.log
timeout -k 10 400 python -u tools/block_times.py --model unet-xl --img 1024 --mbs 1 2 4 8 16 --out gpurun_out/pipe/block_times_unetxl_1024.json > gpurun_out/pipe/bt_xl.log 2>&1 || { echo bt xl failed; tail gpurun_out/pipe/bt_xl.log; exit 1; }
tail -2 gpurun_out/pipe/bt_xl.log
timeout -k 10 400 python -u tools/defer_mem.py --model unet --img 512 --stages 2 --microbatches 8 --batch 256 --cap-gb 8 64 > gpurun_out/pipe/defer_unet.log 2>&1 || { echo defer unet failed; tail -3 gpurun_out/pipe/defer_unet.log; exit 1; }
cat gpurun_out/pipe/defer_unet.log | grep peak_gb
timeout -k 10 400 python -u tools/defer_mem.py --model unet-xl --img 1024 --stages 8 --microbatches 8 --batch 16 --cap-gb 8 64 > gpurun_out/pipe/defer_xl.log 2>&1 || { echo defer xl failed; tail -3 gpurun_out/pipe/defer_xl.log; exit 1; }
cat gpurun_out/pipe/defer_xl.log | grep peak_gb
