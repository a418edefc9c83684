#!/bin/bash
# Round-4: conv-level pipeline cuts -- half-block tests, head prefetch tests, bench, unit block-time tables.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/split
O=gpurun_out/split
timeout -k 10 600 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_split_blocks.py tests/test_fp32_engine.py tests/test_hip_multirank.py tests/test_bwd_fused.py tests/test_hip_kernels.py tests/test_hip_model.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py > $O/bench_$i.log 2>&1 || { echo "bench failed"; tail -3 $O/bench_$i.log; exit 1; }
  tail -1 $O/bench_$i.log | cut -c80-200
done
timeout -k 10 600 python -u tools/block_times.py --model unet --img 512 --mbs 8 16 32 64 128 256 --out $O/block_times_unet_512.json > $O/bt_unet.log 2>&1 || { echo bt unet failed; tail $O/bt_unet.log; exit 1; }
tail -2 $O/bt_unet.log
timeout -k 10 600 python -u tools/block_times.py --model unet-xl --img 1024 --mbs 1 2 4 8 16 --out $O/block_times_unetxl_1024.json > $O/bt_xl.log 2>&1 || { echo bt xl failed; tail $O/bt_xl.log; exit 1; }
tail -2 $O/bt_xl.log
