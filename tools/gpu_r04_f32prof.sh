#!/bin/bash
# Round-4: fp32 engine kernel profile (hand-written fp32 kernels vs stock PyTorch fp32), block-time tables.
set -o pipefail
cd "$(dirname "$0")/.." && R=$(pwd) && export TMPDIR=/tmp && mkdir -p gpurun_out/f32prof gpurun_out/bt2
O=$R/gpurun_out/f32prof
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/hip -o run -- python3 $R/bench.py --dtype fp32 --batch 16 --steps 4 --warmup 2 > $O/hip.log 2>&1) || { echo "hip prof failed"; tail -3 $O/hip.log; exit 1; }
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/torch -o run -- python3 $R/bench.py --dtype fp32 --backend torch --batch 16 --steps 4 --warmup 2 > $O/torch.log 2>&1) || { echo "torch prof failed"; tail -3 $O/torch.log; exit 1; }
O=gpurun_out/bt2
if [ -z "$NO_BT" ]; then
timeout -k 10 600 python -u tools/block_times.py --model unet --img 512 --mbs 8 16 32 64 128 256 --out $O/block_times_unet_512.json > $O/bt_unet.log 2>&1 || { echo bt unet failed; tail $O/bt_unet.log; exit 1; }
tail -2 $O/bt_unet.log
timeout -k 10 600 python -u tools/block_times.py --model unet-xl --img 1024 --mbs 1 2 4 8 16 --out $O/block_times_unetxl_1024.json > $O/bt_xl.log 2>&1 || { echo bt xl failed; tail $O/bt_xl.log; exit 1; }
tail -2 $O/bt_xl.log
fi
