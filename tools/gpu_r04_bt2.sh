#!/bin/bash
# Round-4: block-time tables re-measured without the skip-leaf gradient copy (tools/block_times.py
# accumulates only parameters and the block input), then the launch-geometry knob A/B.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/bt2
O=gpurun_out/bt2
timeout -k 10 600 python -u tools/block_times.py --model unet --img 512 --mbs 8 16 32 64 128 256 --out $O/block_times_unet_512.json > $O/bt_unet.log 2>&1 || { echo bt unet failed; tail $O/bt_unet.log; exit 1; }
tail -2 $O/bt_unet.log
timeout -k 10 600 python -u tools/block_times.py --model unet-xl --img 1024 --mbs 1 2 4 8 16 --out $O/block_times_unetxl_1024.json > $O/bt_xl.log 2>&1 || { echo bt xl failed; tail $O/bt_xl.log; exit 1; }
tail -2 $O/bt_xl.log
[ -z "$SKIP_KNOBS" ] && bash tools/gpu_r04_knobs.sh; true
