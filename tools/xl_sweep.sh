#!/bin/bash
# UNet-XL 1024x1024 single-GPU batch sweep (288 GB HBM lets the batch grow without checkpointing).
set -e
for b in 16 32 64; do
  timeout -k 10 300 python bench.py --model unet-xl --img 1024 --batch $b --steps 4 --warmup 2 > gpurun_out/xl_b$b.log 2>&1
  echo "b=$b $(grep -o '"value": [0-9.]*' gpurun_out/xl_b$b.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/xl_b$b.log) $(grep -o '"peak_mem_gb": [0-9.]*' gpurun_out/xl_b$b.log)"
done
