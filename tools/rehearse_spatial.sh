#!/bin/bash
# One-GPU rehearsal of the config-5 row-split pipeline (UNet-XL 1024^2, 8 stages, b16): all 8 ranks on cuda:0 over
# gloo (host-staged P2P), so this checks the engine end to end at the real size -- memory per rank and
# compute only, no link time.  Usage: bash tools/rehearse_spatial.sh
O=gpurun_out/s24; mkdir -p $O
export DPA_SAME_DEVICE=1 DPA_DIST_BACKEND=gloo
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 8 --parallelism mp --mp-cut spatial --model unet-xl --img 1024 --batch 16 --steps 2 --warmup 1 --out $O/bench.jsonl > $O/spatial8.log 2>&1
