#!/bin/bash
# final-tree numbers for the other BASELINE configs on one GPU: UNet-XL 1024^2 single stage, the 2-stage -t MP
# V plan rehearsal (both stages on cuda:0), and the 2-rank DDP path over gloo (ranks share cuda:0)
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/configs
O=gpurun_out/configs
timeout -k 10 300 python bench.py --model unet-xl --img 1024 --batch 16 --steps 6 --warmup 2 > $O/xl.log 2>&1 || { echo "xl failed"; tail -3 $O/xl.log; exit 1; }
echo "xl: $(tail -1 $O/xl.log | cut -c80-150)"
timeout -k 10 300 python bench.py --parallelism mp --stages 2 --steps 10 --warmup 3 > $O/mp2.log 2>&1 || { echo "mp2 failed"; tail -3 $O/mp2.log; exit 1; }
echo "mp2: $(tail -1 $O/mp2.log | cut -c80-150)"
DPA_SAME_DEVICE=1 DPA_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --batch 64 --steps 5 --warmup 2 > $O/ddp2.log 2>&1 || { echo "ddp2 failed"; tail -5 $O/ddp2.log; exit 1; }
echo "ddp2 (gloo, one GPU): $(grep '"metric"' $O/ddp2.log | tail -1 | cut -c80-150)"
