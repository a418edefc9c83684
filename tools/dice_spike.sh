#!/bin/bash
# Seed-42 epoch-2 validation-loss spike of the HIP run (profiles/dice_parity_512_r02.txt:11): retrain
# the same 2 epochs (same seed, split, schedule), then score the SAME epoch-2 weights on the SAME
# validation images with the HIP engine (bf16) and with stock PyTorch in fp32 (reference semantics).
# Same spike in both -> it is in the weights (training trajectory), not in the engine's forward.
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/dice_spike
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
O=/tmp/dice_spike; rm -rf $O; mkdir -p $O
common="--synthetic --synthetic-len 1024 --img-size 512 -b 16 --lr 3e-4 -s 42"
timeout -k 10 300 python train.py $common -e 2 --backend hip --dtype bf16 --out-dir $O/hip > gpurun_out/dice_spike/train_hip.log 2>&1 || { echo "train rc=$?"; tail -5 gpurun_out/dice_spike/train_hip.log; exit 1; }
cp $O/hip/logs/singleGPU.jsonl gpurun_out/dice_spike/hip_lr3e-4.jsonl
timeout -k 10 300 python evaluate.py --load $O/hip/checkpoints/singleGPU.pth --synthetic --synthetic-len 1024 --img-size 512 -b 16 -s 42 --backend hip > gpurun_out/dice_spike/eval_hip.log 2>&1 || { echo "eval hip rc=$?"; tail -5 gpurun_out/dice_spike/eval_hip.log; exit 1; }
tail -2 gpurun_out/dice_spike/eval_hip.log
MIOPEN_FIND_MODE=FAST timeout -k 10 600 python evaluate.py --load $O/hip/checkpoints/singleGPU.pth --synthetic --synthetic-len 1024 --img-size 512 -b 16 -s 42 --backend torch --dtype fp32 > gpurun_out/dice_spike/eval_torch_fp32.log 2>&1 || { echo "eval torch rc=$?"; tail -5 gpurun_out/dice_spike/eval_torch_fp32.log; exit 1; }
tail -2 gpurun_out/dice_spike/eval_torch_fp32.log
for lr in 1e-4; do
  timeout -k 10 300 python train.py --synthetic --synthetic-len 1024 --img-size 512 -b 16 --lr $lr -s 42 -e 3 --backend hip --dtype bf16 --out-dir $O/hip_$lr > gpurun_out/dice_spike/train_hip_$lr.log 2>&1 || exit 1
  cp $O/hip_$lr/logs/singleGPU.jsonl gpurun_out/dice_spike/hip_lr$lr.jsonl
done
python - <<'PY'
import json
for f in ["hip_lr3e-4", "hip_lr1e-4"]:
    rows = [json.loads(l) for l in open(f"gpurun_out/dice_spike/{f}.jsonl")]
    print(f, [(r["epoch"] + 1, round(r["val_loss"], 4), round(r["val_dice"], 4)) for r in rows if r.get("kind") == "epoch"])
PY
