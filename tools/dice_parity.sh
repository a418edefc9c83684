#!/bin/bash
# Dice parity run (BASELINE.json "Dice parity"): the same synthetic segmentation task, seed, split,
# optimiser and schedule trained twice on one MI355X -- the HIP engine (bf16 kernels) and the
# reference-semantics stock-PyTorch path in fp32 -- and the per-epoch validation loss / Dice of both
# printed side by side (logs/singleGPU.jsonl of each run).
#   bash tools/dice_parity.sh [EPOCHS] [IMG] [N_IMAGES]
set -euo pipefail
cd "$(dirname "$0")/.."
E=${1:-6}; S=${2:-256}; NI=${3:-1024}
OUT=${DICE_OUT:-/tmp/dice_parity}   # checkpoints stay out of gpurun_out/ (64 MiB merge cap)
rm -rf "$OUT"; mkdir -p "$OUT"
common="--synthetic --synthetic-len $NI --img-size $S -b 16 -e $E --lr 3e-4 -s 42"
timeout -k 10 900 python train.py $common --backend hip --dtype bf16 --out-dir "$OUT/hip" > "$OUT/hip.log" 2>&1
timeout -k 10 900 python train.py $common --backend torch --dtype fp32 --out-dir "$OUT/torch" > "$OUT/torch.log" 2>&1
python - "$OUT" <<'PY'
import json, sys, os
out = sys.argv[1]
def epochs(run):
    rows = [json.loads(l) for l in open(os.path.join(out, run, "logs", "singleGPU.jsonl"))]
    return [r for r in rows if r.get("kind") == "epoch"]
h, t = epochs("hip"), epochs("torch")
print(f"{'epoch':>5} | {'HIP bf16 val_loss':>17} {'Dice':>6} {'img/s':>7} | {'torch fp32 val_loss':>19} {'Dice':>6} {'img/s':>7}")
for a, b in zip(h, t):
    print(f"{a['epoch'] + 1:>5} | {a['val_loss']:17.4f} {a['val_dice']:6.4f} {a['img_per_s']:7.1f} | "
          f"{b['val_loss']:19.4f} {b['val_dice']:6.4f} {b['img_per_s']:7.1f}")
PY
