#!/bin/bash
# Dice parity at the bench batch (round 4): the same synthetic segmentation task, seed, split, optimiser
# and schedule trained on one MI355X by the bf16 HIP engine and by the fp32 HIP engine (the reference's
# precision, hand-written fp32-MFMA kernels); per-epoch validation loss / Dice side by side.
#   DICE_SEEDS="42 7" bash tools/dice_parity_r04.sh [EPOCHS] [IMG] [N_IMAGES] [BATCH] [LR]
set -euo pipefail
cd "$(dirname "$0")/.."
E=${1:-10}; S=${2:-512}; NI=${3:-4096}; B=${4:-256}; LR=${5:-1e-3}
OUT=${DICE_OUT:-/tmp/dice_parity_r04}
rm -rf "$OUT"; mkdir -p "$OUT" gpurun_out/dice
for SEED in ${DICE_SEEDS:-42}; do
  common="--synthetic --synthetic-len $NI --img-size $S -b $B -e $E --lr $LR -s $SEED"
  timeout -k 10 900 python train.py $common --backend hip --dtype bf16 --out-dir "$OUT/bf16_$SEED" > "$OUT/bf16_$SEED.log" 2>&1
  echo "bf16 seed $SEED done"
  timeout -k 10 1000 python train.py $common --backend hip --dtype fp32 --out-dir "$OUT/fp32_$SEED" > "$OUT/fp32_$SEED.log" 2>&1
  echo "fp32 seed $SEED done"
done
python - "$OUT" ${DICE_SEEDS:-42} <<'PY' | tee gpurun_out/dice/dice_parity_r04.txt
import json, sys, os
out, seeds = sys.argv[1], sys.argv[2:]
def epochs(run):
    rows = [json.loads(l) for l in open(os.path.join(out, run, "logs", "singleGPU.jsonl"))]
    return [r for r in rows if r.get("kind") == "epoch"]
for seed in seeds:
    h, t = epochs("bf16_" + seed), epochs("fp32_" + seed)
    print(f"seed {seed}")
    print(f"{'epoch':>5} | {'HIP bf16 val_loss':>17} {'Dice':>6} {'img/s':>7} | {'HIP fp32 val_loss':>17} {'Dice':>6} {'img/s':>7}")
    for a, b in zip(h, t):
        print(f"{a['epoch'] + 1:>5} | {a['val_loss']:17.4f} {a['val_dice']:6.4f} {a['img_per_s']:7.1f} | "
              f"{b['val_loss']:17.4f} {b['val_dice']:6.4f} {b['img_per_s']:7.1f}")
    print(f"best Dice: bf16 {max(r['val_dice'] for r in h):.4f}  fp32 {max(r['val_dice'] for r in t):.4f}; "
          f"last-3-epoch mean: bf16 {sum(r['val_dice'] for r in h[-3:]) / 3:.4f}  fp32 {sum(r['val_dice'] for r in t[-3:]) / 3:.4f}")
PY
