#!/bin/bash
# Dice parity run (BASELINE.json "Dice parity"): the same synthetic segmentation task, seed, split,
# optimiser and schedule trained twice on one MI355X -- the HIP engine (bf16 kernels) and the
# reference-semantics stock-PyTorch path in fp32 -- and the per-epoch validation loss / Dice of both
# printed side by side (logs/singleGPU.jsonl of each run).
#   DICE_SEEDS="42 7" bash tools/dice_parity.sh [EPOCHS] [IMG] [N_IMAGES]
set -euo pipefail
cd "$(dirname "$0")/.."
E=${1:-6}; S=${2:-256}; NI=${3:-1024}
OUT=${DICE_OUT:-/tmp/dice_parity}   # checkpoints stay out of gpurun_out/ (64 MiB merge cap)
rm -rf "$OUT"; mkdir -p "$OUT"
# stock MIOpen's compiled kernels / find results: reuse ./.miopen, bring new ones back in gpurun_out/miopen
mkdir -p gpurun_out/miopen; if [ -d .miopen ]; then cp -r .miopen/. gpurun_out/miopen/; fi
export MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen MIOPEN_CUSTOM_CACHE_DIR=$PWD/gpurun_out/miopen
for SEED in ${DICE_SEEDS:-42}; do
  common="--synthetic --synthetic-len $NI --img-size $S -b 16 -e $E --lr 3e-4 -s $SEED"
  timeout -k 10 900 python train.py $common --backend hip --dtype bf16 --out-dir "$OUT/hip$SEED" > "$OUT/hip$SEED.log" 2>&1
  echo "hip seed $SEED done"
  timeout -k 10 900 python train.py $common --backend torch --dtype fp32 --out-dir "$OUT/torch$SEED" > "$OUT/torch$SEED.log" 2>&1
  echo "torch seed $SEED done"
done
python - "$OUT" ${DICE_SEEDS:-42} <<'PY'
import json, sys, os
out, seeds = sys.argv[1], sys.argv[2:]
def epochs(run):
    rows = [json.loads(l) for l in open(os.path.join(out, run, "logs", "singleGPU.jsonl"))]
    return [r for r in rows if r.get("kind") == "epoch"]
for seed in seeds:
    h, t = epochs("hip" + seed), epochs("torch" + seed)
    print(f"seed {seed}")
    print(f"{'epoch':>5} | {'HIP bf16 val_loss':>17} {'Dice':>6} {'img/s':>7} | {'torch fp32 val_loss':>19} {'Dice':>6} {'img/s':>7}")
    for a, b in zip(h, t):
        print(f"{a['epoch'] + 1:>5} | {a['val_loss']:17.4f} {a['val_dice']:6.4f} {a['img_per_s']:7.1f} | "
              f"{b['val_loss']:19.4f} {b['val_dice']:6.4f} {b['img_per_s']:7.1f}")
    print(f"best Dice: HIP {max(r['val_dice'] for r in h):.4f}  torch {max(r['val_dice'] for r in t):.4f}; "
          f"last-3-epoch mean: HIP {sum(r['val_dice'] for r in h[-3:]) / 3:.4f}  torch {sum(r['val_dice'] for r in t[-3:]) / 3:.4f}")
PY
