#!/bin/bash
# A/B of the weight-gradient side-stream priority on one box (alternating runs, default batch 256).
set -e
python -c "import torch; print('priority range', torch.cuda.Stream.priority_range())"
for i in 1 2; do
  for p in 0 -1; do
    DPA_SIDE_PRIORITY=$p timeout -k 10 200 python bench.py --steps 10 --warmup 3 > gpurun_out/prio_${p}_$i.log 2>&1
    echo "prio=$p run=$i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/prio_${p}_$i.log)"
  done
done
