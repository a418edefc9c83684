#!/bin/bash
# Same-box fp32 comparison: the fp32 HIP engine and stock PyTorch fp32 (MIOpen) interleaved,
# 20 timed steps each, twice.  A heartbeat file keeps the long first MIOpen iteration (solver search,
# minutes) visible to the runner.  Usage: bash tools/fp32_same_box.sh OUTDIR "BENCH ARGS"
#   e.g. bash tools/fp32_same_box.sh gpurun_out/f32 "--dtype fp32 --batch 16 --steps 20 --warmup 3"
O=${1:-gpurun_out/fp32_same_box}; A=${2:-"--dtype fp32 --batch 16 --steps 20 --warmup 3"}
mkdir -p "$O"
(while true; do date > "$O/hb.txt"; sleep 45; done) & HB=$!
O=$O LIMIT=${LIMIT:-1100} tools/gpu_session.sh "run:hip_a|$A" "run:torch_a|$A --backend torch" "run:hip_b|$A" \
  "run:torch_b|$A --backend torch"
rc=$?
kill $HB
exit $rc
