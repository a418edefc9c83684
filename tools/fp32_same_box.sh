#!/bin/bash
# Same-box fp32 comparison: the fp32 HIP engine and stock PyTorch fp32 (MIOpen) interleaved,
# b16 512^2 and the reference default 640x960 b4, 20 timed steps each; a heartbeat file keeps the long
# first MIOpen iteration (solver search, minutes) visible to the runner.  Usage: bash tools/fp32_same_box.sh
O=gpurun_out/s10; mkdir -p $O
(while true; do date > $O/hb.txt; sleep 45; done) & HB=$!
F="--dtype fp32 --batch 16 --steps 20 --warmup 3"
G="--dtype fp32 --img 640x960 --batch 4 --steps 20 --warmup 3"
O=$O LIMIT=1100 tools/gpu_session.sh "run:f32_hip_a|$F" "run:f32_torch_a|$F --backend torch" "run:f32_hip_b|$F" "run:f32_torch_b|$F --backend torch" "run:f32_hip_960a|$G" "run:f32_torch_960a|$G --backend torch" "run:f32_hip_960b|$G" "run:f32_torch_960b|$G --backend torch"
rc=$?; kill $HB; exit $rc
