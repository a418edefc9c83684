#!/bin/bash
# Single-GPU pipeline rehearsals (all stages on cuda:0) vs the single-stage step, same batch.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
B=${BATCH:-256}
run() { local name=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/pipe_$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/pipe_$name.log; return 1; }; echo "$name $(grep '^{' gpurun_out/pipe_$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "img/s", d["ms_per_step"], "ms", d["config"]["parallelism"], d["config"].get("mp_cut"))')"; }
run single --batch $B --steps 10 --warmup 3 &&
run mp2ref --batch $B --steps 10 --warmup 3 --parallelism mp --stages 2 --microbatches ${MB:-8} &&
run mp2bal --batch $B --steps 10 --warmup 3 --parallelism mp --stages 2 --microbatches ${MB:-8} --mp-cut balanced &&
run mp2mb4 --batch $B --steps 10 --warmup 3 --parallelism mp --stages 2 --microbatches 4 &&
run xl1 --model unet-xl --img 1024 --batch 16 --steps 10 --warmup 4 &&
run xl8 --model unet-xl --img 1024 --batch 16 --steps 10 --warmup 4 --parallelism mp --stages 8 --microbatches 8 &&
run xl8mb4 --model unet-xl --img 1024 --batch 16 --steps 10 --warmup 4 --parallelism mp --stages 8 --microbatches 4
