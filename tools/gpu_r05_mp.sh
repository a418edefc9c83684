#!/bin/bash
# Round 5: -t MP plans vs the reference default on ONE box (one-GPU rehearsals: all stages on cuda:0, so
# no link time -- what they compare is the compute of each placement / microbatch count), then the
# two-process DDP and pipeline paths over gloo on the same GPU (bench.py under torch.distributed.run).
set -o pipefail
cd "$(dirname "$0")/.." && export TMPDIR=/tmp && mkdir -p gpurun_out/mp
O=gpurun_out/mp
run() {  # tag, bench args...
  local tag=$1; shift
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 "$@" > $O/$tag.log 2>&1 || { echo "$tag failed"; tail -3 $O/$tag.log; exit 1; }
  echo "$tag $(tail -1 $O/$tag.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"].get("mp_cut"))')"
}
run single
run ref_m2 --parallelism mp --stages 2 --mp-cut reference --microbatches 2
run ref_m8 --parallelism mp --stages 2 --mp-cut reference --microbatches 8
run plan_v --parallelism mp --stages 2
run xl_single --model unet-xl --img 1024 --batch 16
run xl_plan_v --model unet-xl --img 1024 --batch 16 --parallelism mp --stages 8
export DPA_SAME_DEVICE=1 DPA_DIST_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29521 bench.py --gpus 2 --steps 4 --warmup 2 --batch 32 > $O/ddp2.log 2>&1 || { echo "ddp2 failed"; tail -5 $O/ddp2.log; exit 1; }
echo "ddp2 (gloo, one GPU) $(grep '"metric"' $O/ddp2.log | cut -c80-160)"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29522 bench.py --gpus 2 --steps 4 --warmup 2 --batch 16 --img 256 --parallelism mp > $O/mp2.log 2>&1 || { echo "mp2 failed"; tail -5 $O/mp2.log; exit 1; }
echo "mp2 (gloo, one GPU) $(grep '"metric"' $O/mp2.log | cut -c80-160)"
