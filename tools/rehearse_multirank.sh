# Multi-rank rehearsal on a one-GPU box: 2 ranks share cuda:0 over gloo (RCCL refuses two ranks on one
# device). gloo stages CUDA tensors through host memory, so these numbers say nothing about xGMI; the
# point is that the DDP and GPipe code paths run end to end with the HIP engine.
export DPA_SAME_DEVICE=1 DPA_DIST_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 4 --warmup 2 --batch 32 > gpurun_out/ddp2_rehearsal.log 2>&1 && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 4 --warmup 2 --batch 16 --img 256 --parallelism mp > gpurun_out/mp2_rehearsal.log 2>&1
rc=$?; grep -h '"metric"' gpurun_out/ddp2_rehearsal.log gpurun_out/mp2_rehearsal.log; tail -3 gpurun_out/mp2_rehearsal.log; exit $rc
