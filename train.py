#!/usr/bin/env python3
"""CLI entry point, flag-compatible with the reference ``train.py`` (train.py:15-64).

    python3 train.py                                   # -t singleGPU (default)
    python3 train.py -t DP                             # single process, all local GPUs
    torchrun --standalone --nnodes=1 --nproc_per_node=2 train.py -t DDP -b 2
    python3 train.py -t MP                             # single-process 2-stage pipeline (reference form)
    torchrun --nproc_per_node=2 train.py -t MP --microbatches 8   # multi-process GPipe over RCCL

Additions: --synthetic, --img-size, --backend {hip,torch}, --model, --stages, --microbatches,
--bucket-mb, --global-dice, --max-steps, --resume ... (see distributedpytorch_amd/config.py).
"""
import warnings

warnings.filterwarnings("ignore")  # reference train.py:12

from distributedpytorch_amd.config import parse_args  # noqa: E402
from distributedpytorch_amd.trainer import train  # noqa: E402


def main(argv=None):
    cfg = parse_args(argv)
    out = train(cfg)
    import torch.distributed as dist
    if dist.is_initialized():
        dist.destroy_process_group()
    return out


if __name__ == "__main__":
    main()
