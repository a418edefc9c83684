"""Configuration + CLI.

The eight reference flags are kept verbatim (reference ``train.py:15-26``):
``-t/--train-method`` ``-v/--validation`` ``-l/--load`` ``-e/--epochs`` ``--lr/--learning-rate``
``-b/--batch-size`` ``-c/--checkpoint`` ``-s/--seed``.  Additions (SURVEY §5 "Config / flag
system"): image size, dtype, synthetic data, data dirs, backend (hip|torch), model preset,
pipeline stages/microbatches, all-reduce bucket size, global-Dice option, step limits.

``-t`` accepts ``singleGPU | DP | DDP | MP`` like the reference; an unknown value is an error
(the reference silently did nothing).
"""
from __future__ import annotations

import argparse
import os
from dataclasses import dataclass, field, asdict
from typing import Optional, Tuple

METHODS = ("singleGPU", "DP", "DDP", "MP")


@dataclass
class TrainConfig:
    train_method: str = "singleGPU"
    val: float = 10.0
    load: Optional[str] = None
    epochs: int = 10
    lr: float = 1e-4
    batch_size: int = 4
    checkpoint: Optional[str] = None
    seed: int = 42
    # --- additions ---
    img_size: Tuple[int, int] = (640, 960)          # (H, W); reference newsize=[960, 640] (W, H)
    dtype: str = "bf16"                              # compute dtype: bf16 | fp32
    backend: str = "auto"                            # hip | torch | auto
    model: str = "unet"                              # preset name (models.unet.PRESETS)
    synthetic: bool = False
    synthetic_len: int = 5088                        # Carvana's size (train_hq: 5,088 images)
    device_data: bool = True                         # synthetic data rendered once into HBM (no DataLoader/H2D)
    data_dir: str = "./data"
    out_dir: str = "."
    device: Optional[str] = None
    stages: int = 2                                  # pipeline stages for -t MP
    microbatches: int = 0                            # 0: the measured plan's count, else 2 (reference split_size=B/2)
    mp_cut: str = "auto"                             # MP placement: reference | balanced | v | time | auto (mp_plan)
    mp_replicas: int = 1                             # MP: R pipelines of world/R stages, data-parallel across them
    bucket_mb: float = 8.0                           # DDP/DP all-reduce bucket size (MiB of fp32 grads)
    grad_comm_dtype: str = "fp32"                    # DDP gradient all-reduce wire dtype: fp32 | bf16
    comm_overlap: bool = True                        # DDP/DP: launch gradient buckets during the backward
                                                     # (False: all buckets after it, no CU sharing with RCCL)
    global_dice: bool = False                        # DDP: Dice over the global batch (all-reduced sums)
    loss_scale_by_batch: bool = True                 # reference multiplies loss by batch size (A11)
    max_steps: int = 0                               # stop after N optimizer steps (0 = full epochs)
    num_workers: int = 0
    log_every: int = 10
    weight_decay: float = 1e-8
    patience: int = 2
    save_every_epoch: bool = True
    resume: bool = False
    profile: bool = False
    trace_ranges: bool = False                      # roctx ranges per block / bucket / stage op
    cuda_graph: bool = False                         # singleGPU: replay the whole step from a HIP graph
    debug_sync: bool = False                         # synchronise after every kernel / stage op
    watchdog: float = 0.0                            # abort if no step completes for N seconds (0 = off)
    comm_timeout: float = 1800.0                     # process-group (RCCL/gloo) collective timeout, seconds
    nan_policy: str = "raise"                        # non-finite loss: raise | warn | ignore
    progress: Optional[bool] = None                  # tqdm bars (reference); None = only on a terminal

    def to_dict(self):
        return asdict(self)


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="Train UNet on images and target masks (MI355X-native)")
    p.add_argument("--train-method", "-t", type=str, default="singleGPU", help="singleGPU | DP | DDP | MP")
    p.add_argument("--validation", "-v", dest="val", type=float, default=10.0,
                   help="Percentage of data used as validation")
    p.add_argument("--load", "-l", type=str, default=None,
                   help="Load model from a .pth file path (the reference parsed but ignored this)")
    p.add_argument("--epochs", "-e", type=int, default=10, help="Number of epochs")
    p.add_argument("--learning-rate", "--lr", type=float, default=1e-4, help="Learning rate", dest="lr")
    p.add_argument("--batch-size", "-b", type=int, default=4, help="Batch size (per process for DDP)")
    p.add_argument("--checkpoint", "-c", type=str, default=None,
                   help="Name (without .pth) of a checkpoint under checkpoints/ to load")
    p.add_argument("--seed", "-s", type=int, default=42, help="Set seed for reproducibility")
    # additions
    p.add_argument("--img-size", type=int, nargs="+", default=[640, 960], help="H [W] of the training images")
    p.add_argument("--dtype", choices=["bf16", "fp32"], default="bf16")
    p.add_argument("--backend", choices=["auto", "hip", "torch"], default="auto",
                   help="hip = hand-written MI355X kernels; torch = stock PyTorch ops")
    p.add_argument("--model", type=str, default="unet", help="model preset: unet | unet-xl | unet-bn64 | unet-bn | unet-bilinear | unet-bn-bilinear | unet-tiny | unet-tiny-bn")
    p.add_argument("--synthetic", action="store_true", help="use synthetic images/masks instead of data/")
    p.add_argument("--synthetic-len", type=int, default=5088,
                   help="synthetic dataset size (default: Carvana's 5,088 images)")
    p.add_argument("--host-data", dest="device_data", action="store_false",
                   help="synthetic data through the CPU Dataset/DataLoader + H2D path instead of HBM-resident")
    p.add_argument("--data-dir", type=str, default="./data")
    p.add_argument("--out-dir", type=str, default=".")
    p.add_argument("--device", type=str, default=None)
    p.add_argument("--stages", type=int, default=2)
    p.add_argument("--microbatches", type=int, default=0,
                   help="MP microbatches (0: the pipeline plan's count; else 2 for the reference cut, 8 otherwise)")
    p.add_argument("--mp-cut", choices=["auto", "reference", "balanced", "v", "time", "spatial"], default="auto",
                   help="MP stage placement: reference = encoder+mid | decoder+head (2 stages; all skips cross "
                        "the cut); balanced = FLOP-balanced contiguous blocks; v = mirrored, skip-local (stage s "
                        "owns encoder level s and decoder level s); time = the measured-time plan in "
                        "parallel/plans.json; auto = time when planned, else v")
    p.add_argument("--mp-replicas", type=int, default=1,
                   help="-t MP over N ranks: R pipelines of N/R stages each (ranks r*N/R .. (r+1)*N/R - 1), every "
                        "pipeline on its own data shard, stage gradients averaged across the R pipelines")
    p.add_argument("--bucket-mb", type=float, default=8.0)
    p.add_argument("--grad-comm-dtype", choices=["fp32", "bf16"], default="fp32",
                   help="DDP: all-reduce gradient buckets in bf16 (half the bytes) instead of fp32")
    p.add_argument("--no-comm-overlap", dest="comm_overlap", action="store_false",
                   help="DDP/DP: all-reduce the gradient buckets after the backward instead of during it "
                        "(RCCL kernels then never share CUs with the backward's kernels)")
    p.add_argument("--global-dice", action="store_true")
    p.add_argument("--no-batch-loss-scale", dest="loss_scale_by_batch", action="store_false")
    p.add_argument("--max-steps", type=int, default=0)
    p.add_argument("--num-workers", type=int, default=0)
    p.add_argument("--log-every", type=int, default=10)
    p.add_argument("--resume", action="store_true", help="resume from checkpoints/<method>_last.pt")
    p.add_argument("--profile", action="store_true", help="torch.profiler trace of a few steps")
    p.add_argument("--trace-ranges", action="store_true",
                   help="roctx ranges around blocks, pipeline transfers and all-reduce buckets (rocprofv3 --marker-trace)")
    p.add_argument("--cuda-graph", action="store_true",
                   help="capture the training step in a HIP graph (singleGPU: the whole step; -t DP: each "
                        "replica's forward and backward)")
    p.add_argument("--debug-sync", action="store_true",
                   help="synchronise after every HIP kernel and pipeline stage op (race / fault triage)")
    p.add_argument("--watchdog", type=float, default=0.0,
                   help="abort (exit 124, for torchrun --max-restarts + --resume) after N s without a step")
    p.add_argument("--comm-timeout", type=float, default=1800.0, help="collective timeout in seconds")
    p.add_argument("--nan-policy", choices=["raise", "warn", "ignore"], default="raise")
    p.add_argument("--progress", dest="progress", action="store_true", default=None,
                   help="tqdm progress bars for training images and validation batches (default: on a terminal)")
    p.add_argument("--no-progress", dest="progress", action="store_false")
    return p


def parse_args(argv=None) -> TrainConfig:
    a = build_parser().parse_args(argv)
    if a.train_method not in METHODS:
        raise SystemExit(f"unknown --train-method {a.train_method!r}; choose from {METHODS}")
    size = a.img_size
    img_size = (size[0], size[0]) if len(size) == 1 else (size[0], size[1])
    cfg = TrainConfig(
        train_method=a.train_method, val=a.val, load=a.load, epochs=a.epochs, lr=a.lr,
        batch_size=a.batch_size, checkpoint=a.checkpoint, seed=a.seed, img_size=img_size,
        dtype=a.dtype, backend=a.backend, model=a.model, synthetic=a.synthetic,
        synthetic_len=a.synthetic_len, device_data=a.device_data, data_dir=a.data_dir, out_dir=a.out_dir, device=a.device,
        stages=a.stages, microbatches=a.microbatches, mp_cut=a.mp_cut, mp_replicas=a.mp_replicas, bucket_mb=a.bucket_mb,
        grad_comm_dtype=a.grad_comm_dtype,
        comm_overlap=a.comm_overlap, global_dice=a.global_dice,
        loss_scale_by_batch=a.loss_scale_by_batch, max_steps=a.max_steps, num_workers=a.num_workers,
        log_every=a.log_every, resume=a.resume, profile=a.profile, trace_ranges=a.trace_ranges, cuda_graph=a.cuda_graph,
        debug_sync=a.debug_sync, watchdog=a.watchdog, comm_timeout=a.comm_timeout, nan_policy=a.nan_policy, progress=a.progress)
    return cfg


def mp_cut_mode(cfg: "TrainConfig", stages: int) -> str:
    return mp_plan(cfg, stages).mode


@dataclass
class MPPlan:
    """How an MP run is laid out: the stage placement, microbatch count and per-stage op order."""
    mode: str                           # reference | balanced | v | time
    placement: object                   # parallel.placement.Placement
    microbatches: int
    orders: Optional[list] = None       # per-stage static op order (None: derived from FLOP costs)
    policy: str = "feed"
    info: dict = field(default_factory=dict)


def mp_plan(cfg: "TrainConfig", stages: int) -> MPPlan:
    """Placement, microbatch count and op order of an MP run (``--mp-cut``):

    * ``reference``: the reference cut, encoder+mid | decoder+head (unet_model.py:14-20; 2 stages):
      all four skips cross the cut, 31 MiB per image at 512^2 bf16 -- link-bound on xGMI;
    * ``balanced``: FLOP-balanced contiguous block ranges;
    * ``v``: the skip-local mirrored placement (stage s owns encoder level(s) s and the same decoder
      level(s); parallel/placement.py), FLOP-balanced;
    * ``time``: the placement, microbatch count and op order tools/pipeline_plan.py chose from MEASURED
      per-block times with the link-queueing schedule model (parallel/plans.json, keyed by model,
      image, stages and global batch);
    * ``spatial``: the top level(s) split by image ROWS over all stages and the inner chain pipelined
      (parallel/spatial.py; plans.json's row-split plan when it has one, else a FLOP-balanced one): for deep
      pipelines at high resolution, where whole full-resolution tensors cost more link time than compute;
    * ``auto`` (default): ``time`` when plans.json has the configuration, else ``v``.

    Microbatches: ``--microbatches`` when given, else the plan's, else 2 for the reference cut (the
    reference's split_size = B/2) and 8 otherwise (reduced to a divisor of the batch)."""
    import math
    from .models.blocks import n_blocks, partition
    from .models.unet import build_model
    from .parallel.placement import Placement, v_partition
    from .parallel.schedule import load_plan
    mcfg = build_model(cfg.model).cfg
    h, w = cfg.img_size
    mode = cfg.mp_cut
    plan = None
    if mode in ("auto", "time", "spatial"):
        plan = load_plan(cfg.model, h, w, stages, cfg.batch_size, depth=mcfg.depth)
        if mode == "spatial" and plan is not None and not plan.get("spatial"):
            plan = None
        if plan is not None:
            mode = "time"
        elif mode != "spatial":
            mode = "v" if stages > 1 else "balanced"
    if stages == 1:
        pl = Placement.contiguous([0, n_blocks(mcfg.depth)])
    elif mode == "time":
        pl = plan["placement"]
    elif mode == "reference":
        pl = Placement.contiguous(partition(mcfg, stages, h, w, mode="reference"))
    elif mode == "balanced":
        pl = Placement.contiguous(partition(mcfg, stages, h, w, mode="balanced"))
    elif mode == "v":
        pl = v_partition(mcfg, stages, h, w)
    elif mode == "spatial":
        from .parallel.spatial import default_plan
        pl = default_plan(mcfg, stages, h, w)
    else:
        raise ValueError(f"unknown --mp-cut {mode!r}")
    M = cfg.microbatches or (plan["microbatches"] if plan else (2 if mode == "reference" else 8))
    if plan is not None and plan.get("spatial"):
        mode = "spatial"
    if not cfg.microbatches and cfg.batch_size % M:
        M = math.gcd(M, cfg.batch_size)
    orders = plan.get("orders") if plan is not None and M == plan["microbatches"] else None
    info = {k: plan[k] for k in ("predicted_img_s", "predicted_efficiency", "rehearsal_img_s") if plan and k in plan}
    return MPPlan(mode, pl, M, orders, (plan or {}).get("policy", "feed"), info)


def dist_env():
    """(rank, local_rank, world_size) from torchrun's environment (torch/distributed/run.py:191-232)."""
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    return rank, local, world
