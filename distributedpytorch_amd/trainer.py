"""One training loop parametrised by strategy (the reference copy-pasted it three times:
``utils/train_utils.py:22-92`` fit, ``:95-167`` fit_DP, ``:170-248`` fit_DDP).

Per step (reference hot loop ``:59-79``): H2D (prefetched on a side stream), forward to the loss
partial sums, ``(batch_size * loss).backward()`` (A11 kept, switchable), gradient all-reduce
(strategy specific, overlapped with backward), one fused Adam launch, metrics every ``log_every``
steps without a per-step host sync (A17).  Per epoch: sharded evaluation (loss + Dice),
``ReduceLROnPlateau`` stepped identically on all ranks (A5), a checkpoint of the full training
state.  At the end: ``checkpoints/<method>.pth`` (reference keys; ``module.`` prefix for DP/DDP as
the reference wrote them) and ``loss/<method>/{train,val}_loss.pkl``.
"""
from __future__ import annotations

import datetime
import logging
import os
import time
from typing import Optional

import numpy as np
import torch
import torch.distributed as dist

from .compute import loss_from_partials, make_compute, resolve_backend
from .config import TrainConfig, dist_env, mp_plan
from .data import CarvanaDataset, SyntheticSegmentation, build_loaders, split_dataset
from .data.device import DeviceLoader, DeviceSyntheticSegmentation, device_loaders
from .data.loaders import DeviceBatcher
from .loss import dice_score
from .models.unet import build_model
from .optim import FlatParameterSpace, FusedAdam, make_plateau, plateau_step
from .parallel.ddp import BucketedAllReduce, broadcast_parameters, sync_buffers
from .parallel.dp import ReplicatedDataParallel
from .parallel.pipeline import GPipeDist, GPipeLocal, placement_buffer_names
from .utils import LossCurves, MetricsLogger, load_model_state, save_model, set_seed
from .utils.checkpoint import load_training_state, save_training_state
from .utils.resilience import ShutdownGuard, StepWatchdog, check_finite, comm_env_defaults

log = logging.getLogger("dpa")


# ============================================================================ strategies
class Strategy:
    name = "base"
    module_prefix = False

    def __init__(self, cfg: TrainConfig):
        self.cfg = cfg
        self.rank, self.local_rank, self.world = 0, 0, 1
        self.is_main = True
        self.device = torch.device("cpu")

    # must set self.model, self.optimizer
    def train_step(self, images, targets) -> Optional[torch.Tensor]:
        raise NotImplementedError

    def eval_batch(self, images, targets):
        """-> (loss, dice) device tensors or None on ranks without outputs."""
        raise NotImplementedError

    def state_dict(self):
        return self.model.state_dict()

    def reduce_eval(self, vals: torch.Tensor) -> torch.Tensor:
        return vals

    def barrier(self):
        pass

    def lr_scale(self) -> float:
        return 1.0

    def set_train(self, mode: bool):
        """train/eval mode (BatchNorm variants: batch vs running statistics)."""
        self.model.train(mode)

    def before_eval(self):
        pass

    # ---- checkpoint / resume hooks
    def spaces(self):
        opt = getattr(self, "optimizer", None)
        return list(getattr(opt, "spaces", []))

    def after_load(self):
        """Parameters were overwritten in place (resume / load): kernels re-pack their weights."""
        for sp in self.spaces():
            sp.touch()

    def optimizer_state_dict(self):
        """Optimizer state to checkpoint (collective for strategies whose state is sharded)."""
        return self.optimizer.state_dict()

    def load_optimizer_state_dict(self, sd):
        self.optimizer.load_state_dict(sd)


def _loss_scale(cfg, batch):
    return float(batch) if cfg.loss_scale_by_batch else 1.0


def _backward(loss, scale: float):
    """``(loss * scale).backward()`` (reference utils/train_utils.py:69, A11); on a GPU with the HIP loss op
    the scale seeds the backward instead of costing two elementwise launches."""
    if loss.is_cuda and loss.grad_fn is not None and type(loss.grad_fn).__name__.startswith("_LossFromPartials"):
        from .ops.kernels import backward_scaled
        backward_scaled(loss, scale)
    else:
        (loss * scale).backward()


class SingleDevice(Strategy):
    name = "singleGPU"

    def __init__(self, cfg, model, device):
        super().__init__(cfg)
        self.device = torch.device(device)
        self.model = model.to(self.device)
        self.space = FlatParameterSpace(self.model, device=self.device)
        self.compute = make_compute(self.model, cfg.backend, cfg.dtype)
        self.optimizer = FusedAdam(self.space, lr=cfg.lr * self.lr_scale(), weight_decay=cfg.weight_decay)

    def forward_loss(self, images, targets):
        S = self.compute.forward_partials(images, targets)
        return loss_from_partials(S, targets.numel())

    def train_step(self, images, targets):
        self.optimizer.zero_grad()
        loss = self.forward_loss(images, targets)
        _backward(loss, _loss_scale(self.cfg, images.shape[0]))
        self.optimizer.step()
        return loss.detach()

    @torch.no_grad()
    def eval_batch(self, images, targets):
        p = self.compute.probs(images)
        S = _partials(p, targets)
        return loss_from_partials(S, targets.numel()), dice_score(p, targets)


def _partials(p, t):
    from .compute import loss_partials_from_probs
    return loss_partials_from_probs(p, t)


class DDPStrategy(SingleDevice):
    name = "DDP"
    module_prefix = True

    def __init__(self, cfg, model, device):
        self.rank, self.local_rank, self.world = dist.get_rank(), dist_env()[1], dist.get_world_size()
        super().__init__(cfg, model, device)
        self.rank, self.local_rank, self.world = dist.get_rank(), dist_env()[1], dist.get_world_size()
        self.is_main = self.rank == 0
        broadcast_parameters(self.space, src=0)
        scale = float(self.world) if cfg.global_dice else 1.0
        self.reducer = BucketedAllReduce(self.space, bucket_mb=cfg.bucket_mb, scale=scale,
                                         comm_dtype=cfg.grad_comm_dtype,
                                         overlap=cfg.comm_overlap).register_hooks()

    def lr_scale(self):
        # reference: Adam(lr * world_size) (utils/train_utils.py:199) - with the real world size (A6)
        return float(dist.get_world_size())

    def forward_loss(self, images, targets):
        S = self.compute.forward_partials(images, targets)
        n = targets.numel()
        if self.cfg.global_dice:
            S = _all_reduce_sum_autograd(S)
            n = n * self.world
        return loss_from_partials(S, n)

    def train_step(self, images, targets):
        self.optimizer.zero_grad()
        loss = self.forward_loss(images, targets)
        _backward(loss, _loss_scale(self.cfg, images.shape[0]))
        self.reducer.finish()
        self.optimizer.step()
        return loss.detach()

    def reduce_eval(self, vals):
        dist.all_reduce(vals, op=dist.ReduceOp.SUM)
        return vals

    def before_eval(self):
        # torch DDP's broadcast_buffers: every rank evaluates with rank 0's BN running statistics
        if any(True for _ in self.model.buffers()):
            sync_buffers(self.model, src=0)

    def barrier(self):
        dist.barrier()


class _AllReduceSum(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        y = x.clone()
        dist.all_reduce(y, op=dist.ReduceOp.SUM)
        return y

    @staticmethod
    def backward(ctx, g):
        # every rank holds the same global loss; d(global)/d(local) = 1 -> pass the grad through
        return g


def _all_reduce_sum_autograd(x):
    return _AllReduceSum.apply(x)


class DPStrategy(Strategy):
    name = "DP"
    module_prefix = True

    def __init__(self, cfg, model, devices):
        super().__init__(cfg)
        self.dp = ReplicatedDataParallel(model, devices, cfg.backend, cfg.dtype, bucket_mb=cfg.bucket_mb,
                                         overlap=cfg.comm_overlap)
        self.reducer = self.dp.reducer
        self.device = self.dp.devices[0]
        self.model = self.dp.module
        self.optimizer = FusedAdam(self.dp.spaces, lr=cfg.lr, weight_decay=cfg.weight_decay)

    def set_train(self, mode: bool):
        for r in self.dp.replicas:
            r.train(mode)

    def before_eval(self):
        # torch.nn.DataParallel re-broadcasts device 0's buffers every forward: every replica
        # evaluates with replica 0's BatchNorm running statistics
        self.dp.sync_buffers()

    def after_load(self):
        # a resume loads replica 0 only; replicate its parameters and buffers to the others
        self.dp.sync_from_replica0()

    def state_dict(self):
        self.dp.sync_buffers()
        return self.model.state_dict()

    def train_step(self, images, targets):
        self.optimizer.zero_grad()
        loss = self.dp.forward_loss(images, targets)
        _backward(loss, _loss_scale(self.cfg, images.shape[0]))
        self.dp.all_reduce_grads()
        self.optimizer.step()
        return loss.detach()

    @torch.no_grad()
    def eval_batch(self, images, targets):
        p = self.dp.probs(images)
        t = targets.to(p.device)
        return loss_from_partials(_partials(p, t), t.numel()), dice_score(p, t)


class PipelineLocalStrategy(Strategy):
    name = "MP"

    def __init__(self, cfg, model, devices):
        super().__init__(cfg)
        H, W = cfg.img_size
        self.plan = mp_plan(cfg, len(devices))
        pl = self.plan.placement
        if self.plan.mode == "spatial":
            # row-split plans need one process per stage (parallel/spatial_pipe.py): the single-process form
            # runs the FLOP-balanced skip-local V placement instead
            from .parallel.placement import v_partition
            log.warning("MP: the row-split plan needs torchrun (one process per stage); running the V placement")
            pl = v_partition(model.cfg, len(devices), H, W)
        self.pipe = GPipeLocal(model, devices, self.plan.microbatches, cfg.backend, cfg.dtype, img_hw=(H, W),
                               placement=pl)
        self.model = model
        self.device = self.pipe.devices[0]
        self.optimizer = FusedAdam(self.pipe.spaces, lr=cfg.lr, weight_decay=cfg.weight_decay)

    def train_step(self, images, targets):
        self.optimizer.zero_grad()
        loss = self.pipe.forward_loss(images, targets)
        _backward(loss, _loss_scale(self.cfg, images.shape[0]))
        self.optimizer.step()
        return loss.detach()

    @torch.no_grad()
    def eval_batch(self, images, targets):
        p = self.pipe.probs(images)
        t = targets.to(p.device)
        return loss_from_partials(_partials(p, t), t.numel()), dice_score(p, t)


class PipelineDistStrategy(Strategy):
    name = "MP"

    def __init__(self, cfg, model, device):
        super().__init__(cfg)
        self.rank, self.local_rank, self.world = dist.get_rank(), dist_env()[1], dist.get_world_size()
        self.device = torch.device(device)
        self.model = model.to(self.device)
        H, W = cfg.img_size
        # R pipelines of S stages (--mp-replicas): pipeline r = ranks r*S .. r*S + S - 1, stage s of every
        # pipeline in one data-parallel group; R = 1 is the plain pipeline over the whole job
        R = max(1, int(cfg.mp_replicas or 1))
        if self.world % R:
            raise ValueError(f"--mp-replicas {R} does not divide the {self.world} ranks")
        S = self.world // R
        self.replicas, self.stages = R, S
        self.replica, self.stage = divmod(self.rank, S)
        pipe_group = self.dp_group = None
        if R > 1:   # every rank creates every group, in the same order
            pgs = [dist.new_group(list(range(r * S, (r + 1) * S))) for r in range(R)]
            dgs = [dist.new_group([s + k * S for k in range(R)]) for s in range(S)]
            pipe_group, self.dp_group = pgs[self.replica], dgs[self.stage]
        self.plan = mp_plan(cfg, S)
        self.spatial = self.plan.mode == "spatial"
        if self.spatial:
            # top level(s) split by image rows over every stage (parallel/spatial_pipe.py): every rank reads
            # its rows of the same batch
            from .parallel.spatial_pipe import SpatialGPipe
            self.pipe = SpatialGPipe(self.model, self.plan.placement, self.plan.microbatches, cfg.backend, cfg.dtype,
                                     group=pipe_group, img_hw=(H, W))
        else:
            self.pipe = GPipeDist(self.model, self.plan.microbatches, cfg.backend, cfg.dtype, img_hw=(H, W),
                                  placement=self.plan.placement, policy=self.plan.policy, orders=self.plan.orders,
                                  group=pipe_group)
        # the head stage owns the loss (pipeline 0's logs); rank 0 saves
        self.is_main = self.pipe.is_last and self.replica == 0
        self.optimizer = FusedAdam(self.pipe.space, lr=cfg.lr, weight_decay=cfg.weight_decay)
        self.reducer = None
        if R > 1:   # every pipeline starts from pipeline 0's parameters (stage s: global rank s)
            dist.broadcast(self.pipe.space.data, src=self.stage, group=self.dp_group)
            self.pipe.space.touch()
            self.sync_stage_buffers()
            # data parallel across the pipelines: each stage's flat gradient averaged over its R copies in
            # buckets launched as soon as their gradients are final -- during the stage's last microbatch's
            # backward (the pipeline drain), not after it.  The HIP engine announces a layer once its last
            # microbatch's contribution is issued (``early_ready``: the merged weight-gradient launch + the
            # bucket's all-reduce ordered on its side stream); the torch backend's autograd hooks fire once
            # per microbatch, so a parameter is final at its M-th.
            blocks = self.pipe.blocks
            per_param = 1
            if hasattr(blocks, "early_ready"):
                blocks.early_ready = True
            else:
                per_param = self.plan.microbatches
            # (row-split pipelines all-reduce their split levels' gradients inside the step: the replicas'
            # all-reduce follows it as one collective instead of racing it bucket by bucket)
            self.reducer = BucketedAllReduce(self.pipe.space, bucket_mb=cfg.bucket_mb, group=self.dp_group,
                                             comm_dtype=cfg.grad_comm_dtype,
                                             overlap=cfg.comm_overlap and not self.spatial,
                                             per_param=per_param).register_hooks()

    def sync_stage_buffers(self):
        """Pipeline 0's stage buffers (BatchNorm running statistics) to every replica of the stage: torch
        DDP's ``broadcast_buffers`` across the pipelines, so validation and the checkpoint (pipeline 0's)
        describe one model."""
        if self.replicas <= 1 or self.spatial:        # row-split plans exclude BatchNorm models
            return
        bufs = dict(self.model.named_buffers())
        for n in placement_buffer_names(self.model, self.pipe.pl, self.stage):
            b = bufs[n]
            if self.pipe._host_staged:
                h = b.cpu()
                dist.broadcast(h, src=self.stage, group=self.dp_group)
                b.copy_(h)
            else:
                dist.broadcast(b, src=self.stage, group=self.dp_group)

    def before_eval(self):
        self.sync_stage_buffers()

    def train_step(self, images, targets):
        self.optimizer.zero_grad()
        B = images.shape[0]
        loss = self.pipe.train_step(images, targets, B, self.cfg.img_size,
                                    loss_scale=_loss_scale(self.cfg, B))
        if self.reducer is not None:
            # DDP semantics: the mean over the pipelines of each pipeline's gradient
            self.reducer.finish()
        self.optimizer.step()
        return None if loss is None else loss.detach()

    @torch.no_grad()
    def eval_batch(self, images, targets):
        p = self.pipe.eval_probs(images, images.shape[0], self.cfg.img_size)
        if p is None or (self.spatial and not self.pipe.is_last):
            return None             # (row-split: every stage holds the gathered probabilities; stage 0 counts)
        return loss_from_partials(_partials(p, targets), targets.numel()), dice_score(p, targets)

    def state_dict(self):
        self.sync_stage_buffers()
        if self.replica != 0:
            return None        # replicas hold pipeline 0's state; only pipeline 0 gathers (rank 0 saves)
        return self.pipe.gather_state_dict()

    def optimizer_state_dict(self):
        """Each stage owns the Adam state of its own parameters: gather all of them to rank 0 as
        ``{"stages": [state of stage 0, ..., state of stage S-1]}``."""
        mine = self.optimizer.state_dict()
        out = [None] * self.world if self.rank == 0 else None
        dist.gather_object(mine, out, dst=0)
        # pipelines hold identical optimizer states (same averaged gradients): pipeline 0's are kept
        return {"stages": out[:self.stages]} if self.rank == 0 else None

    def load_optimizer_state_dict(self, sd):
        if "stages" in sd and len(sd["stages"]) != self.stages:
            raise ValueError(f"checkpoint holds optimizer state for {len(sd['stages'])} pipeline stages, "
                             f"this run has {self.stages}")
        self.optimizer.load_state_dict(sd["stages"][self.stage] if "stages" in sd else sd)

    def barrier(self):
        dist.barrier()


# ============================================================================ driver
def _devices_for(cfg, n_needed=None):
    if torch.cuda.is_available():
        n = torch.cuda.device_count()
        return [torch.device(f"cuda:{i}") for i in range(n if n_needed is None else n_needed)]
    return [torch.device("cpu")] * (n_needed or 2)


def build_strategy(cfg: TrainConfig, model) -> Strategy:
    m = cfg.train_method
    rank, local, world = dist_env()
    if m in ("DDP",) or (m == "MP" and world > 1):
        # DPA_SAME_DEVICE=1 maps every rank to cuda:0 (rehearsal of the multi-rank path on one GPU;
        # use with DPA_DIST_BACKEND=gloo, RCCL refuses two ranks on one device)
        if os.environ.get("DPA_SAME_DEVICE", "0") == "1":
            local = 0
        if not dist.is_initialized():
            backend = os.environ.get("DPA_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
            if torch.cuda.is_available():
                torch.cuda.set_device(local)   # A15: bind each rank to its own GPU
            comm_env_defaults()
            dist.init_process_group(backend=backend, init_method="env://",
                                    timeout=datetime.timedelta(seconds=cfg.comm_timeout))
        device = torch.device(f"cuda:{local}") if torch.cuda.is_available() else torch.device("cpu")
        return DDPStrategy(cfg, model, device) if m == "DDP" else PipelineDistStrategy(cfg, model, device)
    if m == "singleGPU":
        dev = cfg.device or ("cuda:0" if torch.cuda.is_available() else "cpu")
        return SingleDevice(cfg, model, dev)
    if m == "DP":
        devs = _devices_for(cfg)
        reps = int(os.environ.get("DPA_DP_REPLICAS", "0") or 0)
        if reps > 0:                  # rehearsal: replicas round-robin over the visible devices
            devs = [devs[i % len(devs)] for i in range(reps)]
        if torch.cuda.is_available():
            assert len(devs) >= 2, f"Requires at least 2 GPUs to run, but got {len(devs)}"
        return DPStrategy(cfg, model, devs)
    if m == "MP":
        devs = _devices_for(cfg, cfg.stages)
        if torch.cuda.is_available():
            assert torch.cuda.device_count() >= cfg.stages, "not enough GPUs for the pipeline stages"
        return PipelineLocalStrategy(cfg, model, devs)
    raise ValueError(m)


def build_datasets(cfg: TrainConfig, device=None):
    H, W = cfg.img_size
    if cfg.synthetic and device is not None and cfg.device_data and torch.device(device).type == "cuda":
        ds = DeviceSyntheticSegmentation(cfg.synthetic_len, (H, W), 3, seed=cfg.seed, device=device)
        log.info(f"synthetic dataset resident on {device}: {len(ds)} images, {ds.nbytes / 2 ** 30:.2f} GiB")
    elif cfg.synthetic:
        ds = SyntheticSegmentation(cfg.synthetic_len, (H, W), 3, seed=cfg.seed)
    else:
        root = cfg.data_dir
        ds = CarvanaDataset(os.path.join(root, "train_hq"), os.path.join(root, "train_masks"), newsize=(W, H))
    return split_dataset(ds, cfg.val, seed=0)


def _base_dataset(ds):
    while isinstance(ds, torch.utils.data.Subset):
        ds = ds.dataset
    return ds


def _batches(loader, device):
    """(images, targets) on the device: HBM-resident loaders yield them directly; host loaders go
    through the prefetching H2D batcher."""
    return loader if isinstance(loader, DeviceLoader) else DeviceBatcher(loader, device)


def _setup_logging(cfg, rank):
    os.makedirs(os.path.join(cfg.out_dir, "logs"), exist_ok=True)
    # one log file per rank (the reference had all DDP ranks append to one file)
    suffix = "" if rank == 0 else f".rank{rank}"
    path = os.path.join(cfg.out_dir, "logs", f"{cfg.train_method}{suffix}.log")
    handler = logging.FileHandler(path, mode="a")
    handler.setFormatter(logging.Formatter("%(message)s"))
    log.handlers[:] = [handler]
    log.setLevel(logging.INFO)
    log.propagate = False


def train(cfg: TrainConfig):
    rank, local, world = dist_env()
    if cfg.debug_sync:
        from .ops._lib import set_debug_sync
        set_debug_sync(True)
    if cfg.trace_ranges or cfg.profile:
        from .utils.tracing import enable_ranges
        enable_ranges(True)
    set_seed(cfg.seed)
    _setup_logging(cfg, rank)
    log.info("UNet for Carvana Image Masking (Segmentation)")
    log.info(f"config: {cfg.to_dict()}")
    from .ops.config import removed_in_env
    for k, why in removed_in_env().items():
        log.warning(f"{k} is set but has no effect: {why}")
    model = build_model(cfg.model)
    if cfg.checkpoint is not None:
        load_model_state(model, os.path.join(cfg.out_dir, "checkpoints", f"{cfg.checkpoint}.pth"))
    if cfg.load:
        load_model_state(model, cfg.load)
    strat = build_strategy(cfg, model)
    backend = resolve_backend(cfg.backend, strat.device, cfg.dtype, model)
    log.info(f"strategy={strat.name} backend={backend}{'-fp32' if backend == 'hip' and cfg.dtype == 'fp32' else ''} "
             f"device={strat.device}")
    if backend == "hip" and cfg.dtype != "fp32":
        from .ops import kernels as _K
        log.info(_K.CFG.describe())        # the run's kernel switches, once (ops/config.py)

    train_set, val_set = build_datasets(cfg, strat.device)
    # data shards: DDP ranks, or the pipelines of a replicated -t MP (every stage of one pipeline reads the
    # same shard; only its first / head stage uses it)
    mp_dist = isinstance(strat, PipelineDistStrategy)
    dp_ranks = world if strat.name == "DDP" else (strat.replicas if mp_dist else 1)
    dp_rank = strat.rank if strat.name == "DDP" else (strat.replica if mp_dist else 0)
    if isinstance(_base_dataset(train_set), DeviceSyntheticSegmentation):
        train_loader, val_loader, sampler = device_loaders(
            train_set, val_set, cfg.batch_size, rank=dp_rank, world_size=dp_ranks, seed=cfg.seed,
            drop_last=strat.name in ("MP",))
    else:
        train_loader, val_loader, sampler = build_loaders(
            train_set, val_set, cfg.batch_size, rank=dp_rank, world_size=dp_ranks, num_workers=cfg.num_workers,
            pin_memory=strat.device.type == "cuda", seed=cfg.seed, drop_last=strat.name in ("MP",))
    scheduler = make_plateau(strat.optimizer, cfg.patience)
    metrics = MetricsLogger(os.path.join(cfg.out_dir, "logs", f"{cfg.train_method}.jsonl"), strat.is_main)
    curves = LossCurves()
    last_path = os.path.join(cfg.out_dir, "checkpoints", f"{cfg.train_method}_last.pt")
    start_epoch, step = 0, 0
    if cfg.resume and os.path.exists(last_path):
        start_epoch, step = load_training_state(last_path, model=strat.model, optimizer=_OptIO(strat),
                                                scheduler=scheduler)
        strat.after_load()
        log.info(f"resumed from {last_path} at epoch {start_epoch} step {step}")

    t_start = time.time()
    pending = []
    prof = _Profiler(cfg, strat) if cfg.profile else None
    guard = ShutdownGuard()
    dog = StepWatchdog(cfg.watchdog) if cfg.watchdog > 0 else None
    graphed = None
    # --cuda-graph: the whole singleGPU step, or every -t DP replica's forward / backward (GraphedDP)
    graph_cls = next((c for c in (GraphedStep, GraphedDP) if c.supported(strat)), None)
    if cfg.cuda_graph and graph_cls is None:
        log.warning(f"--cuda-graph: not supported for {strat.name} on {strat.device}; running eagerly")
    stop_signal = None
    for epoch in range(start_epoch, cfg.epochs):
        if sampler is not None:
            sampler.set_epoch(epoch)  # A7
        n_img, t_ep = 0, time.perf_counter()
        steady = _SteadyMeter(strat.device)
        bar = _progress(cfg, strat, f"Epoch {epoch + 1}/{cfg.epochs}", len(train_loader) * cfg.batch_size, "img")
        for images, targets in _batches(train_loader, strat.device):
            steady.tick(images.shape[0])
            if prof is not None:
                prof.before(step)
            if cfg.cuda_graph and graphed is None and graph_cls is not None:
                graphed = graph_cls(strat, images, targets)
            if graphed is not None and graphed.matches(images, targets):
                loss = graphed(images, targets)
            else:
                loss = strat.train_step(images, targets)
            step += 1
            if dog is not None:
                dog.kick(step)
            if prof is not None:
                prof.after(step)
            n_img += images.shape[0]
            bar.update(images.shape[0])
            if loss is not None:
                pending.append(loss)
            if step % cfg.log_every == 0:
                if pending:
                    vals = torch.stack([p.float().to("cpu") for p in pending]).numpy()
                    if cfg.nan_policy != "ignore":
                        check_finite(vals.tolist(), step, cfg.nan_policy)
                    mean_loss = float(np.mean(vals[-10:]))
                    pending = []
                    curves.add_train(step, time.time() - t_start, mean_loss)
                    red = getattr(strat, "reducer", None)
                    comm_ms = red.exposed_comm_ms() if red is not None else None
                    metrics.log(kind="train", step=step, epoch=epoch, loss=mean_loss,
                                lr=strat.optimizer.param_groups[0]["lr"], exposed_comm_ms=comm_ms)
                    if strat.is_main:
                        log.info(f"step {step} loss {mean_loss:.5f}")
                    bar.set_postfix(loss=f"{mean_loss:.4f}")
                stop_signal = _agree_stop(strat, guard.requested)
                if stop_signal is not None:
                    break
            if cfg.max_steps and step >= cfg.max_steps:
                break
        if stop_signal is not None:
            # SIGTERM/SIGUSR1 (e.g. torchrun tearing the job down): save where we are and leave
            sd_model, sd_opt = strat.state_dict(), strat.optimizer_state_dict()
            if strat.rank == 0 and sd_model is not None:
                save_training_state(last_path, model=_SD(sd_model), optimizer=_SD(sd_opt),
                                    scheduler=scheduler, epoch=epoch, step=step)
            log.warning(f"stopped by signal {stop_signal} at step {step}; state saved to {last_path}")
            break
        if strat.device.type == "cuda":
            torch.cuda.synchronize(strat.device)    # epoch time = work done, not work enqueued
        ep_time = time.perf_counter() - t_ep
        steady_ips = steady.finish()
        bar.close()
        val_loss, val_dice = evaluate(strat, val_loader, cfg)
        curves.add_val(step, time.time() - t_start, val_loss)
        plateau_step(scheduler, val_loss)
        metrics.log(kind="epoch", epoch=epoch, step=step, val_loss=val_loss, val_dice=val_dice,
                    img_per_s=n_img * dp_ranks / max(ep_time, 1e-9),
                    img_per_s_steady=(None if steady_ips is None else steady_ips * dp_ranks),
                    peak_mem_gb=(torch.cuda.max_memory_allocated(strat.device) / 2 ** 30
                                 if strat.device.type == "cuda" else 0.0))
        if strat.is_main:
            log.info(f"epoch {epoch}: val_loss {val_loss:.5f} val_dice {val_dice:.4f}")
            sps = "" if steady_ips is None else f", {steady_ips:.1f} img/s/rank after {steady.skip} warm-up steps"
            print(f"epoch {epoch + 1}/{cfg.epochs} step {step} val_loss {val_loss:.5f} dice {val_dice:.4f} "
                  f"({n_img / max(ep_time, 1e-9):.1f} img/s/rank{sps})", flush=True)
        if cfg.save_every_epoch:
            sd_model, sd_opt = strat.state_dict(), strat.optimizer_state_dict()
            if strat.rank == 0 and sd_model is not None:
                save_training_state(last_path, model=_SD(sd_model), optimizer=_SD(sd_opt),
                                    scheduler=scheduler, epoch=epoch + 1, step=step)
        if cfg.max_steps and step >= cfg.max_steps:
            break
    guard.close()
    if dog is not None:
        dog.close()
    if stop_signal is not None:
        strat.barrier()
        return {"step": step, "paths": {"last": last_path}, "curves": curves, "strategy": strat,
                "stopped_by_signal": stop_signal}

    sd = strat.state_dict()
    paths = {}
    if strat.rank == 0 and sd is not None:
        ck = os.path.join(cfg.out_dir, "checkpoints", f"{cfg.train_method}.pth")
        save_model(_SD(sd), ck, module_prefix=strat.module_prefix)
        paths["checkpoint"] = ck
    if strat.is_main:
        paths["loss"] = curves.save(cfg.out_dir, cfg.train_method)
    strat.barrier()
    return {"step": step, "paths": paths, "curves": curves, "strategy": strat}


def _agree_stop(strat, requested):
    """All ranks stop at the same step boundary if any of them was signalled (a rank leaving alone
    would strand its peers inside the next collective)."""
    flag = 0 if requested is None else int(requested)
    if strat.world > 1 and dist.is_initialized():
        dev = strat.device if dist.get_backend() == "nccl" else torch.device("cpu")
        t = torch.tensor([flag], dtype=torch.int64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        flag = int(t.item())
    return flag or None


class GraphedStep:
    """``--cuda-graph``: the whole singleGPU training step — weight packing, forward, fused loss,
    backward (explicit per-block HIP kernels), Adam — captured once in a HIP graph and replayed
    (one ``hipGraphLaunch`` instead of ~130 kernel launches + the Python autograd walk per step).

    Adam runs in device-state mode (step count / lr / bias corrections in a device block the
    captured kernels update), new LR values are uploaded before a replay, and batches of another
    shape (a short last batch) fall back to the eager step.  Capture needs one eager warm-up step
    (lazy allocations); its effect on parameters and optimizer state is rolled back."""

    @staticmethod
    def supported(strat) -> bool:
        return type(strat) is SingleDevice and strat.device.type == "cuda"

    def __init__(self, strat, images, targets):
        self.strat = strat
        opt, space = strat.optimizer, strat.space
        opt.enable_device_state()
        self.x = images.detach().clone()
        self.t = targets.detach().clone()
        snap = (space.data.clone(), [m.clone() for m in opt.exp_avg], [v.clone() for v in opt.exp_avg_sq],
                opt.step_count)
        side = torch.cuda.Stream(strat.device)
        side.wait_stream(torch.cuda.current_stream(strat.device))
        with torch.cuda.stream(side):
            strat.train_step(self.x, self.t)
        torch.cuda.current_stream(strat.device).wait_stream(side)
        torch.cuda.synchronize(strat.device)
        self._restore(snap)
        space.touch()                    # the captured forward must repack the weights
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.loss = strat.train_step(self.x, self.t)
        opt.step_count = snap[3]         # capture recorded kernels but ran none
        opt.sync_device_state()
        log.info(f"captured the training step in a HIP graph (batch {tuple(images.shape)})")

    def _restore(self, snap):
        opt, space = self.strat.optimizer, self.strat.space
        space.data.copy_(snap[0])
        for m, s in zip(opt.exp_avg, snap[1]):
            m.copy_(s)
        for v, s in zip(opt.exp_avg_sq, snap[2]):
            v.copy_(s)
        opt.step_count = snap[3]
        opt.sync_device_state()
        space.touch()

    def matches(self, images, targets) -> bool:
        return images.shape == self.x.shape and targets.shape == self.t.shape

    def __call__(self, images, targets):
        opt = self.strat.optimizer
        if float(opt.param_groups[0]["lr"]) != opt._dev_lr:
            opt.sync_device_state()
        if images.data_ptr() != self.x.data_ptr():
            self.x.copy_(images, non_blocking=True)
            self.t.copy_(targets, non_blocking=True)
        self.graph.replay()
        opt.step_count += 1
        self.strat.space.touch()         # eager users (eval) must see the updated weights
        return self.loss.clone()


class GraphedDP:
    """``-t DP`` with every replica's forward and backward replayed from HIP graphs (VERDICT r5 #3b).

    One process drives all replicas: eagerly that is ~140 kernel launches plus the Python autograd walk per
    replica under one GIL -- measured on one GPU with 8 replicas at 32 images each, 60.6 ms of host issue per
    step against 11.9 ms of device time per replica (``bench.py --parallelism dp1proc``, BASELINE.md round
    6), so 8 real GPUs would wait on the host.  Here each replica's forward (weight packing, blocks, fused
    loss partial sums) and its backward are two graphs captured once; a step is, per replica, two replays
    and a few copies, plus the cross-replica coupling done eagerly between them: the reference's global
    BCE - log Dice needs the SUM of all replicas' partial sums before any backward (dL/dS is then the same
    seed for every replica), and the gradient sum runs after the backward graphs as one reduction (the
    native RCCL clique; the bucketed overlap would have to live inside one replica's graph) before Adam.
    Capture needs one eager warm-up (lazy allocations); it changes no parameter (no optimizer step).
    Measured (profiles/session6_graph_reserve_prio_r06.txt, 8 replicas x 8 images on one GPU): host issue
    46.1 -> 20.3 ms per step, 1370 -> 1827 img/s.  ``train.py -t DP --cuda-graph`` / ``bench.py --graph``."""

    @staticmethod
    def supported(strat) -> bool:
        return type(strat) is DPStrategy and strat.device.type == "cuda"

    def __init__(self, strat, images, targets):
        self.strat = strat
        dp = strat.dp
        if dp.reducer is not None:
            dp.reducer.overlap = False          # one reduction after the backward graphs (see above)
            n = len(dp.spaces[0].numels)
            dp.reducer.buckets, dp.reducer.bucket_of = [(0, dp.spaces[0].offsets[-1], 0, n)], [0] * n
            dp.reducer.expected = [n * len(dp.spaces)]
            dp.reducer.reset()
        self.devices = dp.devices
        self.xs = [x.detach().clone() for x in dp.scatter(images)]
        self.ts = [t.detach().clone() for t in dp.scatter(targets)]
        self.n = targets.numel()
        bufs = [{k: v.clone() for k, v in r.named_buffers()} for r in dp.replicas]
        # eager warm-up: lazy allocations, packed weights, kernel caches (no optimizer step)
        for sp in dp.spaces:
            sp.zero_grad()
        loss = dp.forward_loss(images, targets)
        _backward(loss, _loss_scale(strat.cfg, images.shape[0]))
        dp.all_reduce_grads()
        torch.cuda.synchronize()
        self.S, self.dS, self.fwd, self.bwd = [], [], [], []
        for r, (comp, d) in enumerate(zip(dp.computes, self.devices)):
            with torch.cuda.device(d):
                dp.spaces[r].touch()            # the captured forward repacks the weights every replay
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    S = comp.forward_partials(self.xs[r], self.ts[r])
                self.fwd.append(g)
                self.S.append(S)
                self.dS.append(torch.zeros_like(S))
        for r, d in enumerate(self.devices):
            with torch.cuda.device(d):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=self.fwd[r].pool()):
                    torch.autograd.backward(self.S[r], self.dS[r])
                self.bwd.append(g)
        if dp.reducer is not None:
            dp.reducer.reset()                  # the captures announced gradients: nothing was reduced
        torch.cuda.synchronize()
        with torch.no_grad():                   # BatchNorm running statistics as before the captures
            for rep, b in zip(dp.replicas, bufs):
                for k, v in rep.named_buffers():
                    v.copy_(b[k])
        log.info(f"DP: captured forward + backward graphs of {len(self.devices)} replicas")

    def matches(self, images, targets) -> bool:
        return images.shape[0] == sum(x.shape[0] for x in self.xs) and images.shape[1:] == self.xs[0].shape[1:]

    def __call__(self, images, targets):
        strat, dp = self.strat, self.strat.dp
        strat.optimizer.zero_grad()
        for x, xs in zip(dp.scatter(images), self.xs):
            xs.copy_(x, non_blocking=True)
        for t, ts in zip(dp.scatter(targets), self.ts):
            ts.copy_(t, non_blocking=True)
        for r, d in enumerate(self.devices):
            with torch.cuda.device(d):
                self.fwd[r].replay()
        d0 = self.devices[0]
        St = sum(S.to(d0) for S in self.S).detach().requires_grad_(True)
        loss = loss_from_partials(St, self.n)
        _backward(loss, _loss_scale(strat.cfg, images.shape[0]))
        for r, d in enumerate(self.devices):
            with torch.cuda.device(d):
                self.dS[r].copy_(St.grad.to(d), non_blocking=True)
                self.bwd[r].replay()
        dp.all_reduce_grads()
        strat.optimizer.step()
        for sp in dp.spaces:
            sp.touch()
        return loss.detach()


class _Profiler:
    """``--profile``: torch.profiler (CPU + HIP kernel activity via roctracer) over steps 3..7 of the
    run; writes a Chrome trace ``logs/<method>_rank<r>_trace.json`` and a per-kernel table
    ``logs/<method>_rank<r>_kernels.txt``.  For counters use rocprofv3 (see README)."""

    def __init__(self, cfg, strat, start: int = 3, steps: int = 5):
        self.cfg, self.strat, self.start, self.stop = cfg, strat, start, start + steps
        self.prof = None

    def before(self, step):
        if step == self.start and self.prof is None:
            from torch.profiler import ProfilerActivity, profile
            acts = [ProfilerActivity.CPU] + ([ProfilerActivity.CUDA] if self.strat.device.type == "cuda" else [])
            self.prof = profile(activities=acts, record_shapes=False)
            self.prof.__enter__()

    def after(self, step):
        if self.prof is not None and step >= self.stop:
            if self.strat.device.type == "cuda":
                torch.cuda.synchronize(self.strat.device)
            self.prof.__exit__(None, None, None)
            base = os.path.join(self.cfg.out_dir, "logs", f"{self.cfg.train_method}_rank{self.strat.rank}")
            self.prof.export_chrome_trace(base + "_trace.json")
            sort = "self_cuda_time_total" if self.strat.device.type == "cuda" else "self_cpu_time_total"
            with open(base + "_kernels.txt", "w") as f:
                f.write(self.prof.key_averages().table(sort_by=sort, row_limit=40))
            log.info(f"profile written to {base}_trace.json")
            self.prof = None
            self.start = 1 << 60


class _SD:
    """Adapter so checkpoint helpers can take a plain state dict."""

    def __init__(self, sd):
        self._sd = sd

    def state_dict(self):
        return self._sd


class _OptIO:
    """Adapter: ``load_training_state`` hands the saved optimizer state to the strategy."""

    def __init__(self, strat):
        self.strat = strat

    def load_state_dict(self, sd):
        self.strat.load_optimizer_state_dict(sd)


class _SteadyMeter:
    """Training throughput without the first ``skip`` steps of an epoch (weight packing, allocator
    warm-up, lazy communicator setup): device-synchronised at the start mark and at the end."""

    def __init__(self, device, skip: int = 3):
        self.device, self.skip = torch.device(device), skip
        self.k, self.n, self.t0 = 0, 0, None

    def _sync(self):
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    def tick(self, batch: int):
        """Called before each step with its batch size."""
        if self.k == self.skip:
            self._sync()
            self.t0 = time.perf_counter()
        if self.k >= self.skip:
            self.n += batch
        self.k += 1

    def finish(self) -> Optional[float]:
        if self.t0 is None or self.n == 0:
            return None
        self._sync()
        return self.n / max(time.perf_counter() - self.t0, 1e-9)


class _NoBar:
    def update(self, n=1):
        pass

    def set_postfix(self, **kw):
        pass

    def close(self):
        pass


def _progress(cfg, strat, desc, total, unit):
    """tqdm bar on the main rank (reference: images per epoch, ``utils/train_utils.py:57,132``, and
    validation batches, ``evaluate.py:12``); ``--progress`` auto = only on a terminal."""
    import sys
    on = cfg.progress if cfg.progress is not None else sys.stderr.isatty()
    if not (on and strat.is_main):
        return _NoBar()
    from tqdm import tqdm
    return tqdm(total=total, desc=desc, unit=unit, leave=False)


@torch.no_grad()
def evaluate(strat: Strategy, val_loader, cfg: Optional[TrainConfig] = None):
    """Reference ``evaluate.py:6-25`` (``model.eval()``, mean per-batch loss, ``model.train()``) + Dice;
    sharded and all-reduced."""
    tot = torch.zeros(3, dtype=torch.float64)
    strat.before_eval()
    strat.set_train(False)
    bar = _progress(cfg, strat, "Validation round", len(val_loader), "batch") if cfg is not None else _NoBar()
    try:
        for images, targets in _batches(val_loader, strat.device):
            bar.update(1)
            r = strat.eval_batch(images, targets)
            if r is not None:
                loss, dice = r
                tot += torch.tensor([float(loss), float(dice), 1.0], dtype=torch.float64)
    finally:
        strat.set_train(True)
        bar.close()
    if strat.name == "DDP":
        t = tot.to(strat.device) if strat.device.type == "cuda" else tot
        tot = strat.reduce_eval(t).cpu()
    elif strat.name == "MP" and isinstance(strat, PipelineDistStrategy):
        # each pipeline's head stage holds its shard's sums (the last stage for a contiguous placement,
        # stage 0 for a mirrored one), every other rank zeros: the sum over the job is the total, on all
        t = tot.to(strat.device) if strat.device.type == "cuda" else tot
        dist.all_reduce(t)
        tot = t.cpu()
    if tot[2] == 0:
        return float("nan"), float("nan")
    return float(tot[0] / tot[2]), float(tot[1] / tot[2])
