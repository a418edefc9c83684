"""Multi-process tests on CPU with the gloo backend (world size 2-3, 127.0.0.1 rendezvous).

* DDP: bucketed all-reduce == mean of per-rank gradients; replicas stay bit-identical; the plateau
  scheduler decision is the same on every rank (reference defect A5); rank-0-only checkpoint with
  the reference ``module.`` prefix.
* GPipe over process groups: loss and every gradient equal a single-process run of the full batch
  (reference MP probe7 equivalence), for the reference 2-stage cut, balanced contiguous cuts (up to 8
  stages), half-block cuts and the mirrored V placements (2 / 3 / 4 / 8 stages).
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from distributedpytorch_amd.loss import bce_dice_from_probs
from distributedpytorch_amd.models.unet import build_model


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)


def _data(n, seed, hw=32):
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(n, 3, hw, hw, generator=g)
    t = (torch.rand(n, 1, hw, hw, generator=g) > 0.5).float()
    return x, t


def _ddp_worker(rank, world, port, bucket_mb, q, comm="fp32", overlap=True):
    _init(rank, world, port)
    from distributedpytorch_amd.config import TrainConfig
    from distributedpytorch_amd.trainer import DDPStrategy
    model = build_model("unet-tiny")
    if rank == 1:   # different init on purpose: DDP must broadcast rank 0's parameters
        for p in model.parameters():
            p.data.add_(1.0)
    cfg = TrainConfig(train_method="DDP", backend="torch", dtype="fp32", lr=1e-3, bucket_mb=bucket_mb,
                      grad_comm_dtype=comm, comm_overlap=overlap)
    st = DDPStrategy(cfg, model, "cpu")
    x, t = _data(4, seed=10 + rank)
    # expected: per-rank plain-autograd grads of the (broadcast) rank-0 weights, averaged
    plain = build_model("unet-tiny")
    plain.load_state_dict(st.model.state_dict())
    (bce_dice_from_probs(plain(x), t) * x.shape[0]).backward()
    pg = dict(plain.named_parameters())
    local = torch.cat([pg[n].grad.reshape(-1) for n in st.space.names])     # flat-buffer layout order
    allg = [torch.zeros_like(local) for _ in range(world)]
    dist.all_gather(allg, local)
    expect = sum(allg) / world
    st.optimizer.zero_grad()
    loss = st.forward_loss(x, t)
    (loss * x.shape[0]).backward()      # buckets are all-reduced in place, overlapped with backward
    launched_in_backward = len(st.reducer.launch_log)
    st.reducer.finish()
    if comm == "bf16":   # bf16 wire: relative error of a few bf16 ulps
        ok_reduce = torch.allclose(st.space.grad, expect, rtol=2e-2, atol=1e-4 * float(expect.abs().max()))
    else:
        ok_reduce = torch.allclose(st.space.grad, expect, atol=1e-6)
    st.optimizer.step()
    for i in range(2):
        st.train_step(*_data(4, seed=100 + 10 * i + rank))
    params = st.space.data.clone()
    allp = [torch.zeros_like(params) for _ in range(world)]
    dist.all_gather(allp, params)
    same = all(torch.equal(allp[0], p) for p in allp)
    # scheduler sync (A5): rank-local val losses differ, decision must not
    from distributedpytorch_amd.optim import make_plateau, plateau_step
    sch = make_plateau(st.optimizer, patience=0)
    for v in ([1.0, 2.0, 3.0] if rank == 0 else [3.0, 2.0, 1.0]):
        plateau_step(sch, v)
    lr = torch.tensor([st.optimizer.param_groups[0]["lr"]])
    alllr = [torch.zeros_like(lr) for _ in range(world)]
    dist.all_gather(alllr, lr)
    q.put((rank, ok_reduce, same, [float(v) for v in alllr], len(st.reducer.buckets), launched_in_backward))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,bucket_mb,comm,overlap", [(2, 0.001, "fp32", True), (2, 8.0, "fp32", True),
                                                          (4, 0.004, "fp32", True), (2, 0.004, "bf16", True),
                                                          (2, 0.001, "fp32", False)])
def test_ddp_gloo_ranks(world, bucket_mb, comm, overlap):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ddp_worker, args=(r, world, port, bucket_mb, q, comm, overlap))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, ok_reduce, same, lrs, nb, in_bwd in res:
        assert ok_reduce, f"rank {rank}: bucketed all-reduce != mean of grads"
        assert same, "replicas diverged"
        assert len(set(lrs)) == 1, f"scheduler diverged across ranks: {lrs}"
        if not overlap:   # --no-comm-overlap: one collective, launched after the backward
            assert nb == 1 and in_bwd == 0
        elif bucket_mb < 0.01:
            assert nb > 3 and in_bwd >= nb - 1


def _pipe_worker(rank, world, port, microbatches, mode, q, model_name="unet-tiny"):
    _init(rank, world, port)
    from distributedpytorch_amd.parallel.pipeline import GPipeDist
    torch.manual_seed(0)
    model = build_model(model_name)
    ref = build_model(model_name)
    ref.load_state_dict(model.state_dict())
    from distributedpytorch_amd.parallel.placement import parse_placement, v_partition
    cuts = list(mode) if isinstance(mode, (list, tuple)) else None
    placement = None
    if mode == "v":
        placement = v_partition(model.cfg, world, 32, 32)
    elif isinstance(mode, str) and (":" in mode or "@" in mode):
        placement = parse_placement(mode)
    pipe = GPipeDist(model, microbatches, backend="torch", dtype="fp32", img_hw=(32, 32),
                     mode="balanced" if (cuts or placement) else mode, cuts=cuts, placement=placement)
    x, t = _data(4, seed=5)
    loss = pipe.train_step(x if pipe.is_first else None, t if pipe.is_last else None, 4, (32, 32))
    lref = bce_dice_from_probs(ref(x), t)
    lref.backward()
    own = dict(model.named_parameters())
    refp = dict(ref.named_parameters())
    bad = []
    for n, p in own.items():
        if p.requires_grad and p.grad is not None:
            if not torch.allclose(p.grad, refp[n].grad, atol=1e-5):
                bad.append(n)
    nown = sum(1 for p in own.values() if p.requires_grad)
    probs = pipe.eval_probs(x if pipe.is_first else None, 4, (32, 32))
    probs_ok = True
    if pipe.is_last:
        with torch.no_grad():
            probs_ok = torch.allclose(probs, ref(x), atol=1e-5)
    sd = pipe.gather_state_dict()
    sd_ok = True
    if rank == 0:
        # (BatchNorm running statistics: the reference model ran one more train-mode forward above)
        sd_ok = set(sd) == set(ref.state_dict()) and all(torch.equal(sd[k], v) for k, v in ref.state_dict().items()
                                                         if "running_" not in k and "num_batches" not in k)
    q.put((rank, None if loss is None else float(loss), float(lref), bad, nown, probs_ok, sd_ok, pipe.is_last))
    dist.destroy_process_group()


# cuts inside DoubleConv blocks (x.5: a stage boundary between a block's two convs): unet-tiny is
# enc0 enc1 mid dec0 dec1 head; [0, 1.5, 3.5, 6] splits enc1 and dec0, [0, .5, 2.5, 4.5, 6] the first
# encoder block, the bottleneck and the last decoder block; unet-tiny-bn adds BatchNorm + bilinear ups
# (one microbatch: BatchNorm statistics over a microbatch are not the full batch's)
# V placements (parallel/placement.py): stage s owns encoder level(s) s and the same decoder level(s); the
# head stage is stage 0.  "v:0,1,3,6" keeps mid with enc1 on stage 1, so skip1 crosses 1 -> 0 with x;
# "v:0,1,2,5,8,10" (unet-tiny4) sends skips 2 and 3 from stage 2 to stage 1 in one message while skip 1 is
# handed over locally between stage 1's two segments; "0,1,5,8,10@0,1,0,1" is not a V at all (stage 1
# owns enc1..mid and the last decoder + head): two segments of one stage feed the other stage on
# separate communicators
@pytest.mark.parametrize("world,mb,mode,model_name", [(2, 2, "reference", "unet-tiny"), (3, 4, "balanced", "unet-tiny"),
                                                      (3, 2, (0, 1.5, 3.5, 6), "unet-tiny"),
                                                      (4, 2, (0, 0.5, 2.5, 4.5, 6), "unet-tiny"),
                                                      (3, 1, (0, 1.5, 3.5, 6), "unet-tiny-bn"),
                                                      (2, 4, "v", "unet-tiny"),
                                                      (2, 2, "v:0,1.5,3.5,6", "unet-tiny"),
                                                      (2, 2, "v:0,1,3,6", "unet-tiny"),
                                                      (3, 2, "v:0,1,2,5,8,10", "unet-tiny4"),
                                                      (2, 4, "0,1,5,8,10@0,1,0,1", "unet-tiny4"),
                                                      (4, 4, "v", "unet-tiny4"),
                                                      (2, 1, "v", "unet-tiny-bn"),
                                                      (8, 2, "v", "unet-tiny4"),
                                                      (8, 2, "balanced", "unet-tiny4")])
def test_gpipe_gloo_matches_single_process(world, mb, mode, model_name):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipe_worker, args=(r, world, port, mb, mode, q, model_name)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    total_own = 0
    assert sum(r[-1] for r in res) == 1                # exactly one head stage
    for rank, loss, lref, bad, nown, probs_ok, sd_ok, is_head in res:
        assert not bad, f"rank {rank}: grads differ for {bad}"
        total_own += nown
        assert probs_ok and sd_ok
        if is_head:
            assert abs(loss - lref) < 1e-5
    assert total_own == len(list(build_model(model_name).parameters()))   # each parameter owned by one stage


def _ddp_bn_worker(rank, world, port, q):
    _init(rank, world, port)
    from distributedpytorch_amd.config import TrainConfig
    from distributedpytorch_amd.trainer import DDPStrategy
    model = build_model("unet-tiny-bn")
    st = DDPStrategy(TrainConfig(train_method="DDP", backend="torch", dtype="fp32", lr=1e-3), model, "cpu")
    st.train_step(*_data(4, seed=20 + rank))          # rank-local batch statistics
    rm = st.model.encoder.conv1.conv_block[1].running_mean.clone()
    before = [torch.zeros_like(rm) for _ in range(world)]
    dist.all_gather(before, rm)
    st.before_eval()                                  # torch DDP broadcast_buffers semantics
    rm = st.model.encoder.conv1.conv_block[1].running_mean.clone()
    after = [torch.zeros_like(rm) for _ in range(world)]
    dist.all_gather(after, rm)
    q.put((rank, not torch.equal(before[0], before[1]), all(torch.equal(after[0], a) for a in after)))
    dist.destroy_process_group()


def test_ddp_bn_running_stats_follow_rank0():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ddp_bn_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, differed, same in res:
        assert differed and same, (rank, differed, same)


@pytest.mark.parametrize("layout", [torch.channels_last, torch.contiguous_format])
def test_pipeline_wire_roundtrip(layout):
    """GPipe wire format: a stage-layout tensor flattened in storage order on the send side and the
    receive buffer's 1-D storage view reassemble the same logical NCHW tensor in the stage layout."""
    import types
    from distributedpytorch_amd.parallel.pipeline import GPipeDist
    f = types.SimpleNamespace(comm_dtype=torch.float32, device=torch.device("cpu"), _recv_layout=lambda: layout)
    t = torch.randn(2, 5, 3, 4).contiguous(memory_format=layout)
    wire = GPipeDist._wire(f, t)
    assert wire.dim() == 1 and wire.is_contiguous() and wire.numel() == t.numel()
    r, flat = GPipeDist._empty_wire(f, tuple(t.shape))
    assert flat.dim() == 1 and flat.is_contiguous()
    flat.copy_(wire)
    assert torch.equal(r, t) and r.is_contiguous(memory_format=layout)


def _ddp_train_worker(rank, world, port, out, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    try:
        from distributedpytorch_amd.config import parse_args
        from distributedpytorch_amd.trainer import train
        args = ["--synthetic", "--synthetic-len", str(8 * world), "-v", "25", "--img-size", "32", "--model",
                "unet-tiny", "--backend", "torch", "--dtype", "fp32", "-b", "2", "--log-every", "1", "--lr", "1e-3",
                "-t", "DDP", "-e", "2", "--bucket-mb", "0.004", "--out-dir", out]
        r = train(parse_args(args))
        st = r["strategy"]
        flat = st.space.data.detach().clone()
        allp = [torch.zeros_like(flat) for _ in range(world)]
        dist.all_gather(allp, flat)
        log = torch.tensor([b for b, _, _ in st.reducer.last_launch_log], dtype=torch.int64)
        logs = [torch.zeros_like(log) for _ in range(world)]
        dist.all_gather(logs, log)
        in_bwd = sum(1 for _, _, fin in st.reducer.last_launch_log if not fin)
        lr = torch.tensor([st.optimizer.param_groups[0]["lr"]])
        lrs = [torch.zeros_like(lr) for _ in range(world)]
        dist.all_gather(lrs, lr)
        q.put((rank, r["step"], all(torch.equal(allp[0], p) for p in allp), [l.tolist() for l in logs],
               len(st.reducer.buckets), in_bwd, [float(v) for v in lrs], None))
    except Exception as e:   # surface the failure instead of a queue timeout
        import traceback
        q.put((rank, -1, False, None, 0, 0, None, repr(e) + traceback.format_exc()[-1500:]))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_ddp_trainer_eight_ranks(tmp_path):
    """The whole DDP training loop (train.py -t DDP) at world 8 on gloo: replicas bit-identical after two
    epochs; every rank launched the same bucket sequence 0..n-1, all but the last during the backward;
    the plateau scheduler's LR identical on all ranks (A5); rank 0 alone wrote checkpoints/DDP.pth with
    the reference ``module.`` keys and the loss pickles."""
    world = 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ddp_train_worker, args=(r, world, port, str(tmp_path), q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=400) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    errs = [(r[0], r[-1]) for r in res if r[-1] is not None]
    assert not errs, errs
    nb = res[0][4]
    assert nb > 3
    for rank, steps, same, logs, _, in_bwd, lrs, _ in res:
        assert steps > 0 and same, f"rank {rank}: replicas diverged"
        assert all(l == list(range(nb)) for l in logs), f"bucket order differs across ranks: {logs}"
        assert in_bwd >= nb - 1
        assert len(set(lrs)) == 1, lrs
    sd = torch.load(tmp_path / "checkpoints" / "DDP.pth", map_location="cpu", weights_only=True)
    assert sd and all(k.startswith("module.") for k in sd)
    assert set(k[len("module."):] for k in sd) == set(build_model("unet-tiny").state_dict())
    assert (tmp_path / "loss" / "DDP" / "train_loss.pkl").exists() and (tmp_path / "loss" / "DDP" / "val_loss.pkl").exists()


def _mp_train_worker(rank, world, port, out, cut, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    try:
        from distributedpytorch_amd.config import parse_args
        from distributedpytorch_amd.trainer import train
        args = ["--synthetic", "--synthetic-len", "16", "-v", "25", "--img-size", "32", "--model", "unet-tiny",
                "--backend", "torch", "--dtype", "fp32", "-b", "4", "--log-every", "1", "--lr", "1e-3", "-t", "MP",
                "-e", "2", "--mp-cut", cut, "--out-dir", out]
        r = train(parse_args(args))
        st = r["strategy"]
        lr = torch.tensor([st.optimizer.param_groups[0]["lr"]])
        lrs = [torch.zeros_like(lr) for _ in range(world)]
        dist.all_gather(lrs, lr)
        q.put((rank, r["step"], str(st.pipe.pl), st.pipe.head_rank, [float(v) for v in lrs], None))
    except Exception as e:
        import traceback
        q.put((rank, -1, None, None, None, repr(e) + traceback.format_exc()[-1500:]))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("cut", ["v", "reference"])
def test_mp_trainer_two_ranks(tmp_path, cut):
    """The whole -t MP training loop at world 2 on gloo, for the mirrored (V) placement -- head and loss
    on stage 0 -- and the reference encoder|decoder cut (head on the last stage): finite validation loss
    shared with every stage (the broadcast comes from the head stage), the plateau LR identical on both
    ranks, the gathered checkpoint with every reference key written once by rank 0."""
    import pickle  # noqa: F401  (the loss pickles are only checked for existence)
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_mp_train_worker, args=(r, world, port, str(tmp_path), cut, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=400) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    errs = [(r[0], r[-1]) for r in res if r[-1] is not None]
    assert not errs, errs
    assert res[0][3] == (0 if cut == "v" else 1), res[0][2]
    for rank, steps, _, _, lrs, _ in res:
        assert steps > 0 and len(set(lrs)) == 1, (rank, lrs)
    sd = torch.load(tmp_path / "checkpoints" / "MP.pth", map_location="cpu", weights_only=True)
    assert set(sd) == set(build_model("unet-tiny").state_dict())
    import json
    rows = [json.loads(l) for l in open(tmp_path / "logs" / "MP.jsonl")]
    vals = [r["val_loss"] for r in rows if "val_loss" in r]
    assert vals and all(v == v and abs(v) < 1e3 for v in vals), vals


def _hybrid_worker(rank, world, port, replicas, mode, q, model_name="unet-tiny"):
    _init(rank, world, port)
    from distributedpytorch_amd.config import TrainConfig
    from distributedpytorch_amd.trainer import PipelineDistStrategy
    torch.manual_seed(0)
    model = build_model(model_name)
    ref = build_model(model_name)
    ref.load_state_dict(model.state_dict())
    S = world // replicas
    if rank >= S:   # other pipelines start from different weights: pipeline 0's must be broadcast
        for p in model.parameters():
            p.data.add_(0.5)
    cfg = TrainConfig(train_method="MP", backend="torch", dtype="fp32", lr=1e-3, mp_replicas=replicas,
                      mp_cut=mode, microbatches=2, img_size=(32, 32), model=model_name, batch_size=4)
    try:
        st = PipelineDistStrategy(cfg, model, "cpu")
    except Exception as e:      # surface the failure instead of a queue timeout
        q.put((rank, -1, -1, repr(e), False, False, False))
        raise
    r = st.replica
    x, t = _data(4, seed=50 + r)
    st.train_step(x, t)
    # expected: the mean over the pipelines of the plain full-batch gradient (loss x batch, A11)
    grads = []
    for k in range(replicas):
        ref.zero_grad()
        xk, tk = _data(4, seed=50 + k)
        (bce_dice_from_probs(ref(xk), tk) * 4).backward()
        rp = dict(ref.named_parameters())
        grads.append(torch.cat([rp[n].grad.reshape(-1) for n in st.pipe.space.names]))
    expect = sum(grads) / replicas
    if model_name.endswith("-bn"):
        # BatchNorm statistics are per microbatch in the pipeline: no full-batch reference gradient
        ok_grad = bool(torch.isfinite(st.pipe.space.grad).all())
    else:
        ok_grad = torch.allclose(st.pipe.space.grad, expect, atol=1e-5, rtol=1e-4)
    # the replicas' gradient all-reduce launched its buckets from the backward, not after it (ADVICE r5 /
    # overlapped with the pipeline drain)
    log = st.reducer.last_launch_log if st.reducer is not None else []
    overlapped = all(not in_finish for _, _, in_finish in log)
    for i in range(2):
        st.train_step(*_data(4, seed=200 + 10 * i + r))
    params = st.pipe.space.data.clone()
    # the same stage of every pipeline holds the same parameters
    same = []
    if st.dp_group is not None:
        allp = [torch.zeros_like(params) for _ in range(replicas)]
        dist.all_gather(allp, params, group=st.dp_group)
        same = [torch.equal(allp[0], p) for p in allp]
        # BatchNorm running statistics: pipeline 0's after the buffer sync that precedes validation
        st.before_eval()
        from distributedpytorch_amd.parallel.pipeline import placement_buffer_names
        bufs = dict(st.model.named_buffers())
        for n in placement_buffer_names(st.model, st.pipe.pl, st.stage):
            b = bufs[n].double().reshape(-1)
            allb = [torch.zeros_like(b) for _ in range(replicas)]
            dist.all_gather(allb, b, group=st.dp_group)
            same += [torch.equal(allb[0], v) for v in allb]
        sd = st.state_dict()
        same.append((sd is None) == (st.replica != 0 or st.stage != 0))
    q.put((rank, st.replica, st.stage, ok_grad and overlapped, all(same), st.pipe.is_last, st.is_main))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,replicas,mode,model_name", [(4, 2, "v", "unet-tiny"), (4, 2, "reference", "unet-tiny"),
                                                         (6, 3, "v", "unet-tiny"), (4, 4, "balanced", "unet-tiny"),
                                                         (4, 2, "v", "unet-tiny-bn")])
def test_pipeline_replicas_data_parallel(world, replicas, mode, model_name):
    """-t MP with --mp-replicas R: R pipelines of world/R stages (ranks r*S .. r*S+S-1), each on its own
    batch; every stage's gradient equals the mean over the pipelines of the plain full-batch gradients,
    pipeline 0's initial parameters reach every pipeline, and the same stage of all pipelines stays
    bit-identical across optimizer steps (R = world: plain data parallelism through the pipeline code)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_hybrid_worker, args=(r, world, port, replicas, mode, q, model_name))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    S = world // replicas
    for rank, rep, stage, ok_grad, same, _, _ in res:
        assert isinstance(ok_grad, bool), ok_grad
        assert (rep, stage) == divmod(rank, S)
        assert ok_grad, f"rank {rank}: stage gradient != mean of the pipelines' gradients"
        assert same, f"rank {rank}: stage parameters differ across pipelines"
    assert sum(r[-2] for r in res) == replicas          # one head stage per pipeline
    assert sum(r[-1] for r in res) == 1                 # one main (logging) rank: pipeline 0's head


def _spatial_worker(rank, world, port, plan_kw, M, q):
    _init(rank, world, port)
    from distributedpytorch_amd.parallel.spatial import SpatialPlan
    from distributedpytorch_amd.parallel.spatial_pipe import SpatialGPipe
    torch.manual_seed(0)
    model = build_model("unet-tiny4")
    ref = build_model("unet-tiny4")
    ref.load_state_dict(model.state_dict())
    plan = SpatialPlan(**plan_kw)
    try:
        pipe = SpatialGPipe(model, plan, M, backend="torch", dtype="fp32", img_hw=(64, 64))
        x, t = _data(4, seed=11, hw=64)
        loss = pipe.train_step(x, t, 4, (64, 64))
    except Exception as e:
        import traceback
        q.put((rank, repr(e) + traceback.format_exc(), None, None, None, None))
        raise
    lref = bce_dice_from_probs(ref(x), t)
    lref.backward()
    refp = dict(ref.named_parameters())
    # relative to each gradient's own scale (an absolute bound hid swapped microbatches once)
    bad = [n for n, p in model.named_parameters()
           if p.requires_grad and float((p.grad - refp[n].grad).abs().max()) > 1e-4 * float(refp[n].grad.abs().max())]
    nown = sum(1 for p in model.parameters() if p.requires_grad)
    probs = pipe.eval_probs(x, 4, (64, 64))
    with torch.no_grad():
        probs_ok = bool(torch.allclose(probs, ref(x), atol=1e-5))
    sd = pipe.gather_state_dict()
    sd_ok = rank != 0 or (set(sd) == set(ref.state_dict())
                          and all(torch.equal(sd[k], v) for k, v in ref.state_dict().items()))
    q.put((rank, None, float(loss), float(lref), bad, (nown, probs_ok, sd_ok)))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,plan_kw,M", [
    (2, dict(S=2, inner_cuts=(1, 3, 6, 8), inner_owner=(0, 1, 0), L=1), 2),              # inner V
    (2, dict(S=2, inner_cuts=(1, 4, 8), inner_owner=(0, 1), L=1, bounds=(0, 24, 64)), 1),  # uneven rows
    (4, dict(S=4, inner_cuts=(2, 3, 3.5, 4, 5, 5.5, 6, 7), inner_owner=(0, 1, 2, 3, 2, 1, 0), L=2), 2),
    (8, dict(S=8, inner_cuts=(1, 1.5, 2, 3, 4, 5, 6, 7, 8), inner_owner=tuple(range(8)), L=1), 2),
])
def test_spatial_pipeline_matches_single_process(world, plan_kw, M):
    """Row-split top levels (parallel/spatial.py, spatial_pipe.py): every stage runs the split levels on its
    own image rows (halo rows recomputed, never exchanged), the inner chain is pipelined; loss, every
    parameter gradient (split levels after their all-reduce), the probabilities and the gathered state dict
    equal a single-process run of the full batch -- at 2, 4 and 8 stages, 1 and 2 split levels, inner V and
    contiguous chains and uneven row slices."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_spatial_worker, args=(r, world, port, plan_kw, M, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    for rank, err, loss, lref, bad, extra in res:
        assert err is None, f"rank {rank}: {err}"
        assert abs(loss - lref) < 1e-5, (rank, loss, lref)
        assert not bad, f"rank {rank}: grads differ for {bad}"
        nown, probs_ok, sd_ok = extra
        assert probs_ok and sd_ok, (rank, probs_ok, sd_ok)


def _spatial_trainer_worker(rank, world, port, q):
    _init(rank, world, port)
    from distributedpytorch_amd.config import TrainConfig
    from distributedpytorch_amd.trainer import PipelineDistStrategy
    torch.manual_seed(0)
    model = build_model("unet-tiny4")
    ref = build_model("unet-tiny4")
    ref.load_state_dict(model.state_dict())
    cfg = TrainConfig(train_method="MP", backend="torch", dtype="fp32", lr=1e-3, mp_cut="spatial", microbatches=2,
                      img_size=(64, 64), model="unet-tiny4", batch_size=4)
    try:
        st = PipelineDistStrategy(cfg, model, "cpu")
        x, t = _data(4, seed=3, hw=64)
        loss = st.train_step(x, t)
        ev = st.eval_batch(x, t)
        sd = st.state_dict()
        res = (st.plan.mode, float(loss), ev is not None, sd is not None, st.is_main)
    except Exception as e:
        import traceback
        res = (repr(e) + traceback.format_exc(),)
    q.put((rank, res))
    dist.destroy_process_group()


def test_spatial_plan_through_mp_strategy():
    """``-t MP --mp-cut spatial``: the FLOP-balanced row-split plan (parallel/spatial.py ``default_plan``)
    drives PipelineDistStrategy: a training step, validation counted once (stage 0), rank 0's state dict."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_spatial_trainer_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    for rank, r in res:
        assert len(r) == 5, r[0]
        mode, loss, has_eval, has_sd, main = r
        assert mode == "spatial" and loss == loss
        assert has_eval == (rank == 0) and has_sd == (rank == 0) and main == (rank == 0)
    assert res[0][1][1] == res[1][1][1]            # every stage holds the same full-batch loss
