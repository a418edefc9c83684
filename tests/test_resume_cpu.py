"""Checkpoint / resume for every strategy whose state is not a single replica (CPU, gloo).

A run stopped after epoch 1 and resumed with ``--resume`` must end where an uninterrupted run
ends: same parameters, every DP replica identical, every pipeline stage's own Adam state restored
(the advisor found DP resuming only replica 0 and multi-process MP crashing on a stage-0-only
optimizer state).  Also: the training order is a pure function of (seed, epoch), so the pipeline's
first stage (images) and last stage (masks) pair up whatever the process-global RNG did.
"""
import os
import socket

import torch
import torch.multiprocessing as mp

from distributedpytorch_amd.config import parse_args

ARGS = ["--synthetic", "--synthetic-len", "16", "-v", "25", "--img-size", "32", "--model", "unet-tiny",
        "--backend", "torch", "--dtype", "fp32", "-b", "4", "--log-every", "1", "--lr", "1e-3"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _load(path):
    return torch.load(path, map_location="cpu", weights_only=True)


def test_epoch_sampler_is_rank_independent():
    from distributedpytorch_amd.data.loaders import build_loaders
    ds = list(range(20))
    orders = []
    for rng_seed in (1, 2):                       # different global RNG state per "rank"
        torch.manual_seed(rng_seed)
        tl, _, sampler = build_loaders(ds, ds[:4], 4, seed=7)
        per_epoch = []
        for ep in range(2):
            sampler.set_epoch(ep)
            per_epoch.append(torch.cat(list(tl)).tolist())
        orders.append(per_epoch)
    assert orders[0] == orders[1]
    assert orders[0][0] != orders[0][1]           # reshuffled per epoch (A7)
    assert sorted(orders[0][0]) == ds


def test_dp_resume_matches_uninterrupted(tmp_path):
    from distributedpytorch_amd.trainer import train
    a = train(parse_args(ARGS + ["-t", "DP", "-e", "2", "--out-dir", str(tmp_path / "a")]))
    train(parse_args(ARGS + ["-t", "DP", "-e", "1", "--out-dir", str(tmp_path / "b")]))
    b = train(parse_args(ARGS + ["-t", "DP", "-e", "2", "--resume", "--out-dir", str(tmp_path / "b")]))
    assert a["step"] == b["step"] > 0
    reps = b["strategy"].dp.replicas
    for p, q in zip(reps[0].parameters(), reps[1].parameters()):
        assert torch.equal(p, q), "DP replicas diverged after resume"
    sa, sb = _load(tmp_path / "a" / "checkpoints" / "DP.pth"), _load(tmp_path / "b" / "checkpoints" / "DP.pth")
    assert set(sa) == set(sb) and all(k.startswith("module.") for k in sa)
    for k in sa:
        torch.testing.assert_close(sa[k], sb[k], rtol=1e-5, atol=1e-6, msg=k)


def _mp_worker(rank, world, port, out, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist
    from distributedpytorch_amd.trainer import train
    try:
        base = ARGS + ["-t", "MP", "--microbatches", "2"]
        a = train(parse_args(base + ["-e", "2", "--out-dir", os.path.join(out, "a")]))
        train(parse_args(base + ["-e", "1", "--out-dir", os.path.join(out, "b")]))
        b = train(parse_args(base + ["-e", "2", "--resume", "--out-dir", os.path.join(out, "b")]))
        # each stage's own Adam moments must match the uninterrupted run
        ma = a["strategy"].optimizer.exp_avg[0]
        mb = b["strategy"].optimizer.exp_avg[0]
        q.put((rank, a["step"], b["step"], bool(torch.allclose(ma, mb, rtol=1e-5, atol=1e-7)), None))
    except Exception as e:  # report instead of hanging the parent
        import traceback
        q.put((rank, -1, -1, False, repr(e) + traceback.format_exc()[-1500:]))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_mp_pipeline_resume_matches_uninterrupted(tmp_path):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_mp_worker, args=(r, 2, port, str(tmp_path), q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    errs = [(r[0], r[4]) for r in res if r[4] is not None]
    assert not errs, errs
    for rank, sa, sb, moments_ok, err in res:
        assert sa == sb > 0
        assert moments_ok, f"stage {rank}: Adam state not restored"
    ck = tmp_path / "b" / "checkpoints" / "MP_last.pt"
    st = _load(ck)
    assert len(st["optimizer"]["stages"]) == 2
    sa, sb = _load(tmp_path / "a" / "checkpoints" / "MP.pth"), _load(tmp_path / "b" / "checkpoints" / "MP.pth")
    assert set(sa) == set(sb)
    for k in sa:
        torch.testing.assert_close(sa[k], sb[k], rtol=1e-5, atol=1e-6, msg=k)


def test_dp_bn_buffers_follow_replica0():
    """-t DP with BatchNorm: each replica updates running statistics from its own shard; before
    eval (and in the checkpoint) every replica uses replica 0's, as torch.nn.DataParallel does."""
    from distributedpytorch_amd.config import TrainConfig
    from distributedpytorch_amd.models.unet import build_model
    from distributedpytorch_amd.trainer import DPStrategy
    torch.manual_seed(0)
    st = DPStrategy(TrainConfig(train_method="DP", backend="torch", dtype="fp32", lr=1e-3),
                    build_model("unet-tiny-bn"), ["cpu", "cpu"])
    x = torch.rand(4, 3, 32, 32)
    x[2:] *= 3.0                                   # shards with different statistics
    t = (torch.rand(4, 1, 32, 32) > 0.5).float()
    st.train_step(x, t)
    bufs = lambda r: [b.clone() for b in r.buffers() if b.is_floating_point()]  # noqa: E731
    b0, b1 = bufs(st.dp.replicas[0]), bufs(st.dp.replicas[1])
    assert any(not torch.equal(u, v) for u, v in zip(b0, b1))
    st.before_eval()
    assert all(torch.equal(u, v) for u, v in zip(b0, bufs(st.dp.replicas[1])))
