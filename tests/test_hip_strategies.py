"""Strategies on the HIP engine (one GPU: stages / replicas placed on cuda:0 twice).

The pipeline splits the batch into microbatches and sums their loss partials on the last stage
(reference MP semantics, unet_model.py:24-53) and DP sums replica gradients (reference
DataParallel); both must match a single-device step of the same batch with the same kernels.
"""
import gc
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _cos(a, b):
    a, b = a.double().reshape(-1), b.double().reshape(-1)
    return (a @ b / (a.norm() * b.norm()).clamp_min(1e-30)).item()


def _batch(n=4, hw=64):
    from distributedpytorch_amd.data.synthetic import synthetic_batch
    img, mask = synthetic_batch(n, hw, hw, 3, seed=11)
    return img.cuda(), mask.float().unsqueeze(1).cuda()


def _single(model, x, t):
    from distributedpytorch_amd.config import TrainConfig
    from distributedpytorch_amd.trainer import SingleDevice
    st = SingleDevice(TrainConfig(backend="hip", lr=1e-3), model, "cuda:0")
    st.optimizer.zero_grad()
    loss = st.forward_loss(x, t)
    (loss * x.shape[0]).backward()
    return loss.detach(), {n: p.grad.detach().clone() for n, p in model.named_parameters()}


@pytest.mark.parametrize("cut", ["reference", "v"])
def test_pipeline_local_hip_matches_single(hip_lib, cut):
    from distributedpytorch_amd.models.unet import build_model
    from distributedpytorch_amd.parallel.pipeline import GPipeLocal
    from distributedpytorch_amd.parallel.placement import Placement
    torch.manual_seed(0)
    a, b = build_model("unet"), build_model("unet")
    b.load_state_dict(a.state_dict())
    x, t = _batch()
    l_ref, g_ref = _single(b.cuda(), x, t)
    pl = Placement.mirrored([0, 2, 7, 10]) if cut == "v" else None
    pipe = GPipeLocal(a, ["cuda:0", "cuda:0"], 2, backend="hip", dtype="bf16", img_hw=(64, 64), mode="reference",
                      placement=pl)
    for s in pipe.spaces:
        s.zero_grad()
    loss = pipe.forward_loss(x, t)
    (loss * x.shape[0]).backward()
    torch.cuda.synchronize()
    assert abs(loss.item() - l_ref.item()) < 1e-3 * abs(l_ref.item())
    for n, p in a.named_parameters():
        assert _cos(p.grad, g_ref[n]) > 0.999, n
    # the encoder stage's concat buffers (consumed as copies by the decoder stage's engine) must not
    # outlive the step: repeated steps keep allocated memory flat
    del loss
    gc.collect()
    torch.cuda.synchronize()
    base = torch.cuda.memory_allocated()
    for _ in range(3):
        for s in pipe.spaces:
            s.zero_grad()
        (pipe.forward_loss(x, t) * x.shape[0]).backward()
    gc.collect()
    torch.cuda.synchronize()
    assert torch.cuda.memory_allocated() <= base + (1 << 20)
    assert len(pipe.stage_blocks[0]._cats) == 0


def test_dp_hip_matches_single(hip_lib):
    from distributedpytorch_amd.config import TrainConfig
    from distributedpytorch_amd.models.unet import build_model
    from distributedpytorch_amd.trainer import DPStrategy
    torch.manual_seed(1)
    a, b = build_model("unet"), build_model("unet")
    b.load_state_dict(a.state_dict())
    x, t = _batch()
    l_ref, g_ref = _single(b.cuda(), x, t)
    st = DPStrategy(TrainConfig(backend="hip", lr=1e-3, bucket_mb=1.0), a, ["cuda:0", "cuda:0"])
    st.optimizer.zero_grad()
    loss = st.dp.forward_loss(x, t)
    (loss * x.shape[0]).backward()
    # overlap: the HIP backward announced gradients block by block on both replicas, and every
    # bucket but the last was launched during the backward (in index order), not by finish()
    red = st.dp.reducer
    log = list(red.launch_log)
    assert len(red.buckets) >= 3
    assert [b for b, _, _ in log] == list(range(len(log))) and len(log) >= len(red.buckets) - 1, log
    assert not any(fin for _, _, fin in log) and log[0][1] < 2 * len(st.dp.spaces[0].names), log
    st.dp.all_reduce_grads()
    torch.cuda.synchronize()
    assert abs(loss.item() - l_ref.item()) < 1e-3 * abs(l_ref.item())
    for n, p in st.model.named_parameters():
        assert _cos(p.grad, g_ref[n]) > 0.999, n
    st.optimizer.step()
    for p, q in zip(st.dp.replicas[0].parameters(), st.dp.replicas[1].parameters()):
        assert torch.equal(p, q)


@pytest.mark.parametrize("model_name", ["unet", "unet-bn"])
def test_graphed_dp_matches_eager_dp(hip_lib, model_name):
    """-t DP with every replica's forward and backward replayed from HIP graphs (trainer.GraphedDP, VERDICT r5
    #3b): three steps give the losses, parameters and BatchNorm running statistics of the eager DP steps on
    the same batches (2 replicas sharing cuda:0)."""
    from distributedpytorch_amd.config import TrainConfig
    from distributedpytorch_amd.models.unet import build_model
    from distributedpytorch_amd.trainer import DPStrategy, GraphedDP
    torch.manual_seed(1)
    a, b = build_model(model_name), build_model(model_name)
    b.load_state_dict(a.state_dict())
    batches = [_batch() for _ in range(3)]
    runs = []
    for model, graphed in ((a, False), (b, True)):
        st = DPStrategy(TrainConfig(backend="hip", lr=1e-3, bucket_mb=1.0), model, ["cuda:0", "cuda:0"])
        step = GraphedDP(st, *batches[0]) if graphed else st.train_step
        losses = [float(step(x, t)) for x, t in batches]
        torch.cuda.synchronize()
        runs.append((losses, st.dp.spaces[0].data.clone(), st.dp.spaces[1].data.clone(),
                     {k: v.clone() for k, v in st.dp.replicas[0].named_buffers()}))
    (l0, p0, q0, b0), (l1, p1, q1, b1) = runs
    for x, y in zip(l0, l1):
        assert abs(x - y) <= 1e-5 * abs(x), (l0, l1)
    assert torch.equal(p1, q1)                        # graphed replicas stay identical
    assert float((p1 - p0).abs().max()) <= 1e-6 * float(p0.abs().max())
    for k in b0:
        assert torch.allclose(b1[k].float(), b0[k].float(), rtol=1e-5, atol=1e-6), k


def test_train_py_dp_cuda_graph(hip_lib, tmp_path):
    """``train.py -t DP --cuda-graph`` runs the replicas from captured graphs (trainer.GraphedDP) end to end:
    training, validation and the checkpoint."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, os.path.join(root, "train.py"), "-t", "DP", "--cuda-graph", "--synthetic",
           "--synthetic-len", "16", "--img-size", "128", "-e", "1", "-b", "4", "--out-dir", str(tmp_path)]
    env = dict(os.environ, DPA_DP_REPLICAS="2")           # two replicas on the box's one GPU
    r = subprocess.run(cmd, cwd=root, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    logs = "".join(p.read_text() for p in (tmp_path / "logs").glob("*.log"))
    assert "captured forward + backward graphs" in logs, logs[-2000:]
    assert list((tmp_path / "checkpoints").glob("*.pth"))


def test_train_step_loss_decreases(hip_lib):
    """A few optimizer steps on one synthetic batch reduce the loss (end-to-end engine sanity)."""
    from distributedpytorch_amd.config import TrainConfig
    from distributedpytorch_amd.models.unet import build_model
    from distributedpytorch_amd.trainer import SingleDevice
    torch.manual_seed(2)
    x, t = _batch(4, 64)
    st = SingleDevice(TrainConfig(backend="hip", lr=1e-3), build_model("unet"), "cuda:0")
    losses = [st.train_step(x, t).item() for _ in range(8)]
    assert losses[-1] < losses[0], losses


def test_graphed_step_matches_eager(hip_lib):
    """--cuda-graph: replaying the captured step (pack, fwd, loss, bwd, Adam) gives the eager
    trajectory, including an LR change between replays and an eager fallback batch."""
    from distributedpytorch_amd.config import TrainConfig
    from distributedpytorch_amd.models.unet import build_model
    from distributedpytorch_amd.trainer import GraphedStep, SingleDevice
    torch.manual_seed(4)
    a, b = build_model("unet"), build_model("unet")
    b.load_state_dict(a.state_dict())
    batches = [_batch(4, 64) for _ in range(3)]
    ea = SingleDevice(TrainConfig(backend="hip", lr=1e-3), a, "cuda:0")
    gb = SingleDevice(TrainConfig(backend="hip", lr=1e-3), b, "cuda:0")
    ea.optimizer.enable_device_state()
    g = GraphedStep(gb, *batches[0])
    la, lb = [], []
    for k in range(5):
        if k == 3:
            ea.optimizer.param_groups[0]["lr"] = gb.optimizer.param_groups[0]["lr"] = 3e-4
        x, t = batches[k % 3]
        la.append(ea.train_step(x, t))
        lb.append(g(x, t))
    xs, ts = _batch(2, 64)        # other shape -> eager step on the graphed strategy
    la.append(ea.train_step(xs, ts))
    assert not g.matches(xs, ts)
    lb.append(gb.train_step(xs, ts))
    torch.cuda.synchronize()
    assert gb.optimizer.step_count == ea.optimizer.step_count == 6
    for u, v in zip(la, lb):
        assert abs(u.item() - v.item()) <= 1e-5 * abs(u.item()), (la, lb)
    torch.testing.assert_close(gb.space.data, ea.space.data, rtol=1e-5, atol=1e-6)


def test_step_is_deterministic_and_debug_sync_invariant(hip_lib):
    """Race triage: the same step from the same state gives bitwise-identical gradients, with and
    without per-launch synchronisation (a stream-ordering race or an LDS race shows up here)."""
    from distributedpytorch_amd.ops._lib import set_debug_sync
    from distributedpytorch_amd.models.unet import build_model
    torch.manual_seed(5)
    model = build_model("unet").cuda()
    x, t = _batch(4, 64)
    grads = []
    for dbg in (False, False, True):
        set_debug_sync(dbg)
        try:
            _, g = _single(model, x, t)
        finally:
            set_debug_sync(False)
        grads.append(g)
    for n in grads[0]:
        assert torch.equal(grads[0][n], grads[1][n]), n
        assert torch.equal(grads[0][n], grads[2][n]), n


def test_native_dp_comm_single_device(hip_lib):
    """csrc/dp_comm.cpp on the one device a test box has: a one-member clique (ncclCommInitAll) whose
    grouped all-reduce (sum/avg) and broadcast are the identity, ordered on the current stream."""
    from distributedpytorch_amd.parallel import dp_comm
    assert dp_comm.available(), dp_comm.LIB_PATH
    assert dp_comm.lib().dpa_dp_version() > 0
    c = dp_comm.DPComm(["cuda:0"])
    x = torch.randn(1 << 20, device="cuda")
    ref = x.clone()
    c.all_reduce([x], "sum")
    c.all_reduce([x], "avg")
    b = torch.randn(4096, device="cuda").to(torch.bfloat16)
    bref = b.clone()
    c.broadcast([b], root=0)
    torch.cuda.synchronize()
    assert torch.equal(x, ref) and torch.equal(b, bref)
    with pytest.raises(AssertionError):
        c.all_reduce([x.cpu()])
    c.close()


@pytest.mark.parametrize("extra", [[], ["--infer"], ["--parallelism", "mp", "--stages", "2", "--microbatches", "2"]])
def test_bench_json_contract(hip_lib, extra):
    """bench.py prints ONE JSON line with the fields the round driver reads (metric, value, unit,
    n_gpus, steps, warmup, ms_per_step, higher_is_better, scaling, vs_baseline, dtype, data, config)."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--steps", "2", "--warmup", "1", "--batch", "4",
                        "--img", "128"] + extra, capture_output=True, text=True, timeout=300, cwd=root)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in out, k
    assert out["n_gpus"] == 1 and out["steps"] == 2 and out["warmup"] == 1 and out["dtype"] == "bf16"
    assert out["value"] > 0 and out["higher_is_better"] is True
    assert abs(out["value"] - 4 * 1000.0 / out["ms_per_step"]) < 0.02 * out["value"]
    assert out["config"]["global_batch"] == 4
    assert out["scaling"] == ("strong" if "mp" in extra else "weak")


@pytest.mark.parametrize("extra", [[], ["--grad-comm-dtype", "bf16"], ["--no-comm-overlap"],
                                   ["--parallelism", "mp", "--microbatches", "2"],
                                   # row-split top level (parallel/spatial_pipe.py) through bench.py
                                   ["--parallelism", "mp", "--microbatches", "2", "--mp-cut", "spatial"]])
def test_bench_two_ranks_same_device(hip_lib, extra):
    """Rehearsal of the multi-rank bench path on one GPU: torchrun with 2 ranks sharing cuda:0 over
    gloo (DPA_SAME_DEVICE=1) - DDP bucketed all-reduce of HIP-engine gradients, and GPipe send/recv of
    channels_last activations/skips (flattened in storage order on the wire)."""
    import json
    import os
    import socket
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, DPA_SAME_DEVICE="1", DPA_DIST_BACKEND="gloo")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(root, "bench.py"),
                        "--gpus", "2", "--steps", "2", "--warmup", "1", "--batch", "4", "--img", "128"] + extra,
                       capture_output=True, text=True, timeout=300, cwd=root, env=env)
    assert r.returncode == 0, (r.stdout[-1500:], r.stderr[-3000:])
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["value"] > 0
    mp_run = "mp" in extra
    assert out["config"]["global_batch"] == (4 if mp_run else 8)
    assert out["final_loss"] is not None and out["final_loss"] == out["final_loss"]
    assert out["rccl_world"]["world_size"] == 2 and out["rccl_world"]["backend"] == "gloo"
    rm = out["rank_ms_per_step"]
    assert len(rm["per_rank"]) == 2 and 0 < rm["min"] <= rm["max"]
    assert out["config"]["comm_overlap"] == ("--no-comm-overlap" not in extra)
    if "spatial" in extra:
        assert out["config"]["mp_plan"]["cut_mode"] == "spatial" and "spatial" in out["config"]["mp_cut"]
    if not mp_run:  # DDP: the reducer timed the stall on outstanding all-reduce buckets, on every rank
        assert out["exposed_comm_ms_last_step"] is not None and out["exposed_comm_ms_last_step"] >= 0
        assert 0 <= out["exposed_comm_ms"]["min"] <= out["exposed_comm_ms"]["max"]


def test_dp_bucket_reducer_native_clique(hip_lib):
    """-t DP's bucketed reducer on the native RCCL clique (one member here): buckets are launched
    on the comm stream while the HIP backward runs (readiness from notify_ready), the compute
    stream waits for them at the end, and a one-member sum leaves the gradients bitwise unchanged."""
    from distributedpytorch_amd.compute import make_compute
    from distributedpytorch_amd.models.unet import build_model
    from distributedpytorch_amd.optim import FlatParameterSpace
    from distributedpytorch_amd.parallel import dp_comm
    from distributedpytorch_amd.parallel.dp import DPBucketReducer
    torch.manual_seed(6)
    m = build_model("unet").cuda()
    sp = FlatParameterSpace(m)
    comp = make_compute(m, "hip", "bf16")
    x, t = _batch(4, 64)
    sp.zero_grad()
    from distributedpytorch_amd.compute import loss_from_partials
    (loss_from_partials(comp.forward_partials(x, t), t.numel()) * 4).backward()
    torch.cuda.synchronize()
    ref = sp.grad.clone()
    red = DPBucketReducer([sp], [torch.device("cuda:0")], dp_comm.DPComm(["cuda:0"]), bucket_mb=1.0)
    sp.zero_grad()
    (loss_from_partials(comp.forward_partials(x, t), t.numel()) * 4).backward()
    assert red.next_launch >= len(red.buckets) - 1     # launched during the backward
    red.finish()
    torch.cuda.synchronize()
    assert torch.equal(sp.grad, ref)
    assert red.exposed_comm_ms() >= 0


def _bench(extra, timeout=300):
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--steps", "3", "--warmup", "1"] + extra,
                       capture_output=True, text=True, timeout=timeout, cwd=root)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_dp1proc_replicas_share_one_gpu(hip_lib):
    """VERDICT r5 #3a: ``-t DP`` has a bench path (DPStrategy, one process, a host thread per replica); on one
    GPU its replicas share cuda:0 (host-issue rehearsal, Python-sum reduction instead of the RCCL clique)."""
    out = _bench(["--parallelism", "dp1proc", "--replicas", "2", "--batch", "4", "--img", "128"])
    assert out["config"]["parallelism"].startswith("dp1proc2") and out["config"]["global_batch"] == 8
    assert abs(out["value"] - 8 * 1000.0 / out["ms_per_step"]) < 0.02 * out["value"]
    d = out["dp1proc"]
    assert d["replicas"] == 2 and d["host_ms_per_step"] > 0 and d["device_ms_per_step_dev0"] > 0
    assert out["vs_baseline"] is None


def test_bench_comm_probe_reports_every_bucket(hip_lib):
    """VERDICT r5 #3c: the RCCL-bucket stand-in launched at each bucket-ready point of the backward
    (utils/comm_probe.py) reports its wait for CUs next to its idle time, for every DDP bucket."""
    out = _bench(["--batch", "8", "--img", "256", "--comm-probe", "--bucket-mb", "1"])
    cp = out["comm_probe"]
    assert cp["unlaunched"] == 0 and len(cp["buckets"]) >= 2
    for b in cp["buckets"]:
        assert b["total_us"] > 0 and b["run_us"] > 0 and b["idle"]["run_us"] > 0
        assert 0 <= b["ready_at_us"] <= cp["step_us"]
