"""CPU tests (no GPU): model spec, loss semantics, checkpoint layout, CLI, partitioner, and the
single-process strategies against a plain reference computation.

Reference behaviour cited: model/unet_parts.py, model/unet_model.py (UNet), utils/utils.py:9-25
(loss), utils/train_utils.py:88,163,244 (checkpoints), train.py:15-26 (flags), SURVEY §2.7.
"""
import os

import pytest
import torch
import torch.nn.functional as F

from distributedpytorch_amd.compute import loss_from_partials, loss_partials_from_probs, make_compute
from distributedpytorch_amd.config import parse_args
from distributedpytorch_amd.loss import Loss, bce_dice_from_probs, dice_score
from distributedpytorch_amd.models.blocks import boundary_names, partition
from distributedpytorch_amd.models.unet import build_model, count_params, forward_flops
from distributedpytorch_amd.optim import FlatParameterSpace, FusedAdam


REF_KEYS = (
    [f"encoder.conv{i}.conv_block.{j}.{t}" for i in range(1, 5) for j in (0, 2) for t in ("weight", "bias")]
    + [f"mid.conv_block.{j}.{t}" for j in (0, 2) for t in ("weight", "bias")]
    + [f"decoder.conv{i}.conv_block.{j}.{t}" for i in range(1, 5) for j in (0, 2) for t in ("weight", "bias")]
    + [f"decoder.deconv{i}.{t}" for i in range(1, 5) for t in ("weight", "bias")]
    + ["segmap.weight", "segmap.bias"])


def test_reference_model_spec():
    m = build_model("unet")
    assert count_params(m) == 7_760_097                      # model/modelsummary.txt:63
    sd = m.state_dict()
    assert len(sd) == 46 and set(sd) == set(REF_KEYS)
    assert tuple(sd["decoder.deconv1.weight"].shape) == (512, 256, 2, 2)
    assert tuple(sd["segmap.weight"].shape) == (1, 32, 1, 1)
    assert len(list(m.buffers())) == 0
    # FLOPs per image from SURVEY §2.7
    assert abs(forward_flops(m.cfg, 512, 512) / 1e9 - 96.6) < 0.5
    assert abs(forward_flops(m.cfg, 640, 960) / 1e9 - 226.3) < 1.0


def test_forward_shape_and_range():
    m = build_model("unet")
    with torch.no_grad():
        y = m(torch.rand(1, 3, 64, 96))
    assert tuple(y.shape) == (1, 1, 64, 96) and 0 <= y.min() and y.max() <= 1


def test_loss_semantics():
    torch.manual_seed(0)
    p = torch.rand(2, 1, 8, 8).clamp(0.01, 0.99)
    t = (torch.rand(2, 1, 8, 8) > 0.5).float()
    bce = F.binary_cross_entropy(p, t)
    dice = 2 * (p * t).sum() / (p.sum() + t.sum() + 1e-15)    # global over the batch (utils.py:17-23)
    assert torch.allclose(Loss()(p, t), bce - torch.log(dice))
    assert torch.allclose(Loss(dice_weight=5)(p, t), bce - torch.log(dice))   # weight is a toggle (A12)
    assert torch.allclose(Loss(dice_weight=0)(p, t), bce)
    S = loss_partials_from_probs(p, t)
    assert torch.allclose(loss_from_partials(S, t.numel()), bce_dice_from_probs(p, t))
    # partial sums compose over a split batch (pipeline/DP combine rule)
    S2 = loss_partials_from_probs(p[:1], t[:1]) + loss_partials_from_probs(p[1:], t[1:])
    assert torch.allclose(loss_from_partials(S2, t.numel()), bce_dice_from_probs(p, t), atol=1e-6)
    assert 0.0 <= dice_score(p, t).item() <= 1.0


def test_cli_reference_flags():
    cfg = parse_args(["-t", "DDP", "-v", "20", "-e", "3", "--lr", "2e-4", "-b", "2", "-c", "DDP", "-s", "7"])
    assert (cfg.train_method, cfg.val, cfg.epochs, cfg.lr, cfg.batch_size, cfg.checkpoint, cfg.seed) == \
        ("DDP", 20.0, 3, 2e-4, 2, "DDP", 7)
    d = parse_args([])
    assert (d.train_method, d.val, d.epochs, d.lr, d.batch_size, d.seed) == ("singleGPU", 10.0, 10, 1e-4, 4, 42)
    with pytest.raises(SystemExit):
        parse_args(["-t", "bogus"])


def test_partition_reference_and_balanced():
    cfg = build_model("unet").cfg
    assert partition(cfg, 2, mode="reference") == [0, 5, 10]        # encoder+mid | decoder+head
    cuts = partition(cfg, 4, 512, 512)
    assert cuts[0] == 0 and cuts[-1] == 10 and len(cuts) == 5 and cuts == sorted(cuts)
    # reference cut carries the bottleneck + 4 skips (unet_model.py:36-37)
    assert boundary_names(5, 4) == ["x", "skip0", "skip1", "skip2", "skip3"]


def test_checkpoint_layout_roundtrip(tmp_path):
    from distributedpytorch_amd.utils import load_model_state, save_model
    m = build_model("unet-tiny")
    p = save_model(m, str(tmp_path / "checkpoints" / "DDP.pth"), module_prefix=True)
    sd = torch.load(p, weights_only=True)
    assert all(k.startswith("module.") for k in sd)
    m2 = build_model("unet-tiny")
    load_model_state(m2, p)                       # prefix tolerant
    for a, b in zip(m.state_dict().values(), m2.state_dict().values()):
        assert torch.equal(a, b)


def _ref_grads(model, x, t):
    (x.shape[0] * bce_dice_from_probs(model(x), t)).backward()
    return {n: p.grad.detach().clone() for n, p in model.named_parameters()}


def _ref_step(model, x, t, lr=1e-3):
    opt = torch.optim.Adam(model.parameters(), lr=lr, weight_decay=1e-8)
    loss = bce_dice_from_probs(model(x), t)
    (x.shape[0] * loss).backward()
    opt.step()
    return loss.detach()


def test_single_device_strategy_matches_reference_step():
    from distributedpytorch_amd.config import TrainConfig
    from distributedpytorch_amd.trainer import SingleDevice
    torch.manual_seed(0)
    a, b = build_model("unet-tiny"), build_model("unet-tiny")
    b.load_state_dict(a.state_dict())
    x = torch.rand(2, 3, 32, 32)
    t = (torch.rand(2, 1, 32, 32) > 0.5).float()
    cfg = TrainConfig(backend="torch", lr=1e-3, dtype="fp32")
    st = SingleDevice(cfg, a, "cpu")
    l1 = st.train_step(x, t)
    l2 = _ref_step(b, x, t)
    assert torch.allclose(l1, l2, atol=1e-6)
    for (n, p), (_, q) in zip(a.named_parameters(), b.named_parameters()):
        assert torch.allclose(p, q, atol=1e-6), n


def test_dp_strategy_cpu_matches_full_batch():
    """-t DP semantics: loss (incl. global Dice) over the whole batch, grads summed over replicas."""
    from distributedpytorch_amd.config import TrainConfig
    from distributedpytorch_amd.trainer import DPStrategy
    torch.manual_seed(1)
    a, b = build_model("unet-tiny"), build_model("unet-tiny")
    b.load_state_dict(a.state_dict())
    x = torch.rand(4, 3, 32, 32)
    t = (torch.rand(4, 1, 32, 32) > 0.5).float()
    st = DPStrategy(TrainConfig(backend="torch", lr=1e-3, dtype="fp32"), a, ["cpu", "cpu"])
    l1 = st.train_step(x, t)
    l2 = _ref_step(b, x, t)
    assert torch.allclose(l1, l2, atol=1e-6)
    for (n, p), (_, q) in zip(st.model.named_parameters(), b.named_parameters()):
        assert torch.allclose(p, q, atol=1e-5), n
    # replicas identical after the step
    for p, q in zip(st.dp.replicas[0].parameters(), st.dp.replicas[1].parameters()):
        assert torch.equal(p, q)


@pytest.mark.parametrize("n_img", [1, 2])
def test_dp_batch_smaller_than_replicas(n_img):
    """torch.nn.DataParallel semantics for a short batch (a last or validation batch of fewer images than
    replicas): only the first replicas get images, the idle replicas' zero gradients join the bucketed sum,
    and the step equals the full-batch reference; eval probabilities cover the batch."""
    from distributedpytorch_amd.config import TrainConfig
    from distributedpytorch_amd.trainer import DPStrategy
    torch.manual_seed(3)
    a, b = build_model("unet-tiny"), build_model("unet-tiny")
    b.load_state_dict(a.state_dict())
    x = torch.rand(n_img, 3, 32, 32)
    t = (torch.rand(n_img, 1, 32, 32) > 0.5).float()
    st = DPStrategy(TrainConfig(backend="torch", lr=1e-3, dtype="fp32", bucket_mb=0.002), a, ["cpu"] * 3)
    l1 = st.train_step(x, t)
    l2 = _ref_step(b, x, t)
    assert torch.allclose(l1, l2, atol=1e-6)
    for (n, p), (_, q) in zip(st.model.named_parameters(), b.named_parameters()):
        assert torch.allclose(p, q, atol=1e-5), n
    for r in st.dp.replicas[1:]:
        for p, q in zip(st.dp.replicas[0].parameters(), r.parameters()):
            assert torch.equal(p, q)
    assert st.dp.probs(x).shape[0] == n_img


@pytest.mark.parametrize("stages,mb", [(2, 2), (3, 4)])
def test_local_pipeline_matches_plain_forward(stages, mb):
    """Reference probe7: pipelined forward == plain forward, grads agree."""
    from distributedpytorch_amd.parallel.pipeline import GPipeLocal
    torch.manual_seed(2)
    a, b = build_model("unet-tiny"), build_model("unet-tiny")
    b.load_state_dict(a.state_dict())
    x = torch.rand(4, 3, 32, 32)
    t = (torch.rand(4, 1, 32, 32) > 0.5).float()
    pipe = GPipeLocal(a, ["cpu"] * stages, mb, backend="torch", dtype="fp32", img_hw=(32, 32),
                      mode="reference" if stages == 2 else "balanced")
    loss = pipe.forward_loss(x, t)
    loss.backward()
    ref = bce_dice_from_probs(b(x), t)
    ref.backward()
    assert torch.allclose(loss, ref, atol=1e-6)
    for (n, p), (_, q) in zip(a.named_parameters(), b.named_parameters()):
        assert torch.allclose(p.grad, q.grad, atol=1e-6), n
    with torch.no_grad():
        assert torch.allclose(pipe.probs(x), b(x), atol=1e-6)


def test_flat_space_ready_notifications():
    m = build_model("unet-tiny")
    space = FlatParameterSpace(m)
    seen = []
    space.add_ready_listener(seen.append)
    space.notify_ready([m.segmap.weight, m.segmap.bias])
    assert seen == [space.index_of(m.segmap.weight), space.index_of(m.segmap.bias)]
    v = space.version
    FusedAdam(space, lr=1e-3).step()
    assert space.version == v + 1


def test_trainer_end_to_end_outputs(tmp_path):
    """python train.py -t singleGPU on synthetic data writes the reference artefacts."""
    import pandas as pd
    from distributedpytorch_amd.trainer import train
    cfg = parse_args(["-e", "2", "-b", "4", "--synthetic", "--synthetic-len", "24", "--img-size", "32",
                      "--model", "unet-tiny", "--backend", "torch", "--dtype", "fp32", "--out-dir", str(tmp_path),
                      "--log-every", "2"])
    out = train(cfg)
    assert os.path.exists(tmp_path / "checkpoints" / "singleGPU.pth")
    tl = pd.read_pickle(tmp_path / "loss" / "singleGPU" / "train_loss.pkl")   # our own file
    vl = pd.read_pickle(tmp_path / "loss" / "singleGPU" / "val_loss.pkl")
    assert list(tl.columns) == ["Step", "Time", "Loss"] and len(vl) == 2
    assert out["step"] > 0
    # resume continues from the saved epoch
    cfg2 = parse_args(["-e", "3", "-b", "4", "--synthetic", "--synthetic-len", "24", "--img-size", "32",
                       "--model", "unet-tiny", "--backend", "torch", "--dtype", "fp32", "--out-dir", str(tmp_path),
                       "--resume"])
    out2 = train(cfg2)
    assert out2["step"] > out["step"]


def test_variant_presets_layout():
    """BN / bilinear variants (north-star DoubleConv = Conv2d+BN+ReLU, bilinear Up): torch key layout
    (``conv_block.{0,1,3,4}``, ``deconvN.proj``), running-stat buffers, shapes."""
    m = build_model("unet-bn-bilinear")
    sd = m.state_dict()
    assert "encoder.conv1.conv_block.1.running_mean" in sd and "encoder.conv1.conv_block.3.weight" in sd
    assert tuple(sd["decoder.deconv1.proj.weight"].shape) == (256, 512, 1, 1)
    assert len(list(m.buffers())) == 3 * 18
    with torch.no_grad():
        assert tuple(m(torch.rand(2, 3, 32, 48)).shape) == (2, 1, 32, 48)


def test_local_pipeline_bn_variant_one_microbatch():
    """BN running statistics live on their stage's device; with one microbatch the pipelined step
    equals the plain model exactly (batch statistics over the same images)."""
    from distributedpytorch_amd.parallel.pipeline import GPipeLocal
    torch.manual_seed(4)
    a, b = build_model("unet-tiny-bn"), build_model("unet-tiny-bn")
    b.load_state_dict(a.state_dict())
    x = torch.rand(4, 3, 32, 32)
    t = (torch.rand(4, 1, 32, 32) > 0.5).float()
    pipe = GPipeLocal(a, ["cpu"] * 2, 1, backend="torch", dtype="fp32", img_hw=(32, 32), mode="reference")
    loss = pipe.forward_loss(x, t)
    loss.backward()
    ref = bce_dice_from_probs(b(x), t)
    ref.backward()
    assert torch.allclose(loss, ref, atol=1e-6)
    for (n, p), (_, q) in zip(a.named_parameters(), b.named_parameters()):
        assert torch.allclose(p.grad, q.grad, atol=1e-5), n
    for (n, p), (_, q) in zip(a.named_buffers(), b.named_buffers()):
        assert torch.allclose(p.float(), q.float(), atol=1e-6), n
    a.eval()
    b.eval()
    with torch.no_grad():
        assert torch.allclose(pipe.probs(x), b(x), atol=1e-5)


def test_trainer_bn_variant_eval_mode(tmp_path):
    """Evaluation runs in eval mode (running statistics) and training resumes in train mode."""
    from distributedpytorch_amd.trainer import train
    cfg = parse_args(["-e", "1", "-b", "4", "--synthetic", "--synthetic-len", "16", "--img-size", "32",
                      "--model", "unet-tiny-bn", "--backend", "torch", "--dtype", "fp32", "--out-dir", str(tmp_path)])
    out = train(cfg)
    m = out["strategy"].model
    assert m.training
    sd = torch.load(tmp_path / "checkpoints" / "singleGPU.pth", weights_only=True)
    assert int(sd["encoder.conv1.conv_block.1.num_batches_tracked"]) == out["step"]


def test_dp_buckets_launch_during_backward():
    """-t DP gradient sum is bucketed and driven by readiness: with small buckets most of them are
    summed before the backward returns; the result equals the one-shot sum."""
    from distributedpytorch_amd.config import TrainConfig
    from distributedpytorch_amd.trainer import DPStrategy
    torch.manual_seed(3)
    a, b = build_model("unet-tiny"), build_model("unet-tiny")
    b.load_state_dict(a.state_dict())
    x = torch.rand(4, 3, 32, 32)
    t = (torch.rand(4, 1, 32, 32) > 0.5).float()
    st = DPStrategy(TrainConfig(backend="torch", lr=1e-3, dtype="fp32", bucket_mb=0.002), a, ["cpu", "cpu"])
    red = st.dp.reducer
    assert len(red.buckets) > 3
    st.optimizer.zero_grad()
    (st.dp.forward_loss(x, t) * 4).backward()
    launched = red.next_launch
    assert launched >= len(red.buckets) - 1, (launched, len(red.buckets))
    assert not any(fin for _, _, fin in red.launch_log), red.launch_log
    st.dp.all_reduce_grads()
    assert red.next_launch == 0          # reset for the next step
    ref = _ref_grads(b, x, t)
    for n, p in st.model.named_parameters():
        assert torch.allclose(p.grad, ref[n], atol=1e-6), n
    for sp in st.dp.spaces[1:]:
        assert torch.equal(sp.grad, st.dp.spaces[0].grad)


def test_unet_pipe_constructor_matches_plain():
    """Reference API ``UNet(pipe=True)`` (unet_model.py:5,14-53): same state-dict keys, the
    2-microbatch pipelined forward equals the plain forward, gradients agree."""
    from distributedpytorch_amd.models.unet import UNet
    torch.manual_seed(5)
    a = UNet(pipe=True, base=8, depth=2)
    b = UNet(base=8, depth=2)
    b.load_state_dict(a.state_dict())
    assert list(a.state_dict()) == list(b.state_dict())
    x = torch.rand(4, 3, 32, 32)
    pa, pb = a(x), b(x)
    assert torch.equal(pa, pb)
    pa.sum().backward()
    pb.sum().backward()
    for (n, p), q in zip(a.named_parameters(), b.parameters()):
        torch.testing.assert_close(p.grad, q.grad, rtol=1e-4, atol=1e-5, msg=n)


def test_reducers_reject_double_announcement():
    """A gradient announced twice in one step (autograd hook AND notify_ready) is an error, not a
    silently stalled bucket (both reducers)."""
    import pytest
    from distributedpytorch_amd.optim import FlatParameterSpace
    from distributedpytorch_amd.parallel.dp import DPBucketReducer
    m = build_model("unet-tiny")
    sp = FlatParameterSpace(m)
    red = DPBucketReducer([sp], ["cpu"], None, bucket_mb=0.002)
    red.mark_ready(0)
    with pytest.raises(AssertionError, match="announced twice"):
        red.mark_ready(0)


def test_dp_single_reduction_opt_out():
    """--no-comm-overlap: one reduction of the whole buffer at the end of the backward, same result."""
    from distributedpytorch_amd.config import TrainConfig
    from distributedpytorch_amd.trainer import DPStrategy
    torch.manual_seed(3)
    a, b = build_model("unet-tiny"), build_model("unet-tiny")
    b.load_state_dict(a.state_dict())
    x = torch.rand(4, 3, 32, 32)
    t = (torch.rand(4, 1, 32, 32) > 0.5).float()
    st = DPStrategy(TrainConfig(backend="torch", lr=1e-3, dtype="fp32", bucket_mb=0.002, comm_overlap=False),
                    a, ["cpu", "cpu"])
    red = st.dp.reducer
    assert len(red.buckets) == 1
    st.optimizer.zero_grad()
    (st.dp.forward_loss(x, t) * 4).backward()
    assert red.next_launch == 0 and red.launch_log == []
    st.dp.all_reduce_grads()
    assert red.last_launch_log == [(0, 2 * len(st.dp.spaces[0].names), True)]
    ref = _ref_grads(b, x, t)
    for n, p in st.model.named_parameters():
        assert torch.allclose(p.grad, ref[n], atol=1e-6), n
