"""GPipe pipeline model parallelism for the UNet (``-t MP``).

Reference: a hand-written 2-stage, 2-microbatch pipeline inside ``UNet.forward``
(``model/unet_model.py:14-53``): encoder+mid on cuda:0, decoder+head on
cuda:1, the bottleneck and all four skips copied with ``.to('cuda:1')`` per microbatch, overlap
only from async launch order, backward via plain autograd.

Here, generalised to N stages x M microbatches (GPipe: all forwards, then all backwards) over a
:class:`.placement.Placement`: the reference's encoder|decoder cut (``--mp-cut reference``), any
contiguous partition, or the mirrored V placement in which stage s owns encoder level(s) s on the way
down and the same decoder level(s) on the way up, so skips never leave their GPU and each stage has
two segments (half the fill / drain bubble).  The reference cut moves 31 MiB per image across one
xGMI link at 512^2 bf16 (all four skips), which makes it link-bound (parallel/schedule.py);
the V placement moves 6 MiB.

* :class:`GPipeDist` - one process per GPU (torchrun), the MI355X-native form.  Activations AND skip
  tensors go *directly* from producer to consumer segment with RCCL ``isend/irecv`` (one xGMI hop on
  the fully connected MI355X mesh), in the compute dtype (bf16: half the reference's bytes), on one
  communicator per sending segment; every receive of a phase is posted before its first op computes,
  so transfers overlap compute.  The head stage sums the per-microbatch loss partial sums, which gives
  exactly the reference's full-batch loss (global Dice), then back-propagates op by op so gradients
  start flowing upstream immediately.
* :class:`GPipeLocal` - single process, N local devices (the reference's own form, kept for
  ``python train.py -t MP`` without torchrun): segments issued in wavefront order; cross-device
  copies are peer copies.

Both are numerically transparent: pipelined forward == plain forward (SURVEY §3.4 probe7), checked
by the tests against a single-device run.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

import torch
import torch.distributed as dist

from ..compute import loss_from_partials, make_blocks
from ..models.blocks import block_kind, partition, run_segment, segment_units, skip_name
from ..optim import FlatParameterSpace
from ..utils.tracing import trace_range
from .placement import Placement, channel_members, flop_orders, remote_groups, seg_io
from .placement import stage_io as _stage_io


def _debug_point(device):
    """Debug-sync mode (``--debug-sync``): drain the device after every stage op so a
    stream-ordering race between compute and the send/recv streams shows up at its source."""
    from ..ops._lib import debug_sync
    if debug_sync() and device is not None and torch.device(device).type == "cuda":
        torch.cuda.synchronize(device)


def _block_param_prefixes(idx: int, depth: int) -> List[str]:
    kind, i = block_kind(idx, depth)
    if kind == "enc":
        return [f"encoder.conv{i + 1}."]
    if kind == "mid":
        return ["mid."]
    if kind == "dec":
        return [f"decoder.conv{i + 1}.", f"decoder.deconv{i + 1}."]
    return ["segmap."]


def _unit_param_prefixes(model, idx: int, part: str) -> List[str]:
    """Parameter-name prefixes of block ``idx`` or of one of its halves (``a``: the first conv [+BN],
    and the transposed conv of a decoder block; ``b``: the second conv [+BN])."""
    depth = model.cfg.depth
    prefixes = _block_param_prefixes(idx, depth)
    if part == "full":
        return prefixes
    kind, i = block_kind(idx, depth)
    blk = {"enc": lambda: model.encoder.blocks()[i], "mid": lambda: model.mid,
           "dec": lambda: model.decoder.blocks()[i]}[kind]()
    n = len(blk.conv_block) // 2
    layers = range(n) if part == "a" else range(n, 2 * n)
    out = [f"{prefixes[0]}conv_block.{k}." for k in layers]
    if kind == "dec" and part == "a":
        out.append(prefixes[1])              # decoder.deconv{i+1}.
    return out


def _segment_prefixes(model, start: float, end: float) -> List[str]:
    return [p for idx, part in segment_units(start, end, model.cfg.depth) for p in _unit_param_prefixes(model, idx, part)]


def stage_param_names(model, start: float, end: float) -> List[str]:
    prefixes = _segment_prefixes(model, start, end)
    return [n for n, _ in model.named_parameters() if any(n.startswith(p) for p in prefixes)]


def stage_buffer_names(model, start: float, end: float) -> List[str]:
    """Buffers (BatchNorm running statistics) of the blocks in ``[start, end)``."""
    prefixes = _segment_prefixes(model, start, end)
    return [n for n, _ in model.named_buffers() if any(n.startswith(p) for p in prefixes)]


def placement_param_names(model, pl: Placement, stage: int) -> List[str]:
    """Parameters of every segment stage ``stage`` owns under placement ``pl``."""
    out = []
    for j in pl.segments(stage):
        out += stage_param_names(model, *pl.seg_range(j))
    return out


def placement_buffer_names(model, pl: Placement, stage: int) -> List[str]:
    out = []
    for j in pl.segments(stage):
        out += stage_buffer_names(model, *pl.seg_range(j))
    return out


def stage_io(cuts, depth: int):
    """Per stage: ``recv`` list of (name, src_stage) and ``send`` list of (name, dst_stage) for a
    contiguous cut list or a :class:`.placement.Placement`."""
    pl = cuts if isinstance(cuts, Placement) else Placement.contiguous(cuts)
    return _stage_io(pl, depth)


def infer_shapes(cfg, microbatch: int, h: int, w: int) -> Dict[str, tuple]:
    """Shapes (NCHW) of every skip tensor for one microbatch, by arithmetic (no tracing)."""
    shapes = {}
    H, W = h, w
    for lvl, wd in enumerate(cfg.widths):
        shapes[skip_name(lvl)] = (microbatch, wd, H, W)
        H, W = H // 2, W // 2
    return shapes


class _Capture(torch.autograd.Function):
    """Boundary of a segment's input: forward is the identity (same storage, so the HIP engine still
    finds a skip's concat buffer by address), backward stores the incoming gradient under ``key`` in
    ``box`` as produced -- no ``AccumulateGrad`` on a detached leaf, which would copy a strided
    skip gradient (a 64-of-128-channel view of the decoder's dgrad output) into a fresh dense ``.grad``."""

    @staticmethod
    def forward(ctx, anchor, t, box, key):
        ctx.box, ctx.key = box, key
        return t.detach()

    @staticmethod
    def backward(ctx, g):
        ctx.box[ctx.key] = g
        return None, None, None, None


class GPipeDist:
    """Multi-process GPipe over a process group whose size == number of stages, on any
    :class:`.placement.Placement` (contiguous block ranges, or the mirrored V placement where stage s
    owns encoder levels on the way down and the same decoder levels on the way up).

    Communication (RCCL over xGMI, or gloo on CPU):
    * one communicator PER SEGMENT (:func:`.placement.channel_members`): segment j's owner is its only
      sender (activations to the stages of j's consumer segments, gradients to the stages of j's
      producer segments); a rank receives a segment's messages only on that segment's communicator.
      torch puts every P2P op of a group on that group's single RCCL stream in issue order, so no send
      can ever queue behind the same rank's pre-posted receive (``tests/test_pipeline_p2p_order.py``),
      and each (segment, stage) message stream is matched in microbatch order;
    * the tensors one op sends to one stage go as ONE ``batch_isend_irecv`` group (x and skips
      together); a skip goes straight from its encoder segment to its decoder segment (one hop);
      segments of one stage hand tensors over locally (no copy);
    * every receive of the step is posted before the first op computes (forward: at the start;
      backward: when the loss is known), so transfers land while earlier ops compute;
    * each stage issues its ops in the static order of :func:`.placement.stage_orders` (the list
      scheduler of the schedule model; a plan can carry the order it simulated);
    * every communicator is created at construction (a 1-element exchange from its sender to every
      member), so the lazy RCCL setup never lands inside a training step;
    * a skip that leaves this stage is written by the encoder conv into a dense tensor (HIP engine
      ``dense_skips``) and sent as is; activations travel in the compute dtype (bf16).
    """

    def __init__(self, model, microbatches: int, backend: str = "auto", dtype: str = "bf16",
                 group=None, cuts: Optional[List[float]] = None, img_hw=(512, 512), mode: str = "balanced",
                 warm: bool = True, placement: Optional[Placement] = None, policy: str = "feed",
                 orders: Optional[List[dict]] = None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.S = dist.get_world_size(group)
        self.M = microbatches
        self.model = model
        self.depth = model.cfg.depth
        if placement is None:
            placement = Placement.contiguous(cuts or partition(model.cfg, self.S, img_hw[0], img_hw[1], mode=mode))
        self.pl = placement.validate(self.depth)
        assert self.pl.S == self.S, f"placement has {self.pl.S} stages, the group {self.S} ranks"
        self.cuts = list(self.pl.cuts)
        self.segs = self.pl.segments(self.rank)
        self.ins, self.outs = seg_io(self.pl, self.depth)
        self.recv_spec, self.send_spec = _stage_io(self.pl, self.depth)
        self.device = next(model.parameters()).device
        names = set(placement_param_names(model, self.pl, self.rank))
        own = [(n, p) for n, p in model.named_parameters() if n in names]
        for n, p in model.named_parameters():
            if n not in names:
                p.requires_grad_(False)
        self.space = FlatParameterSpace(own, device=self.device)
        self.blocks = make_blocks(model, backend, dtype)
        # microbatches: one weight-gradient launch per layer per step (HIP engine, see HipBlocks)
        if hasattr(self.blocks, "defer_wgrad"):
            self.blocks.defer_wgrad = microbatches
        if hasattr(self.blocks, "dense_skips"):
            self.blocks.dense_skips = {int(n[len("skip"):]) for n, _ in self.send_spec[self.rank]
                                       if n.startswith("skip")}
        self.comm_dtype = torch.bfloat16 if (dtype == "bf16" and self.device.type == "cuda") else torch.float32
        self.first_rank = self.pl.owner[0]
        self.head_rank = self.pl.owner[self.pl.head_seg]
        self.is_first = self.rank == self.first_rank
        self.is_last = self.rank == self.head_rank
        self.policy = policy
        h, w = img_hw
        self.orders = (orders or flop_orders(self.pl, model.cfg, microbatches, h, w, policy))[self.rank]
        assert sorted(self.orders["fwd"]) == sorted(j for j in self.segs for _ in range(microbatches))
        self._glob = lambda s: dist.get_global_rank(group, s) if group is not None else s
        self._host_staged = self.device.type == "cuda" and dist.get_backend(group) != "nccl"
        self._anchor = torch.zeros((), device=self.device, requires_grad=True)
        # one communicator per segment with a remote edge; its owner is the only sender
        self.members = channel_members(self.pl, self.depth)
        self.groups: Dict[int, object] = {}
        world_pipeline = group is None or dist.get_world_size(group) == dist.get_world_size()
        for j in range(self.pl.K):
            ranks = [self._glob(r) for r in self.members[j]]
            if len(ranks) < 2:
                continue
            if world_pipeline:      # every rank of the job calls new_group, members or not
                g = dist.new_group(ranks)
            elif self.rank in self.members[j]:   # pipeline inside a bigger job: members only, in order
                g = dist.new_group(ranks, use_local_synchronization=True)
            else:
                continue
            if self.rank in self.members[j]:
                self.groups[j] = g
        # messages: per segment, its remote edges grouped by the other end's stage
        self.fwd_msgs = [remote_groups(self.pl, self.outs[j], self.pl.owner[j]) for j in range(self.pl.K)]
        self.bwd_msgs = [remote_groups(self.pl, self.ins[j], self.pl.owner[j]) for j in range(self.pl.K)]
        self.op_log: Optional[list] = None   # tests: [(segment channel, "send"/"recv", peer stage)] per posted op
        if warm:
            self.warm_up()

    def warm_up(self):
        """One tiny exchange on every communicator this stage belongs to (its sender to each member), in
        segment order on every rank: creates the RCCL communicators now instead of inside the first
        timed step, and every group's first operation involves all of its members."""
        dev = "cpu" if self._host_staged else self.device
        for j in sorted(self.groups):
            g = self.groups[j]
            sender = self.pl.owner[j]
            others = [r for r in self.members[j] if r != sender]
            keep = []
            if sender == self.rank:
                out = torch.full((1,), float(j), dtype=self.comm_dtype, device=dev)
                keep.append(out)
                ops = [dist.P2POp(dist.isend, out, self._glob(r), g) for r in others]
            else:
                inp = torch.empty(1, dtype=self.comm_dtype, device=dev)
                keep.append(inp)
                ops = [dist.P2POp(dist.irecv, inp, self._glob(sender), g)]
            for wk in dist.batch_isend_irecv(ops):
                wk.wait()
            if sender != self.rank:
                assert int(keep[0].float().item()) == j, f"stage {self.rank}: channel {j} answered {keep[0].item()}"

    # shapes of the boundary tensors for this microbatch size
    def _shape(self, name, mb, h, w, cut):
        """Logical NCHW shape of tensor ``name`` entering the segment that starts at ``cut``."""
        cfg = self.model.cfg
        if name.startswith("skip"):
            return infer_shapes(cfg, mb, h, w)[name]
        kind, i = block_kind(int(cut), self.depth)
        hb, wb = h >> self.depth, w >> self.depth
        if cut != int(cut):          # a cut inside a DoubleConv: x is its first conv's output
            if kind == "enc":
                return (mb, cfg.widths[i], h >> i, w >> i)
            if kind == "mid":
                return (mb, cfg.mid_width, hb, wb)
            return (mb, cfg.widths[self.depth - 1 - i], hb << (i + 1), wb << (i + 1))
        if kind == "enc":
            return (mb, cfg.widths[i - 1], h >> i, w >> i)
        if kind == "mid":
            return (mb, cfg.widths[-1], hb, wb)
        if kind == "dec":
            c = cfg.mid_width if i == 0 else cfg.widths[self.depth - i]
            return (mb, c, hb << i, wb << i)
        return (mb, cfg.base, hb << self.depth, wb << self.depth)

    def _recv_layout(self):
        """channels_last on GPU (matches what the backends produce)."""
        return torch.channels_last if self.device.type == "cuda" else torch.contiguous_format

    def _empty_wire(self, shape):
        """(tensor, flat): a logical-NCHW receive buffer in the stage layout and the 1-D contiguous
        view of its storage that goes on the wire (gloo and RCCL both take a dense 1-D buffer; a
        channels_last 4-D tensor is rejected by gloo as non-contiguous)."""
        n, c, hh, ww = shape
        flat = torch.empty(n * c * hh * ww, dtype=self.comm_dtype, device=self.device)
        if self._recv_layout() == torch.channels_last:
            return flat.view(n, hh, ww, c).permute(0, 3, 1, 2), flat
        return flat.view(n, c, hh, ww), flat

    def _wire(self, t):
        """Send side: ``t`` in the stage layout, flattened in storage order (a view when dense)."""
        t = t.detach().to(self.comm_dtype).contiguous(memory_format=self._recv_layout())
        if self._recv_layout() == torch.channels_last:
            return t.permute(0, 2, 3, 1).reshape(-1)
        return t.reshape(-1)

    def _post(self, sends=(), recvs=(), channel: int = None):
        """One grouped P2P launch on segment ``channel``'s communicator: ``sends`` = [(tensor, dst
        stage)] (this rank owns the segment), or ``recvs`` = [(flat buffer, src stage)] (the segment's
        owner sends).  Returns a :class:`_Transfer` whose ``wait()`` completes it.

        RCCL moves device memory directly (ordered after the producing kernels on the current
        stream).  gloo (CPU tests; the one-GPU rehearsal of this path, ranks sharing cuda:0) is
        host-staged explicitly: a device buffer is copied to host memory before the send and from
        it after the receive completes."""
        g = self.groups[channel]
        ops, keep, copies = [], [], []
        for t, dst in sends:
            buf = self._wire(t)
            if self._host_staged:
                buf = buf.to("cpu")                   # synchronous: the producing kernels have finished
            keep.append(buf)
            ops.append(dist.P2POp(dist.isend, buf, self._glob(dst), g))
            self._log(channel, "send", dst)
        for flat, src in recvs:
            if self._host_staged:
                host = torch.empty(flat.shape, dtype=flat.dtype)
                copies.append((host, flat))
                flat = host
            ops.append(dist.P2POp(dist.irecv, flat, self._glob(src), g))
            self._log(channel, "recv", src)
        return _Transfer(dist.batch_isend_irecv(ops) if ops else [], keep, copies)

    def _log(self, channel: int, kind: str, peer: int):
        if self.op_log is not None:
            self.op_log.append((channel, kind, peer))

    def _cap(self, t, box, key):
        # detached: the producer's graph (another segment of this stage) must not be reached from here
        return _Capture.apply(self._anchor, t.detach(), box, key)

    def train_step(self, images: Optional[torch.Tensor], targets: Optional[torch.Tensor], batch: int,
                   hw, dice: bool = True, loss_scale: float = 1.0):
        """One GPipe step. Returns the (full-batch) loss on the head stage, None elsewhere."""
        h, w = hw
        M, pl, me = self.M, self.pl, self.rank
        assert batch % M == 0, f"batch {batch} must be divisible by microbatches {M}"
        mb = batch // M
        head = pl.head_seg
        xs = images.chunk(M) if self.is_first else None
        ts = targets.chunk(M) if self.is_last else None
        # every forward receive of the step: message (producer segment p, microbatch m) to this stage
        frx = {}
        for p in range(pl.K):
            edges = self.fwd_msgs[p].get(me)
            if not edges:
                continue
            for m in range(M):
                bufs, recvs = {}, []
                for name, c in edges:
                    t, flat = self._empty_wire(self._shape(name, mb, h, w, pl.cuts[c]))
                    bufs[name] = t
                    recvs.append((flat, pl.owner[p]))
                frx[(p, m)] = (bufs, self._post(recvs=recvs, channel=p))
        caps: Dict[tuple, Optional[torch.Tensor]] = {}      # (consumer segment, m, name) -> input gradient
        fout: Dict[tuple, Dict[str, torch.Tensor]] = {}      # (segment, m) -> its outputs
        partials: List[Optional[torch.Tensor]] = [None] * M
        pending = []
        nxt = {j: 0 for j in self.segs}
        for j in self.orders["fwd"]:
            m = nxt[j]
            nxt[j] += 1
            env = {}
            for name, p in self.ins[j]:
                if pl.owner[p] == me:
                    t = fout[(p, m)][name]
                else:
                    bufs, xfer = frx[(p, m)]
                    xfer.wait()
                    t = bufs[name]
                env[name] = self._cap(t, caps, (j, m, name))
            if j == 0:
                env["x"] = xs[m]
            a, b = pl.seg_range(j)
            # a skip leaving this stage is sent the moment its encoder level finishes, while
            # the deeper levels compute; per destination the tensors go in the message's (sorted) order,
            # which is the production order (skips by level, x last), so the receiver's one grouped
            # receive matches the sender's separate sends
            sent = {d: 0 for d in self.fwd_msgs[j]}

            def emit(name, t, j=j):
                for d, edges in self.fwd_msgs[j].items():
                    k = sent[d]
                    if k < len(edges) and edges[k][0] == name:
                        pending.append(self._post(sends=[(t, d)], channel=j))
                        sent[d] = k + 1

            with trace_range(f"stage{me}_fwd_seg{j}_mb{m}"):
                out = run_segment(self.blocks, a, b, self.depth, env, ts[m] if j == head else None, "partials",
                                  emit=emit if self.fwd_msgs[j] else None)
            _debug_point(self.device)
            if j == head:
                partials[m] = out["partials"]
                continue
            fout[(j, m)] = {name: out[name] for name, _ in self.outs[j]}
            for d, edges in self.fwd_msgs[j].items():
                rest = edges[sent[d]:]
                if rest:
                    pending.append(self._post(sends=[(out[name], d) for name, _ in rest], channel=j))
        frx = None

        # ---------------- backward (each segment's microbatches in reverse order) ----------------
        loss = dP = None
        if self.is_last:
            P = torch.stack([p.detach() for p in partials]).requires_grad_(True)
            loss = loss_from_partials(P.sum(0), targets.numel(), dice)
            (loss * loss_scale).backward()
            dP = P.grad
        brx = {}           # gradient messages (consumer segment c, microbatch m) to this stage
        for c in range(pl.K):
            edges = self.bwd_msgs[c].get(me)
            if not edges:
                continue
            for m in reversed(range(M)):
                bufs, recvs = {}, []
                for name, p in edges:
                    g, flat = self._empty_wire(tuple(fout[(p, m)][name].shape))
                    bufs[name] = g
                    recvs.append((flat, pl.owner[c]))
                brx[(c, m)] = (bufs, self._post(recvs=recvs, channel=c))
        if hasattr(self.blocks, "open_defer_window"):
            self.blocks.open_defer_window()     # the microbatches' weight gradients: one launch per layer
        nxt = {j: M - 1 for j in self.segs}
        for j in self.orders["bwd"]:
            m = nxt[j]
            nxt[j] -= 1
            with trace_range(f"stage{me}_bwd_seg{j}_mb{m}"):
                if j == head:
                    torch.autograd.backward(partials[m], dP[m])
                    partials[m] = None
                else:
                    outs, grads = [], []
                    for name, c in self.outs[j]:
                        o = fout[(j, m)][name]
                        if pl.owner[c] == me:
                            assert (c, m, name) in caps, f"segment {c} mb {m} backward must precede segment {j}'s"
                            g = caps.pop((c, m, name))
                        else:
                            bufs, xfer = brx[(c, m)]
                            xfer.wait()
                            g = bufs[name]
                        if g is not None and o.requires_grad:
                            outs.append(o)
                            grads.append(g.to(o.dtype))
                    if outs:
                        torch.autograd.backward(outs, grads)
                    fout[(j, m)] = None
            _debug_point(self.device)
            for d, edges in self.bwd_msgs[j].items():
                gs = []
                for name, _ in edges:
                    g = caps.pop((j, m, name), None)
                    gs.append(g if g is not None else torch.zeros(self._shape(name, mb, h, w, pl.cuts[j]),
                                                                   dtype=self.comm_dtype, device=self.device))
                pending.append(self._post(sends=[(g, d) for g in gs], channel=j))
            for name, p in self.ins[j]:            # local producers read theirs from caps; nothing else left
                if pl.owner[p] != me:
                    caps.pop((j, m, name), None)
        if hasattr(self.blocks, "close_defer_window"):
            self.blocks.close_defer_window()
        for xfer in pending:
            xfer.wait()
        for _, (_, xfer) in brx.items():
            xfer.wait()
        return loss

    @torch.no_grad()
    def eval_probs(self, images, batch, hw):
        """Inference through the pipeline (one microbatch = whole batch); probs on the head stage."""
        h, w = hw
        pl, me = self.pl, self.rank
        fout, sent, probs = {}, [], None
        got = {}                                   # producer segment -> its (one) message to this stage
        for j in range(pl.K):                      # chain order on every rank: no circular wait
            if pl.owner[j] != me:
                continue
            env = {}
            for name, p in self.ins[j]:
                if pl.owner[p] == me:
                    env[name] = fout[p][name]
                    continue
                if p not in got:
                    edges = self.fwd_msgs[p][me]
                    bufs, recvs = {}, []
                    for n2, c in edges:
                        t, flat = self._empty_wire(self._shape(n2, batch, h, w, pl.cuts[c]))
                        bufs[n2] = t
                        recvs.append((flat, pl.owner[p]))
                    self._post(recvs=recvs, channel=p).wait()
                    got[p] = bufs
                env[name] = got[p][name]
            if j == 0:
                env["x"] = images
            a, b = pl.seg_range(j)
            out = run_segment(self.blocks, a, b, self.depth, env, None, "probs" if j == pl.head_seg else "partials")
            if j == pl.head_seg:
                probs = out["probs"]
                continue
            fout[j] = out
            for d, edges in self.fwd_msgs[j].items():
                sent.append(self._post(sends=[(out[n], d) for n, _ in edges], channel=j))
        for x in sent:
            x.wait()
        return probs

    def gather_state_dict(self):
        """Full model state dict on stage 0 (other stages send their parameters and buffers)."""
        params = {**dict(self.model.named_parameters()), **dict(self.model.named_buffers())}
        sd = {}
        for s in range(self.S):
            snames = placement_param_names(self.model, self.pl, s) + placement_buffer_names(self.model, self.pl, s)
            for n in snames:
                if s == 0:
                    if self.rank == 0:
                        sd[n] = params[n].detach().clone()
                elif self.rank == s:
                    t = params[n].detach().contiguous()
                    dist.send(t.cpu() if self._host_staged else t, dst=self._glob(0), group=self.group)
                elif self.rank == 0:
                    dev = "cpu" if self._host_staged else params[n].device
                    t = torch.empty(params[n].shape, dtype=params[n].dtype, device=dev)
                    dist.recv(t, src=self._glob(s), group=self.group)
                    sd[n] = t.to(params[n].device)
        if self.rank == 0:
            full = self.model.state_dict()
            return {k: sd.get(k, v) for k, v in full.items()}
        return None


class _Transfer:
    """Outstanding grouped P2P operations of one pipeline step phase."""

    def __init__(self, works, keep, copies):
        self.works, self.keep, self.copies = works, keep, copies

    def wait(self):
        for w in self.works:
            w.wait()
        for host, dev in self.copies:
            dev.copy_(host)
        self.works, self.keep, self.copies = [], [], []


class GPipeLocal:
    """Single-process pipeline over local devices (reference MP form, N stages x M microbatches) on any
    :class:`.placement.Placement`: segment j runs on ``devices[owner[j]]``."""

    def __init__(self, model, devices: Sequence, microbatches: int, backend: str = "auto", dtype: str = "bf16",
                 cuts: Optional[List[float]] = None, img_hw=(512, 512), mode: str = "balanced",
                 placement: Optional[Placement] = None):
        self.devices = [torch.device(d) for d in devices]
        self.S = len(self.devices)
        self.M = microbatches
        self.model = model
        self.depth = model.cfg.depth
        if placement is None:
            placement = Placement.contiguous(cuts or partition(model.cfg, self.S, img_hw[0], img_hw[1], mode=mode))
        self.pl = placement.validate(self.depth)
        assert self.pl.S == self.S, f"placement has {self.pl.S} stages for {self.S} devices"
        self.cuts = list(self.pl.cuts)
        # place each segment's parameters on its stage's device
        for s in range(self.S):
            for n in placement_param_names(model, self.pl, s):
                mod_name, _, pname = n.rpartition(".")
                mod = model.get_submodule(mod_name)
                setattr(mod, pname, torch.nn.Parameter(getattr(mod, pname).detach().to(self.devices[s])))
            for n in placement_buffer_names(model, self.pl, s):
                mod_name, _, bname = n.rpartition(".")
                mod = model.get_submodule(mod_name)
                setattr(mod, bname, getattr(mod, bname).to(self.devices[s]))
        self.spaces = []
        for s in range(self.S):
            names = set(placement_param_names(model, self.pl, s))
            own = [(n, p) for n, p in model.named_parameters() if n in names]
            self.spaces.append(FlatParameterSpace(own, device=self.devices[s]))
        # each stage's engine packs only its own layers' weights (stages sharing a device would
        # otherwise each re-pack the whole model every step)
        self.stage_blocks = [make_blocks(model, backend, dtype, device=self.devices[s],
                                         owned={id(p) for p in self.spaces[s].params})
                             for s in range(self.S)]
        for s, b in enumerate(self.stage_blocks):
            b.device = self.devices[s]
            if hasattr(b, "defer_wgrad"):      # one weight-gradient launch per layer per step (HipBlocks)
                b.defer_wgrad = microbatches
        # skips between stages: engines on the SAME device share one concat-buffer registry (the decoder
        # stage finds the encoder's concat buffer: zero-copy, as in a single-stage run); a skip that
        # changes device is written dense by its producer (one peer copy into the consumer's buffer)
        _, send = _stage_io(self.pl, self.depth)
        first = {}
        for s, b in enumerate(self.stage_blocks):
            if hasattr(b, "_cats"):
                d = self.devices[s]
                if d in first:
                    b._cats = first[d]._cats
                else:
                    first[d] = b
        for s, b in enumerate(self.stage_blocks):
            if hasattr(b, "dense_skips"):
                b.dense_skips = {int(n[len("skip"):]) for n, dst in send[s]
                                 if n.startswith("skip") and self.devices[dst] != self.devices[s]}
        self.ins, _ = seg_io(self.pl, self.depth)

    def _run(self, j, env, target, want):
        dev = self.devices[self.pl.owner[j]]
        env = {k: v.to(dev, non_blocking=True) for k, v in env.items()}
        if target is not None:
            target = target.to(dev, non_blocking=True)
        ctx = torch.cuda.device(dev) if dev.type == "cuda" else _Null()
        a, b = self.pl.seg_range(j)
        with ctx:
            out = run_segment(self.stage_blocks[self.pl.owner[j]], a, b, self.depth, env, target, want)
        _debug_point(dev)
        return out

    def _wave(self, images, targets, want):
        """Microbatches through the segments in wavefront order: at tick k, segments K-1..0 run
        microbatch k-j (later segments issued first, like unet_model.py:33-44, so a downstream device
        never waits behind upstream launches).  Returns the head outputs per microbatch."""
        K, head = self.pl.K, self.pl.head_seg
        xs = images.chunk(self.M)
        M = len(xs)
        ts = targets.chunk(M) if targets is not None else [None] * M
        outs = {}
        res = [None] * M
        for k in range(M + K - 1):
            for j in reversed(range(K)):
                m = k - j
                if not 0 <= m < M:
                    continue
                env = {name: outs[(p, m)][name] for name, p in self.ins[j]}
                if j == 0:
                    env["x"] = xs[m]
                out = self._run(j, env, ts[m] if j == head else None, want if j == head else "partials")
                if j == head:
                    res[m] = out[want]
                else:
                    outs[(j, m)] = out
        return res

    def forward_partials(self, images, targets):
        return sum(p.to(self.devices[0]) for p in self._wave(images, targets, "partials"))

    def forward_loss(self, images, targets, dice=True):
        return loss_from_partials(self.forward_partials(images, targets), targets.numel(), dice)

    @torch.no_grad()
    def probs(self, images):
        pl = self.pl
        outs = {}
        for j in range(pl.K):
            env = {name: outs[p][name] for name, p in self.ins[j]}
            if j == 0:
                env["x"] = images
            out = self._run(j, env, None, "probs" if j == pl.head_seg else "partials")
            if j == pl.head_seg:
                return out["probs"].to(self.devices[0])
            outs[j] = out

    def forward_probs(self, images):
        """Differentiable pipelined forward to the probability map (``UNet(pipe=True).forward``):
        microbatches in wavefront order, outputs concatenated on the first device (reference
        ``torch.cat(ret).to('cuda:0')``, unet_model.py:53)."""
        return torch.cat([p.to(self.devices[0]) for p in self._wave(images, None, "probs")])


class _Null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
