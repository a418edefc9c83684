"""GPipe pipeline model parallelism for the UNet (``-t MP``).

Reference: a hand-written 2-stage, 2-microbatch pipeline inside ``UNet.forward``
(``model/unet_model.py:14-53``): encoder+mid on cuda:0, decoder+head on
cuda:1, the bottleneck and all four skips copied with ``.to('cuda:1')`` per microbatch, overlap
only from async launch order, backward via plain autograd.

Here, generalised to N stages x M microbatches (GPipe: all forwards, then all backwards):

* :class:`GPipeDist` - one process per GPU (torchrun), the MI355X-native form.  Each rank owns one
  contiguous block range (:func:`..models.blocks.partition`, FLOP-balanced, or the reference cut).
  Activations AND skip tensors go *directly* from producer to consumer stage with RCCL
  ``isend/irecv`` (one xGMI hop on the fully connected MI355X mesh - skips never relay through
  intermediate stages), sent in the compute dtype (bf16: half the reference's bytes).  P2P runs on
  RCCL's per-peer streams, so transfers overlap with the next microbatch's compute; receives are
  posted one microbatch ahead.  The last stage sums the per-microbatch loss partial sums, which
  gives exactly the reference's full-batch loss (global Dice), then back-propagates microbatch by
  microbatch so gradients start flowing upstream immediately.
* :class:`GPipeLocal` - single process, N local devices (the reference's own form, kept for
  ``python train.py -t MP`` without torchrun): stages issued in wavefront order so stage s works
  on microbatch m while stage s+1 works on microbatch m-1; cross-device copies are peer copies.

Both are numerically transparent: pipelined forward == plain forward (SURVEY §3.4 probe7), checked
by the tests against a single-device run.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

import torch
import torch.distributed as dist

from ..compute import loss_from_partials, make_blocks
from ..models.blocks import boundary_names, block_kind, n_blocks, partition, run_segment, segment_units, skip_name
from ..optim import FlatParameterSpace
from ..utils.tracing import trace_range


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


def _tensor_producer(name: str, cut_start: float, cuts: Sequence[float], depth: int) -> int:
    """Stage that produces boundary tensor ``name`` entering the stage starting at ``cut_start``."""
    if name == "x":
        return list(cuts).index(cut_start) - 1
    lvl = int(name[len("skip"):])
    return _stage_of_block(lvl + 0.5, cuts)      # a skip is produced by its encoder block's part b


def _stage_of_block(pos: float, cuts: Sequence[float]) -> int:
    """Stage whose segment contains position ``pos`` (a block index, or ``b + 0.5`` for part b)."""
    for s in range(len(cuts) - 1):
        if cuts[s] <= pos < cuts[s + 1]:
            return s
    raise ValueError(pos)


def stage_io(cuts: Sequence[int], depth: int):
    """Per stage: ``recv`` list of (name, src_stage) and ``send`` list of (name, dst_stage)."""
    S = len(cuts) - 1
    recv = [[] for _ in range(S)]
    send = [[] for _ in range(S)]
    for s in range(1, S):
        # x comes from the previous stage
        recv[s].append(("x", s - 1))
        send[s - 1].append(("x", s))
    for lvl in range(depth):
        p = _stage_of_block(lvl + 0.5, cuts)                      # produced by part b of enc block lvl
        c = _stage_of_block(depth + 1 + (depth - 1 - lvl), cuts)  # consumed by part a of its decoder block
        if p != c:
            recv[c].append((skip_name(lvl), p))
            send[p].append((skip_name(lvl), c))
    return recv, send


def sender_groups(recv_spec, send_spec) -> List[List[int]]:
    """Members of each stage's sender communicator: the stage, the stages it sends activations to
    (forward) and the stages it sends gradients to (backward: its producers), sorted."""
    S = len(send_spec)
    return [sorted({s} | {d for _, d in send_spec[s]} | {p for _, p in recv_spec[s]}) for s in range(S)]


def infer_shapes(cfg, microbatch: int, h: int, w: int) -> Dict[str, tuple]:
    """Shapes (NCHW) of every boundary tensor for one microbatch, by arithmetic (no tracing)."""
    shapes = {}
    H, W = h, w
    for lvl, wd in enumerate(cfg.widths):
        shapes[skip_name(lvl)] = (microbatch, wd, H, W)
        H, W = H // 2, W // 2
    return shapes


class _Stage:
    def __init__(self, model, blocks, start, end, depth):
        self.model, self.blocks, self.start, self.end, self.depth = model, blocks, start, end, depth

    def forward(self, env, target=None, want="partials"):
        return run_segment(self.blocks, self.start, self.end, self.depth, env, target, want)


class GPipeDist:
    """Multi-process GPipe over a process group whose size == number of stages.

    Communication (RCCL over xGMI, or gloo on CPU):
    * one communicator PER SENDING STAGE (:func:`sender_groups`): stage s sends only on its own
      group G[s] = {s} + its consumers + its producers, and receives from p only on G[p].  torch
      puts every coalesced P2P op of a group on that group's single RCCL stream in issue order, so
      with one shared group a pre-posted receive would hold back the same rank's later send (a
      middle stage could not hand microbatch m downstream before m+1 arrived from upstream); with
      sender groups no rank ever both sends and receives on one group, so sends never queue behind
      its own receives (checked op by op in ``tests/test_pipeline_p2p_order.py``);
    * the tensors of one microbatch that go to the same group are posted as ONE
      ``batch_isend_irecv`` group (RCCL group call: the x and skip transfers start together);
    * forward receives for microbatch m+1 and backward gradient receives for microbatch m-1 are
      posted before microbatch m computes, so transfer latency hides behind compute;
    * every group's communicator is created at construction (a 1-element exchange from its sender
      to every member), so the lazy RCCL communicator setup never lands inside a training step;
    * a skip that leaves this stage is written by the encoder conv into a dense tensor (HIP engine
      ``dense_skips``) and sent as is; activations travel in the compute dtype (bf16).
    """

    def __init__(self, model, microbatches: int, backend: str = "auto", dtype: str = "bf16",
                 group=None, cuts: Optional[List[int]] = None, img_hw=(512, 512), mode: str = "balanced",
                 warm: bool = True):
        self.group = group
        self.rank = dist.get_rank(group)
        self.S = dist.get_world_size(group)
        self.M = microbatches
        self.model = model
        self.depth = model.cfg.depth
        self.cuts = cuts or partition(model.cfg, self.S, img_hw[0], img_hw[1], mode=mode)
        assert len(self.cuts) == self.S + 1
        self.start, self.end = self.cuts[self.rank], self.cuts[self.rank + 1]
        self.recv_spec, self.send_spec = stage_io(self.cuts, self.depth)
        self.device = next(model.parameters()).device
        names = set(stage_param_names(model, self.start, self.end))
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
        self.stage = _Stage(model, self.blocks, self.start, self.end, self.depth)
        self.comm_dtype = torch.bfloat16 if (dtype == "bf16" and self.device.type == "cuda") else torch.float32
        self.is_first = self.rank == 0
        self.is_last = self.rank == self.S - 1
        self._glob = lambda s: dist.get_global_rank(group, s) if group is not None else s
        self._host_staged = self.device.type == "cuda" and dist.get_backend(group) != "nccl"
        self.peers = sorted({p for _, p in self.recv_spec[self.rank]} | {p for _, p in self.send_spec[self.rank]})
        # per-sender communicators: stage s sends only on groups[s], receives from p only on groups[p]
        self.members = sender_groups(self.recv_spec, self.send_spec)
        self.groups: Dict[int, object] = {}
        world_pipeline = group is None or dist.get_world_size(group) == dist.get_world_size()
        for s in range(self.S):
            ranks = [self._glob(r) for r in self.members[s]]
            if len(ranks) < 2:
                continue
            if world_pipeline:      # every rank of the job calls new_group, members or not
                g = dist.new_group(ranks)
            elif self.rank in self.members[s]:   # pipeline inside a bigger job: members only, in order
                g = dist.new_group(ranks, use_local_synchronization=True)
            else:
                continue
            if self.rank in self.members[s]:
                self.groups[s] = g
        self.op_log: Optional[list] = None   # tests: [(sender group, "send"/"recv", peer stage)] per posted op
        if warm:
            self.warm_up()

    def warm_up(self):
        """One tiny exchange on every group this stage belongs to (its sender to each member), in
        stage order on every rank: creates the RCCL communicators now instead of inside the first
        timed step, and every group's first operation involves all of its members."""
        dev = "cpu" if self._host_staged else self.device
        for s in sorted(self.groups):
            g = self.groups[s]
            others = [r for r in self.members[s] if r != s]
            ops, keep = [], []
            if s == self.rank:
                out = torch.full((1,), float(self.rank), dtype=self.comm_dtype, device=dev)
                keep.append(out)
                ops = [dist.P2POp(dist.isend, out, self._glob(r), g) for r in others]
            else:
                inp = torch.empty(1, dtype=self.comm_dtype, device=dev)
                keep.append(inp)
                ops = [dist.P2POp(dist.irecv, inp, self._glob(s), g)]
            for w in dist.batch_isend_irecv(ops):
                w.wait()
            if s != self.rank:
                assert int(keep[0].float().item()) == s, f"stage {self.rank}: sender {s} answered {keep[0].item()}"

    # shapes of the boundary tensors for this microbatch size
    def _shape(self, name, mb, h, w):
        cfg = self.model.cfg
        if name.startswith("skip"):
            return infer_shapes(cfg, mb, h, w)[name]
        # "x" entering block `cut`: encoder levels floor-halve, the decoder doubles from the bottom
        cut = self.start
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

    def _post(self, sends=(), recvs=()):
        """One grouped P2P launch: ``sends`` = [(tensor, dst)], ``recvs`` = [(flat buffer, src)].
        Returns a :class:`_Transfer` whose ``wait()`` completes it (and keeps the send buffers alive).

        RCCL moves device memory directly (ordered after the producing kernels on the current
        stream).  gloo (CPU tests; the one-GPU rehearsal of this path, ranks sharing cuda:0) is
        host-staged explicitly: a device buffer is copied to host memory before the send and from
        it after the receive completes."""
        by_group: Dict[int, list] = {}
        keep, copies = [], []
        for t, dst in sends:                      # all on this stage's own sender group
            buf = self._wire(t)
            if self._host_staged:
                buf = buf.to("cpu")                   # synchronous: the producing kernels have finished
            keep.append(buf)
            by_group.setdefault(self.rank, []).append(dist.P2POp(dist.isend, buf, self._glob(dst), self.groups[self.rank]))
            self._log(self.rank, "send", dst)
        for flat, src in recvs:                   # on the SENDER's group
            if self._host_staged:
                host = torch.empty(flat.shape, dtype=flat.dtype)
                copies.append((host, flat))
                flat = host
            by_group.setdefault(src, []).append(dist.P2POp(dist.irecv, flat, self._glob(src), self.groups[src]))
            self._log(src, "recv", src)
        works = []
        for g in sorted(by_group):
            works.extend(dist.batch_isend_irecv(by_group[g]))
        return _Transfer(works, keep, copies)

    def _log(self, group_sender: int, kind: str, peer: int):
        if self.op_log is not None:
            self.op_log.append((group_sender, kind, peer))

    def _irecv(self, mb, h, w):
        bufs, recvs = {}, []
        for name, src in self.recv_spec[self.rank]:
            t, flat = self._empty_wire(self._shape(name, mb, h, w))
            recvs.append((flat, src))
            bufs[name] = t
        return bufs, self._post(recvs=recvs)

    def _irecv_grads(self, outs: Dict[str, torch.Tensor]):
        grads, recvs = [], []
        for name, dst in self.send_spec[self.rank]:
            g, flat = self._empty_wire(tuple(outs[name].shape))
            recvs.append((flat, dst))
            grads.append(g)
        return grads, self._post(recvs=recvs)

    def train_step(self, images: Optional[torch.Tensor], targets: Optional[torch.Tensor], batch: int,
                   hw, dice: bool = True, loss_scale: float = 1.0):
        """One GPipe step. Returns the (full-batch) loss on the last stage, None elsewhere."""
        h, w = hw
        M = self.M
        assert batch % M == 0, f"batch {batch} must be divisible by microbatches {M}"
        mb = batch // M
        xs = images.chunk(M) if self.is_first else [None] * M
        ts = targets.chunk(M) if self.is_last else [None] * M
        saved_in, saved_out, pending = [], [], []
        partials = []
        nxt = self._irecv(mb, h, w) if not self.is_first else None
        for m in range(M):
            if self.is_first:
                env = {"x": xs[m]}
                leaves = {}
            else:
                bufs, xfer = nxt
                xfer.wait()
                if m + 1 < M:
                    nxt = self._irecv(mb, h, w)        # microbatch m+1 lands while m computes
                leaves = {k: v.detach().requires_grad_(True) for k, v in bufs.items()}
                env = dict(leaves)
            with trace_range(f"stage{self.rank}_fwd_mb{m}"):
                out = self.stage.forward(env, ts[m], "partials")
            _debug_point(self.device)
            saved_in.append(leaves)
            if self.is_last:
                partials.append(out["partials"])
                saved_out.append({})
            else:
                sends = {name: out[name] for name, _ in self.send_spec[self.rank]}
                pending.append(self._post(sends=[(sends[n], d) for n, d in self.send_spec[self.rank]]))
                saved_out.append(sends)

        # ---------------- backward (microbatches in reverse order) ----------------
        loss = None
        if self.is_last:
            P = torch.stack([p.detach() for p in partials]).requires_grad_(True)
            loss = loss_from_partials(P.sum(0), targets.numel(), dice)
            (loss * loss_scale).backward()
            dP = P.grad
        gnxt = self._irecv_grads(saved_out[M - 1]) if not self.is_last else None
        if hasattr(self.blocks, "open_defer_window"):
            self.blocks.open_defer_window()     # the microbatches' weight gradients: one launch per layer
        for m in reversed(range(M)):
            rng = trace_range(f"stage{self.rank}_bwd_mb{m}")
            rng.__enter__()
            if self.is_last:
                torch.autograd.backward(partials[m], dP[m])
            else:
                grads, xfer = gnxt
                xfer.wait()
                if m > 0:
                    gnxt = self._irecv_grads(saved_out[m - 1])   # gradients of m-1 land while m runs
                outs = [saved_out[m][name] for name, _ in self.send_spec[self.rank]]
                torch.autograd.backward(outs, [g.to(o.dtype) for o, g in zip(outs, grads)])
            rng.__exit__(None, None, None)
            _debug_point(self.device)
            if not self.is_first:
                gsends = []
                for name, src in self.recv_spec[self.rank]:
                    gr = saved_in[m][name].grad
                    if gr is None:
                        gr = torch.zeros_like(saved_in[m][name])
                    gsends.append((gr, src))
                pending.append(self._post(sends=gsends))
            saved_in[m] = saved_out[m] = None
        if hasattr(self.blocks, "close_defer_window"):
            self.blocks.close_defer_window()
        for xfer in pending:
            xfer.wait()
        return loss

    @torch.no_grad()
    def eval_probs(self, images, batch, hw):
        """Inference through the pipeline (one microbatch = whole batch); probs on the last stage."""
        h, w = hw
        if self.is_first:
            env = {"x": images}
        else:
            bufs, xfer = self._irecv(batch, h, w)
            xfer.wait()
            env = dict(bufs)
        out = self.stage.forward(env, None, "probs")
        if not self.is_last:
            self._post(sends=[(out[n], d) for n, d in self.send_spec[self.rank]]).wait()
        return out.get("probs")

    def gather_state_dict(self):
        """Full model state dict on stage 0 (other stages send their parameters and buffers)."""
        params = {**dict(self.model.named_parameters()), **dict(self.model.named_buffers())}
        all_cuts = self.cuts
        sd = {}
        for s in range(self.S):
            snames = (stage_param_names(self.model, all_cuts[s], all_cuts[s + 1])
                      + stage_buffer_names(self.model, all_cuts[s], all_cuts[s + 1]))
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
    """Single-process pipeline over local devices (reference MP form, N stages x M microbatches)."""

    def __init__(self, model, devices: Sequence, microbatches: int, backend: str = "auto", dtype: str = "bf16",
                 cuts: Optional[List[int]] = None, img_hw=(512, 512), mode: str = "balanced"):
        self.devices = [torch.device(d) for d in devices]
        self.S = len(self.devices)
        self.M = microbatches
        self.model = model
        self.depth = model.cfg.depth
        self.cuts = cuts or partition(model.cfg, self.S, img_hw[0], img_hw[1], mode=mode)
        # place each block's parameters on its stage's device
        for s in range(self.S):
            for n in stage_param_names(model, self.cuts[s], self.cuts[s + 1]):
                mod_name, _, pname = n.rpartition(".")
                mod = model.get_submodule(mod_name)
                setattr(mod, pname, torch.nn.Parameter(getattr(mod, pname).detach().to(self.devices[s])))
            for n in stage_buffer_names(model, self.cuts[s], self.cuts[s + 1]):
                mod_name, _, bname = n.rpartition(".")
                mod = model.get_submodule(mod_name)
                setattr(mod, bname, getattr(mod, bname).to(self.devices[s]))
        self.spaces = []
        for s in range(self.S):
            names = set(stage_param_names(model, self.cuts[s], self.cuts[s + 1]))
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
        _, send = stage_io(self.cuts, self.depth)
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

    def _run(self, s, env, target, want):
        dev = self.devices[s]
        env = {k: v.to(dev, non_blocking=True) for k, v in env.items()}
        if target is not None:
            target = target.to(dev, non_blocking=True)
        ctx = torch.cuda.device(dev) if dev.type == "cuda" else _Null()
        with ctx:
            out = run_segment(self.stage_blocks[s], self.cuts[s], self.cuts[s + 1], self.depth, env, target, want)
        _debug_point(dev)
        return out

    def forward_partials(self, images, targets):
        M, S = self.M, self.S
        xs, ts = images.chunk(M), targets.chunk(M)
        envs = [{"x": x} for x in xs]
        partials = [None] * M
        # wavefront order: at tick k, stages S-1..0 run microbatch k-s (later stages issued first,
        # like unet_model.py:33-44, so the downstream device never waits behind upstream launches)
        for k in range(M + S - 1):
            for s in reversed(range(S)):
                m = k - s
                if 0 <= m < M:
                    out = self._run(s, envs[m], ts[m] if s == S - 1 else None, "partials")
                    if s == S - 1:
                        partials[m] = out["partials"].to(self.devices[0])
                    else:
                        envs[m] = out
        return sum(partials)

    def forward_loss(self, images, targets, dice=True):
        return loss_from_partials(self.forward_partials(images, targets), targets.numel(), dice)

    @torch.no_grad()
    def probs(self, images):
        env = {"x": images}
        for s in range(self.S):
            env = self._run(s, env, None, "probs" if s == self.S - 1 else "partials")
        return env["probs"].to(self.devices[0])

    def forward_probs(self, images):
        """Differentiable pipelined forward to the probability map (``UNet(pipe=True).forward``):
        microbatches in wavefront order, outputs concatenated on the first device (reference
        ``torch.cat(ret).to('cuda:0')``, unet_model.py:53)."""
        M, S = self.M, self.S
        envs = [{"x": x} for x in images.chunk(M)]
        outs = [None] * len(envs)
        for k in range(len(envs) + S - 1):
            for s in reversed(range(S)):
                m = k - s
                if 0 <= m < len(envs):
                    envs[m] = self._run(s, envs[m], None, "probs" if s == S - 1 else "partials")
                    if s == S - 1:
                        outs[m] = envs[m]["probs"].to(self.devices[0])
        return torch.cat(outs)


class _Null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
