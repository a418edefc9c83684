"""Row-split pipeline engine (``-t MP`` with a spatial plan): the top L levels of the UNet split by image rows
over all S stages, the inner chain pipelined over the same stages (geometry, schedule model and plan search:
:mod:`.spatial`; reference pipeline: ``model/unet_model.py:14-53``).

One process per GPU (torchrun), one stage per rank.  Per microbatch m, on stage s (rows ``rp[s]``):

* ``L0f`` -- encoder levels 0..L-1 on the stage's image rows (halo rows computed redundantly, no exchange);
  the pooled rows of level L-1 go to the owner of the inner chain's first block;
* inner segments -- :func:`..models.blocks.run_segment` over the inner placement, x and skips sent straight
  from producer to consumer segment as in :class:`.pipeline.GPipeDist`; the first segment's input is the
  row-concatenation of the S pooled slices, the last segment's output is cut into each stage's rows;
* ``L0g`` -- decoder levels L-1..0 + head on the stage's rows: the loss partial sums of its own rows.

The loss is the reference's global BCE - log Dice over the whole batch: the stages' per-microbatch partial
sums are all-reduced (4 M floats), every stage then back-propagates its own ops.  Because every stage's slice
graph recomputes its halo rows itself, the split levels' parameter gradients are the SUM over the stages
(one all-reduce of their flat fp32 gradients after the backward) and the gradient of the inner chain's output
is the sum of the stages' overlapping row slices -- exactly the single-device gradients (tests:
``test_distributed_cpu.py::test_spatial_pipeline_matches_single_process``).

Communication: one communicator per SENDING op node (its owner is the only sender: activations forward,
gradients backward), every receive of a phase posted before the phase's first op, static per-stage op
orders from a list schedule of the op graph (:func:`.spatial.simulate_graph` on FLOP costs, identical on
every rank) -- a feasible schedule, so blocking on a receive can never deadlock.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

from ..compute import loss_from_partials, make_blocks
from ..models.blocks import block_costs, block_kind, n_blocks, run_segment, segment_units, skip_name
from ..optim import FlatParameterSpace
from ..utils.tracing import trace_range
from .pipeline import _Capture, _debug_point, _Transfer, stage_buffer_names, stage_param_names
from .spatial import GNode, SpatialPlan, simulate_graph


def _rows(t: torch.Tensor, off: int, n: int) -> torch.Tensor:
    """Rows [off, off + n) of a logical-NCHW tensor, dense in its layout (a copy only when the crop is not
    already contiguous: one image per microbatch crops in place)."""
    v = t[:, :, off:off + n, :]
    fmt = torch.channels_last if (t.is_cuda and t.dim() == 4) else torch.contiguous_format
    return v if v.is_contiguous(memory_format=fmt) else v.contiguous(memory_format=fmt)


def inner_io(plan: SpatialPlan, depth: int):
    """Per inner segment: ``ins[j]`` / ``outs[j]`` = [(name, other inner segment)] -- x along the chain and the
    skips of the inner encoder levels L..D-1 (those of the split levels never leave their stage)."""
    K = plan.K
    ins: List[List[Tuple[str, int]]] = [[] for _ in range(K)]
    outs: List[List[Tuple[str, int]]] = [[] for _ in range(K)]
    for j in range(1, K):
        ins[j].append(("x", j - 1))
        outs[j - 1].append(("x", j))
    for lvl in range(plan.L, depth):
        p = plan.seg_of(lvl + 0.5)
        c = plan.seg_of(depth + 1 + (depth - 1 - lvl))
        if p != c:
            ins[c].append((skip_name(lvl), p))
            outs[p].append((skip_name(lvl), c))
    return ins, outs


def split_param_names(model, L: int) -> List[str]:
    depth = model.cfg.depth
    nb = n_blocks(depth)
    names = []
    for b in list(range(L)) + list(range(nb - 1 - L, nb)):
        names += stage_param_names(model, b, b + 1)
    return names


def flop_graph(plan: SpatialPlan, cfg, M: int, h: int, w: int) -> List[GNode]:
    """The op graph with forward-FLOP costs (backward = 2x): deterministic on every rank, for the orders."""
    depth = cfg.depth
    nb = n_blocks(depth)
    c = block_costs(cfg, h, w)
    S, L = plan.S, plan.L
    enc = sum(c[b] for b in range(L)) / S / 1e9
    dec = sum(c[b] for b in range(nb - 1 - L, nb)) / S / 1e9
    nodes = [GNode(f"L0f{s}", s, enc, 2 * enc) for s in range(S)]
    ins, _ = inner_io(plan, depth)
    for j in range(plan.K):
        a, b = plan.seg_range(j)
        f = sum(c[i] * (1.0 if part == "full" else 0.5) for i, part in segment_units(a, b, depth)) / 1e9
        nodes.append(GNode(f"in{j}", plan.inner_owner[j], f, 2 * f, ins=[(S + p, 0) for p in {p for _, p in ins[j]}]))
    nodes[S].ins += [(s, 0) for s in range(S)]
    for s in range(S):
        nodes.append(GNode(f"L0g{s}", s, dec, 2 * dec, ins=[(S + plan.K - 1, 0)], head=True))
    return nodes


class SpatialGPipe:
    def __init__(self, model, plan: SpatialPlan, microbatches: int, backend: str = "auto", dtype: str = "bf16",
                 group=None, img_hw=(1024, 1024), warm: bool = True):
        cfg = model.cfg
        if getattr(cfg, "batchnorm", False):
            raise ValueError("row-split levels need batch statistics across stages: BatchNorm models are not supported")
        self.group = group
        self.rank = dist.get_rank(group)
        self.S = dist.get_world_size(group)
        self.depth = cfg.depth
        self.plan = plan.validate(self.depth)
        assert plan.S == self.S, f"spatial plan for {plan.S} stages, group of {self.S}"
        self.M = microbatches
        self.model = model
        self.H, self.W = img_hw
        self.rp = plan.rows(self.H)
        self.L = plan.L
        self.nb = n_blocks(self.depth)
        self.device = next(model.parameters()).device
        me = self.rank
        # parameters: the split levels (replicated on every stage, first in the flat buffer) + own inner segments
        self.split_names = split_param_names(model, self.L)
        inner_names = []
        for j in plan.segments(me):
            inner_names += stage_param_names(model, *plan.seg_range(j))
        params = dict(model.named_parameters())
        own_set = set(self.split_names) | set(inner_names)
        for n, p in model.named_parameters():
            if n not in own_set:
                p.requires_grad_(False)
        own = [(n, params[n]) for n in self.split_names + inner_names]
        self.space = FlatParameterSpace(own, device=self.device, order="given")
        self.n_split = sum(params[n].numel() for n in self.split_names)
        self.blocks = make_blocks(model, backend, dtype)
        if hasattr(self.blocks, "defer_wgrad"):
            self.blocks.defer_wgrad = microbatches
        self.ins, self.outs = inner_io(plan, self.depth)
        # one message per (sending segment, destination stage) and microbatch, tensors in sorted-name order
        # (the production order: skips by level, x last) -- the receiver posts ONE grouped receive for it
        self.fwd_to: Dict[int, Dict[int, List[str]]] = {}
        self.bwd_to: Dict[int, Dict[int, List[str]]] = {}
        for j in range(plan.K):
            for name, c in self.outs[j]:
                d = plan.inner_owner[c]
                if d != plan.inner_owner[j]:
                    lst = self.fwd_to.setdefault(j, {}).setdefault(d, [])
                    if name not in lst:
                        lst.append(name)
            for name, p_ in self.ins[j]:
                d = plan.inner_owner[p_]
                if d != plan.inner_owner[j]:
                    lst = self.bwd_to.setdefault(j, {}).setdefault(d, [])
                    if name not in lst:
                        lst.append(name)
        for dd in list(self.fwd_to.values()) + list(self.bwd_to.values()):
            for d in dd:
                dd[d].sort()
        if hasattr(self.blocks, "dense_skips"):
            # split levels' skips are cropped by their consumer; inner skips that leave the stage go as is
            self.blocks.dense_skips = set(range(self.L)) | {
                int(n[len("skip"):]) for j in plan.segments(me) for n, c in self.outs[j]
                if n.startswith("skip") and plan.inner_owner[c] != me}
        self.comm_dtype = torch.bfloat16 if (dtype == "bf16" and self.device.type == "cuda") else torch.float32
        self.first, self.last = plan.first_stage, plan.last_stage
        # every stage reads its rows of the batch and holds the loss; stage 0 is the "head" for logging
        self.is_first, self.is_last, self.head_rank = True, self.rank == 0, 0
        self._glob = lambda s: dist.get_global_rank(group, s) if group is not None else s
        self._host_staged = self.device.type == "cuda" and dist.get_backend(group) != "nccl"
        self._anchor = torch.zeros((), device=self.device, requires_grad=True)
        # op nodes: 0..S-1 = L0f_s, S..S+K-1 = inner j, S+K..S+K+S-1 = L0g_s
        S, K = self.S, plan.K
        self.NF, self.NI, self.NG = 0, S, S + K
        g = flop_graph(plan, cfg, microbatches, self.H, self.W)
        tl = simulate_graph(g, S, microbatches)
        self.orders = tl.orders[me]
        # communicators: one per sending node, members = its owner + every stage it sends to / receives from
        members: Dict[int, set] = {}
        for s in range(S):
            members[self.NF + s] = {s, self.first}
            members[self.NG + s] = {s, self.last}
        for j in range(K):
            m = {plan.inner_owner[j]}
            m |= {plan.inner_owner[c] for _, c in self.outs[j]}
            m |= {plan.inner_owner[p] for _, p in self.ins[j]}
            if j == 0 or j == K - 1:
                m |= set(range(S))
            members[self.NI + j] = m
        self.members = members
        self.groups: Dict[int, object] = {}
        for node in sorted(members):
            ranks = sorted(self._glob(r) for r in members[node])
            if len(ranks) < 2:
                continue
            pg = dist.new_group(ranks)            # every rank, same order
            if me in members[node]:
                self.groups[node] = pg
        self.owner = {**{self.NF + s: s for s in range(S)}, **{self.NG + s: s for s in range(S)},
                      **{self.NI + j: plan.inner_owner[j] for j in range(K)}}
        self.op_log: Optional[list] = None
        if warm:
            self.warm_up()
        # the split levels' parameters start identical on every stage (stage 0's)
        if self.n_split:
            self._bcast_split()

    # ------------------------------------------------------------------ comm helpers
    def _bcast_split(self):
        t = self.space.data[:self.n_split]
        if self._host_staged:
            h = t.cpu()
            dist.broadcast(h, src=self._glob(0), group=self.group)
            t.copy_(h)
        else:
            dist.broadcast(t, src=self._glob(0), group=self.group)
        self.space.touch()

    def _allreduce(self, t: torch.Tensor):
        if self._host_staged:
            h = t.cpu()
            dist.all_reduce(h, group=self.group)
            t.copy_(h)
        else:
            dist.all_reduce(t, group=self.group)

    def warm_up(self):
        dev = "cpu" if self._host_staged else self.device
        for node in sorted(self.groups):
            g = self.groups[node]
            sender = self.owner[node]
            others = sorted(r for r in self.members[node] if r != sender)
            if sender == self.rank:
                out = torch.full((1,), float(node), dtype=self.comm_dtype, device=dev)
                works = dist.batch_isend_irecv([dist.P2POp(dist.isend, out, self._glob(r), g) for r in others])
            else:
                inp = torch.empty(1, dtype=self.comm_dtype, device=dev)
                works = dist.batch_isend_irecv([dist.P2POp(dist.irecv, inp, self._glob(sender), g)])
            for w in works:
                w.wait()
            if sender != self.rank:
                assert int(inp.float().item()) == node, f"stage {self.rank}: channel {node} answered {inp.item()}"

    def _layout(self):
        return torch.channels_last if self.device.type == "cuda" else torch.contiguous_format

    def _empty_wire(self, shape):
        n, c, hh, ww = shape
        flat = torch.empty(n * c * hh * ww, dtype=self.comm_dtype, device=self.device)
        if self._layout() == torch.channels_last:
            return flat.view(n, hh, ww, c).permute(0, 3, 1, 2), flat
        return flat.view(n, c, hh, ww), flat

    def _wire(self, t):
        t = t.detach().to(self.comm_dtype).contiguous(memory_format=self._layout())
        if self._layout() == torch.channels_last:
            return t.permute(0, 2, 3, 1).reshape(-1)
        return t.reshape(-1)

    def _post(self, node: int, sends=(), recvs=()):
        g = self.groups[node]
        ops, keep, copies = [], [], []
        for t, dst in sends:
            buf = self._wire(t)
            if self._host_staged:
                buf = buf.to("cpu")
            keep.append(buf)
            ops.append(dist.P2POp(dist.isend, buf, self._glob(dst), g))
            if self.op_log is not None:
                self.op_log.append((node, "send", dst))
        for flat, src in recvs:
            if self._host_staged:
                host = torch.empty(flat.shape, dtype=flat.dtype)
                copies.append((host, flat))
                flat = host
            ops.append(dist.P2POp(dist.irecv, flat, self._glob(src), g))
            if self.op_log is not None:
                self.op_log.append((node, "recv", src))
        return _Transfer(dist.batch_isend_irecv(ops) if ops else [], keep, copies)

    def _cap(self, t, box, key):
        return _Capture.apply(self._anchor, t.detach(), box, key)

    # ------------------------------------------------------------------ shapes
    def _x_shape(self, mb: int, cut: float, name: str):
        """Logical NCHW shape of tensor ``name`` entering the inner segment that starts at ``cut``."""
        cfg, H, W = self.model.cfg, self.H, self.W
        if name.startswith("skip"):
            lvl = int(name[len("skip"):])
            return (mb, cfg.widths[lvl], H >> lvl, W >> lvl)
        kind, i = block_kind(int(cut), self.depth)
        hb, wb = H >> self.depth, W >> self.depth
        if cut != int(cut):
            if kind == "enc":
                return (mb, cfg.widths[i], H >> i, W >> i)
            if kind == "mid":
                return (mb, cfg.mid_width, hb, wb)
            return (mb, cfg.widths[self.depth - 1 - i], hb << (i + 1), wb << (i + 1))
        if kind == "enc":
            return (mb, cfg.widths[i - 1], H >> i, W >> i)
        if kind == "mid":
            return (mb, cfg.widths[-1], hb, wb)
        c = cfg.mid_width if i == 0 else cfg.widths[self.depth - i]
        return (mb, c, hb << i, wb << i)

    def _pool_shape(self, mb, s):
        sl = self.rp[s]
        return (mb, self.model.cfg.widths[self.L - 1], sl.send[1] - sl.send[0], self.W >> self.L)

    def _up_shape(self, mb, s):
        sl = self.rp[s]
        return (mb, self.model.cfg.widths[self.L], sl.recv[1] - sl.recv[0], self.W >> self.L)

    # ------------------------------------------------------------------ the split levels
    def _enc_split(self, x_img: torch.Tensor, m: int, fsplit: Dict):
        """Encoder levels 0..L-1 on this stage's rows of microbatch ``m``'s images (the full-height batch)."""
        sl = self.rp[self.rank]
        a0, a1 = sl.enc_in[0]
        x = self.blocks.prep(_rows(x_img, a0, a1 - a0).contiguous())
        skips = []
        for l in range(self.L):
            s_, pooled = self.blocks.enc(l, x)
            skips.append(s_)
            if l + 1 < self.L:
                n = sl.enc_in[l + 1][1] - sl.enc_in[l + 1][0]
                x = _rows(pooled, sl.enc_next_off(l), n)
        send = _rows(pooled, sl.send_off(), sl.send[1] - sl.send[0])
        fsplit[m] = {"skips": skips, "send": send}
        return send

    def _dec_split(self, up: torch.Tensor, target_rows: Optional[torch.Tensor], m: int, fsplit: Dict, caps: Dict,
                   want: str = "partials"):
        """Decoder levels L-1..0 + head on this stage's rows: ``up`` = the received rows of level L."""
        sl = self.rp[self.rank]
        x = up
        for l in range(self.L - 1, -1, -1):
            i = self.depth - 1 - l                       # decoder block index of level l
            d0, d1 = sl.dec_in[l]
            x = _rows(x, sl.up_off(l), (d1 - d0) // 2)
            skip = _rows(fsplit[m]["skips"][l], sl.skip_off(l), d1 - d0)
            if want == "partials":
                skip = self._cap(skip, caps, ("skip", l, m))
            x = self.blocks.dec(i, x, skip)
        y = _rows(x, sl.out_off(), sl.rows)
        if want == "partials":
            return self.blocks.head_partials(y, target_rows)
        return self.blocks.head_probs(y)

    # ------------------------------------------------------------------ the step
    def train_step(self, images: torch.Tensor, targets: torch.Tensor, batch: int, hw, dice: bool = True,
                   loss_scale: float = 1.0):
        """One GPipe step; every rank holds the full batch's images and targets (it reads its rows).
        Returns the full-batch loss (identical on every rank)."""
        h, w = hw
        assert (h, w) == (self.H, self.W), f"plan built for {self.H}x{self.W}, batch is {h}x{w}"
        M, pl, me, S, K = self.M, self.plan, self.rank, self.S, self.plan.K
        assert batch % M == 0
        mb = batch // M
        sl = self.rp[me]
        xs = images.chunk(M)
        ts = [t[:, :, sl.own[0]:sl.own[1], :].contiguous() for t in targets.chunk(M)]
        NF, NI, NG = self.NF, self.NI, self.NG
        # ---- every forward receive of the step
        frx = {}
        for m in range(M):
            if me == self.first:
                for s in range(S):
                    if s != me:
                        t, flat = self._empty_wire(self._pool_shape(mb, s))
                        frx[("pool", s, m)] = (t, self._post(NF + s, recvs=[(flat, s)]))
            for p in range(K):
                names = self.fwd_to.get(p, {}).get(me)
                if not names:
                    continue
                cut = {n: pl.inner_cuts[c] for n, c in self.outs[p] if pl.inner_owner[c] == me}
                bufs, recvs = {}, []
                for name in names:
                    t, flat = self._empty_wire(self._x_shape(mb, cut[name], name))
                    bufs[name] = t
                    recvs.append((flat, pl.inner_owner[p]))
                frx[("in", p, m)] = (bufs, self._post(NI + p, recvs=recvs))
            if me != self.last:
                t, flat = self._empty_wire(self._up_shape(mb, me))
                frx[("up", m)] = (t, self._post(NI + K - 1, recvs=[(flat, self.last)]))
        caps: Dict[tuple, torch.Tensor] = {}
        fsplit: Dict[int, dict] = {}
        fout: Dict[tuple, Dict[str, torch.Tensor]] = {}
        partials: List[Optional[torch.Tensor]] = [None] * M
        pending = []
        nxt: Dict[int, int] = {}
        for node in self.orders["fwd"]:
            m = nxt.get(node, 0)
            nxt[node] = m + 1
            if node < NI:                                           # L0f (this stage's)
                with trace_range(f"stage{me}_split_fwd_mb{m}"):
                    send = self._enc_split(xs[m], m, fsplit)
                if me != self.first:
                    pending.append(self._post(NF + me, sends=[(send, self.first)]))
            elif node < NG:                                         # inner segment j
                j = node - NI
                env = {}
                if j == 0:
                    parts = []
                    for s in range(S):
                        if s == me:
                            t = fsplit[m]["send"]
                        else:
                            t, xfer = frx[("pool", s, m)]
                            xfer.wait()
                        parts.append(self._cap(t, caps, ("pool", s, m)))
                    fmt = self._layout()
                    env["x"] = torch.cat(parts, dim=2).contiguous(memory_format=fmt)
                for name, p in self.ins[j]:
                    if pl.inner_owner[p] == me:
                        t = fout[(p, m)][name]
                    else:
                        bufs, xfer = frx[("in", p, m)]
                        xfer.wait()
                        t = bufs[name]
                    env[name] = self._cap(t, caps, (j, m, name))
                a, b = pl.seg_range(j)
                msgs = self.fwd_to.get(j, {})
                sent = {d: 0 for d in msgs}

                def emit(name, t, msgs=msgs, sent=sent, j=j):
                    # a skip leaving the stage goes the moment its encoder level finishes, in message order
                    for d, names in msgs.items():
                        k = sent[d]
                        if k < len(names) and names[k] == name:
                            pending.append(self._post(NI + j, sends=[(t, d)]))
                            sent[d] = k + 1

                with trace_range(f"stage{me}_inner_fwd_seg{j}_mb{m}"):
                    out = run_segment(self.blocks, a, b, self.depth, env, None, "partials",
                                      emit=emit if msgs else None)
                _debug_point(self.device)
                fout[(j, m)] = out
                for d, names in msgs.items():
                    rest = names[sent[d]:]
                    if rest:
                        pending.append(self._post(NI + j, sends=[(out[n], d) for n in rest]))
                if j == K - 1:                                      # up rows to every stage
                    full = out["x"]
                    for s in range(S):
                        if s != me:
                            r = self.rp[s].recv
                            pending.append(self._post(NI + j, sends=[(_rows(full, r[0], r[1] - r[0]), s)]))
            else:                                                   # L0g (this stage's)
                if me == self.last:
                    r = sl.recv
                    up = _rows(fout[(K - 1, m)]["x"], r[0], r[1] - r[0])
                else:
                    up, xfer = frx[("up", m)]
                    xfer.wait()
                up = self._cap(up, caps, ("up", m))
                with trace_range(f"stage{me}_split_dec_mb{m}"):
                    partials[m] = self._dec_split(up, ts[m], m, fsplit, caps)
        frx = None
        # ---- loss: the stages' partial sums of every microbatch, summed (global Dice over the batch)
        P = torch.stack([p.detach().float() for p in partials])
        self._allreduce(P)
        P = P.requires_grad_(True)
        loss = loss_from_partials(P.sum(0), targets.numel(), dice)
        (loss * loss_scale).backward()
        dP = P.grad
        # ---- every backward receive, posted in the order the senders send: microbatches M-1 .. 0 (a
        # communicator matches one sender's messages to a receiver in order)
        brx = {}
        for m in reversed(range(M)):
            if me == self.last:
                for s in range(S):
                    if s != me:
                        t, flat = self._empty_wire(self._up_shape(mb, s))
                        brx[("gup", s, m)] = (t, self._post(NG + s, recvs=[(flat, s)]))
            for c in range(K):
                names = self.bwd_to.get(c, {}).get(me)
                if not names:
                    continue
                prod = {n: p_ for n, p_ in self.ins[c] if pl.inner_owner[p_] == me}
                bufs, recvs = {}, []
                for name in names:
                    g_, flat = self._empty_wire(tuple(fout[(prod[name], m)][name].shape))
                    bufs[name] = g_
                    recvs.append((flat, pl.inner_owner[c]))
                brx[("in", c, m)] = (bufs, self._post(NI + c, recvs=recvs))
            if me != self.first:
                t, flat = self._empty_wire(self._pool_shape(mb, me))
                brx[("gpool", m)] = (t, self._post(NI, recvs=[(flat, self.first)]))
        if hasattr(self.blocks, "open_defer_window"):
            self.blocks.open_defer_window()
        nxt = {}
        for node in self.orders["bwd"]:
            m = nxt.get(node, M - 1)
            nxt[node] = m - 1
            if node >= NG:                                          # L0g backward
                with trace_range(f"stage{me}_split_dec_bwd_mb{m}"):
                    torch.autograd.backward(partials[m], dP[m].to(partials[m].dtype))
                partials[m] = None
                g_up = caps.pop(("up", m), None)
                if me != self.last:
                    if g_up is None:
                        g_up = torch.zeros(self._up_shape(mb, me), dtype=self.comm_dtype, device=self.device)
                    pending.append(self._post(NG + me, sends=[(g_up, self.last)]))
                else:
                    caps[("gup", me, m)] = g_up
            elif node >= NI:                                        # inner segment backward
                j = node - NI
                outs_, grads = [], []
                for name, c in self.outs[j]:
                    o = fout[(j, m)][name]
                    if pl.inner_owner[c] == me:
                        g_ = caps.pop((c, m, name), None)
                    else:
                        bufs, xfer = brx[("in", c, m)]
                        xfer.wait()
                        g_ = bufs[name]
                    if g_ is not None and o.requires_grad and not any(o is q for q in outs_):
                        outs_.append(o)
                        grads.append(g_.to(o.dtype))
                if j == K - 1:
                    # the stages' gradients of their (overlapping) up rows, summed into the output's gradient
                    o = fout[(j, m)]["x"]
                    gfull = torch.zeros(o.shape, dtype=torch.float32, device=o.device)
                    for s in range(S):
                        if s == me:
                            g_ = caps.pop(("gup", me, m), None)
                        else:
                            g_, xfer = brx[("gup", s, m)]
                            xfer.wait()
                        if g_ is not None:
                            r = self.rp[s].recv
                            gfull[:, :, r[0]:r[1], :] += g_.float()
                    outs_.append(o)
                    grads.append(gfull.to(o.dtype).contiguous(memory_format=self._layout()))
                with trace_range(f"stage{me}_inner_bwd_seg{j}_mb{m}"):
                    if outs_:
                        torch.autograd.backward(outs_, grads)
                fout[(j, m)] = None
                _debug_point(self.device)
                # gradients of this segment's remote inputs, to their producers' stages (one message each)
                for d, names in self.bwd_to.get(j, {}).items():
                    gs = []
                    for name in names:
                        g_ = caps.pop((j, m, name), None)
                        gs.append(g_ if g_ is not None else torch.zeros(
                            self._x_shape(mb, pl.inner_cuts[j], name), dtype=self.comm_dtype, device=self.device))
                    pending.append(self._post(NI + j, sends=[(g_, d) for g_ in gs]))
                if j == 0:
                    for s in range(S):
                        g_ = caps.pop(("pool", s, m), None)
                        if g_ is None:
                            g_ = torch.zeros(self._pool_shape(mb, s), dtype=self.comm_dtype, device=self.device)
                        if s == me:
                            caps[("gpool", m)] = g_
                        else:
                            pending.append(self._post(NI, sends=[(g_, s)]))
            else:                                                   # L0f backward
                if me == self.first:
                    gp = caps.pop(("gpool", m))
                else:
                    gp, xfer = brx[("gpool", m)]
                    xfer.wait()
                outs_, grads = [fsplit[m]["send"]], [gp.to(fsplit[m]["send"].dtype)]
                for l in range(self.L):
                    g_ = caps.pop(("skip", l, m), None)
                    if g_ is not None:
                        # the skip crop's gradient (a view of the level's output: autograd sums it in)
                        outs_.append(_rows_view(fsplit[m]["skips"][l], self.rp[me].skip_off(l), g_.shape[2]))
                        grads.append(g_)
                with trace_range(f"stage{me}_split_enc_bwd_mb{m}"):
                    torch.autograd.backward(outs_, grads)
                fsplit[m] = None
        if hasattr(self.blocks, "close_defer_window"):
            self.blocks.close_defer_window()
        for xfer in pending:
            xfer.wait()
        for _, (_, xfer) in brx.items():
            xfer.wait()
        # the split levels' parameter gradients: each stage holds its rows' share -> the sum
        if self.n_split:
            self._allreduce(self.space.grad[:self.n_split])
        return loss.detach()

    @torch.no_grad()
    def eval_probs(self, images: torch.Tensor, batch: int, hw) -> torch.Tensor:
        """Inference through the pipeline (one microbatch); the full-height probabilities on every rank."""
        saved = self.M
        try:
            self.M = 1
            probs = self._eval(images, batch)
        finally:
            self.M = saved
        return probs

    def _eval(self, images, batch):
        pl, me, S, K = self.plan, self.rank, self.S, self.plan.K
        NF, NI = self.NF, self.NI
        fsplit: Dict[int, dict] = {}
        send = self._enc_split(images, 0, fsplit)
        sent = []
        if me != self.first:
            sent.append(self._post(NF + me, sends=[(send, self.first)]))
        fout: Dict[int, dict] = {}
        rx: Dict[int, dict] = {}
        for j in range(K):                                  # chain order on every rank
            if pl.inner_owner[j] != me:
                continue
            env = {}
            if j == 0:
                parts = []
                for s in range(S):
                    if s == me:
                        parts.append(send)
                    else:
                        t, flat = self._empty_wire(self._pool_shape(batch, s))
                        self._post(NF + s, recvs=[(flat, s)]).wait()
                        parts.append(t)
                env["x"] = torch.cat(parts, dim=2).contiguous(memory_format=self._layout())
            for name, p in self.ins[j]:
                if pl.inner_owner[p] == me:
                    env[name] = fout[p][name]
                    continue
                if p not in rx:                            # producer p's one message to this stage
                    cut = {n: pl.inner_cuts[c] for n, c in self.outs[p] if pl.inner_owner[c] == me}
                    bufs, recvs = {}, []
                    for n in self.fwd_to[p][me]:
                        t, flat = self._empty_wire(self._x_shape(batch, cut[n], n))
                        bufs[n] = t
                        recvs.append((flat, pl.inner_owner[p]))
                    self._post(NI + p, recvs=recvs).wait()
                    rx[p] = bufs
                env[name] = rx[p][name]
            a, b = pl.seg_range(j)
            out = run_segment(self.blocks, a, b, self.depth, env, None, "partials")
            fout[j] = out
            for d, names in self.fwd_to.get(j, {}).items():
                sent.append(self._post(NI + j, sends=[(out[n], d) for n in names]))
            if j == K - 1:
                for s in range(S):
                    if s != me:
                        r = self.rp[s].recv
                        sent.append(self._post(NI + j, sends=[(_rows(out["x"], r[0], r[1] - r[0]), s)]))
        if me == self.last:
            r = self.rp[me].recv
            up = _rows(fout[K - 1]["x"], r[0], r[1] - r[0])
        else:
            up, flat = self._empty_wire(self._up_shape(batch, me))
            self._post(NI + K - 1, recvs=[(flat, self.last)]).wait()
        probs = self._dec_split(up, None, 0, fsplit, {}, want="probs").float()
        for x in sent:
            x.wait()
        # every stage's rows, gathered along H (padded to the tallest slice: uneven row plans)
        hmax = max(sl.rows for sl in self.rp)
        n, c, hh, ww = probs.shape
        mine = torch.zeros(n, c, hmax, ww, dtype=probs.dtype, device=probs.device)
        mine[:, :, :hh] = probs
        rows = [torch.empty_like(mine) for _ in self.rp]
        if self._host_staged:
            hr = [r.cpu() for r in rows]
            dist.all_gather(hr, mine.cpu(), group=self.group)
            rows = [r.to(probs.device) for r in hr]
        else:
            dist.all_gather(rows, mine, group=self.group)
        return torch.cat([r[:, :, :sl.rows] for r, sl in zip(rows, self.rp)], dim=2)

    def gather_state_dict(self):
        """Full model state dict on rank 0: the split levels from rank 0 itself, each inner segment's
        parameters from its owner."""
        params = {**dict(self.model.named_parameters()), **dict(self.model.named_buffers())}
        sd = {}
        for s in range(self.S):
            names = []
            for j in self.plan.segments(s):
                names += stage_param_names(self.model, *self.plan.seg_range(j))
                names += stage_buffer_names(self.model, *self.plan.seg_range(j))
            if s == 0:
                names += self.split_names
            for n in names:
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


def _rows_view(t: torch.Tensor, off: int, n: int) -> torch.Tensor:
    return t[:, :, off:off + n, :]
