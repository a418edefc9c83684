"""GPipe P2P ordering on RCCL, checked op by op on CPU (gloo, 4 and 8 ranks).

torch coalesces every ``batch_isend_irecv`` of a process group onto that group's single RCCL
communicator and stream, in issue order.  If one rank both received and sent on one group, a receive
it pre-posted for microbatch m+1 would hold back its send of microbatch m (a middle stage could
not hand m downstream before m+1 arrived from upstream).  ``GPipeDist`` therefore gives every
sending stage its own group (``sender_groups``): these tests record each rank's posted operations
per group and assert that on every group a rank only sends (its own group) or only receives (any
other group) -- so no send can follow an unmatched receive on one stream -- and that the pipelined
step still equals a single-process step of the full batch (reference ``model/unet_model.py:33-44``
issues the downstream stage first for the same reason).
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


def _worker(rank, world, port, microbatches, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from distributedpytorch_amd.parallel.pipeline import GPipeDist
        torch.manual_seed(0)
        model = build_model("unet-tiny4")
        ref = build_model("unet-tiny4")
        ref.load_state_dict(model.state_dict())
        pipe = GPipeDist(model, microbatches, backend="torch", dtype="fp32", img_hw=(32, 32), mode="balanced")
        g = torch.Generator().manual_seed(5)
        x = torch.rand(4, 3, 32, 32, generator=g)
        t = (torch.rand(4, 1, 32, 32, generator=g) > 0.5).float()
        pipe.op_log = []
        loss = pipe.train_step(x if pipe.is_first else None, t if pipe.is_last else None, 4, (32, 32))
        lref = bce_dice_from_probs(ref(x), t)
        lref.backward()
        refp = dict(ref.named_parameters())
        bad = [n for n, p in model.named_parameters()
               if p.requires_grad and p.grad is not None and not torch.allclose(p.grad, refp[n].grad, atol=1e-5)]
        q.put((rank, pipe.op_log, pipe.members, pipe.cuts, None if loss is None else float(loss), float(lref), bad))
    except Exception as e:   # surface the failure instead of a queue timeout
        q.put((rank, repr(e), None, None, None, None, None))
    finally:
        dist.destroy_process_group()


def _run(world, microbatches):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, microbatches, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    return res


@pytest.mark.parametrize("world", [4, 8])
def test_no_send_behind_own_receive(world):
    res = _run(world, microbatches=4)
    for rank, log, members, cuts, loss, lref, bad in res:
        assert isinstance(log, list), f"rank {rank} failed: {log}"
        assert log, f"rank {rank} posted nothing"
        groups = {}
        for grp, kind, peer in log:
            assert rank in members[grp], f"rank {rank} used group {grp} it is not a member of"
            groups.setdefault(grp, []).append((kind, peer))
        for grp, ops in groups.items():
            kinds = {k for k, _ in ops}
            if grp == rank:
                assert kinds == {"send"}, f"rank {rank}: its own group carries {kinds}"
            else:
                assert kinds == {"recv"} and all(p == grp for _, p in ops), \
                    f"rank {rank}: group {grp} carries {ops}"
            # the VERDICT's property, stated directly: no send after a receive on one group
            seen_recv = False
            for k, _ in ops:
                assert not (k == "send" and seen_recv), f"rank {rank}: send queued behind a receive on group {grp}"
                seen_recv |= k == "recv"
        assert not bad, f"rank {rank}: gradients differ for {bad}"
        if rank == world - 1:
            assert abs(loss - lref) < 1e-5, (loss, lref)
    # every stage sends: activations downstream (all but the last), gradients upstream (all but the first)
    assert all(any(k == "send" for _, k, _ in r[1]) for r in res)


def test_sender_groups_cover_every_edge():
    from distributedpytorch_amd.parallel.pipeline import sender_groups, stage_io
    from distributedpytorch_amd.models.blocks import partition
    cfg = build_model("unet-tiny4").cfg
    for S in (2, 3, 4, 8):
        cuts = partition(cfg, S, 64, 64, mode="balanced")
        recv, send = stage_io(cuts, cfg.depth)
        members = sender_groups(recv, send)
        for s in range(S):
            for _, d in send[s]:          # forward activation s -> d rides group s
                assert d in members[s]
            for _, p in recv[s]:          # backward gradient s -> p rides group s
                assert p in members[s]
