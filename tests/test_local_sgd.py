"""Local SGD / DiLoCo outer step and pseudo-gradient reducers (gloo, 2 ranks).
Parity: ATorch ``atorch/local_sgd`` (reduce_methods linear / GTA / sparsify)."""

import os

import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn

from conftest import free_port


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        from dlrover_wuqiong_amd.atorch.local_sgd import GTAReducer, LinearReducer, LocalSGD

        dist.init_process_group("gloo", rank=rank, world_size=world)
        ok = True
        # linear mean reducer
        t = torch.full((4,), float(rank + 1))
        ok &= torch.allclose(LinearReducer().reduce_tensor(t), torch.full((4,), 1.5))
        # GTA sign consensus: rank0 [+1, +1, -2], rank1 [+3, -1, -1]
        t = torch.tensor([[1.0, 1.0, -2.0], [3.0, -1.0, -1.0]][rank])
        out = GTAReducer(consensus_method="sum").reduce_tensor(t)
        # elem0 both agree -> mean 2; elem1 sum 0 -> majority +, only rank0 agrees -> 1; elem2 both - -> -1.5
        ok &= torch.allclose(out, torch.tensor([2.0, 1.0, -1.5]))
        out = GTAReducer(consensus_method="count").reduce_tensor(
            torch.tensor([[1.0, 1.0, -2.0], [3.0, -1.0, -1.0]][rank]))
        ok &= torch.allclose(out, torch.tensor([2.0, 1.0, -1.5]))

        # LocalSGD: ranks start from rank-0 weights, diverge with different data,
        # re-synchronise every 3 steps to anchor - outer_lr * mean(delta)
        torch.manual_seed(rank)  # different init: the constructor broadcasts rank 0's
        model = nn.Linear(8, 4)
        inner = torch.optim.SGD(model.parameters(), lr=0.1)
        local = LocalSGD(model, inner, sync_every=3, outer_lr=1.0)
        w = [p.detach().clone() for p in model.parameters()]
        for p in w:
            g = [torch.empty_like(p) for _ in range(world)]
            dist.all_gather(g, p)
            ok &= torch.equal(g[0], g[1])
        gen = torch.Generator().manual_seed(100 + rank)
        for step in range(6):
            x = torch.randn(16, 8, generator=gen)
            loss = model(x).square().mean()
            loss.backward()
            local.step()
            local.zero_grad()
            flat = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
            g = [torch.empty_like(flat) for _ in range(world)]
            dist.all_gather(g, flat)
            synced = torch.equal(g[0], g[1])
            ok &= synced == ((step + 1) % 3 == 0)
        # outer lr 1 + mean reducer == plain parameter averaging
        ok &= torch.allclose(local.anchor, flat.float())
        # Nesterov outer optimizer keeps momentum state and stays in sync
        local2 = LocalSGD(model, torch.optim.SGD(model.parameters(), lr=0.05), sync_every=2, outer_lr=0.7,
                          outer_momentum=0.9, nesterov=True, reducer=GTAReducer(consensus_method=None))
        for _ in range(4):
            model(torch.randn(16, 8, generator=gen)).square().mean().backward()
            local2.step()
            local2.zero_grad()
        flat = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
        g = [torch.empty_like(flat) for _ in range(world)]
        dist.all_gather(g, flat)
        ok &= torch.equal(g[0], g[1]) and local2.momentum_buf.abs().sum() > 0
        q.put((rank, bool(ok)))
    except Exception as e:  # pragma: no cover
        import traceback

        q.put((rank, traceback.format_exc() + repr(e)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_local_sgd_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(30)
    assert res == {0: True, 1: True}, res


def test_sparsify():
    from dlrover_wuqiong_amd.atorch.local_sgd import sparsify

    t = torch.tensor([0.1, -5.0, 0.3, 2.0, -0.2, 1.0, 0.0, 4.0])
    s = sparsify(t, 0.5, "magnitude")
    assert (s != 0).sum() == 4 and s[1] == -5.0 and s[0] == 0
    torch.manual_seed(0)
    b = sparsify(torch.ones(10000), 0.25, "bernoulli")
    assert abs((b != 0).float().mean().item() - 0.25) < 0.03 and torch.allclose(b[b != 0], torch.tensor(4.0))
