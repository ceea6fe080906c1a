"""Dropless top-k MoE with expert parallelism (gloo, 2 ranks) against the
single-process layer holding every expert (parity: ATorch moe tests)."""

import os

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import free_port


def _ref_and_inputs():
    from dlrover_wuqiong_amd.parallel.moe import MoELayer

    torch.manual_seed(0)
    ref = MoELayer(16, 32, num_experts=4, top_k=2)
    xs = [torch.randn(10, 16) for _ in range(2)]
    return ref, xs


def test_moe_single_process_matches_dense_loop():
    ref, xs = _ref_and_inputs()
    x = xs[0]
    y = ref(x)
    w, idx, _ = ref.gate(x)
    e = ref.experts
    want = torch.zeros_like(y)
    for t in range(x.shape[0]):
        for j in range(2):
            ex = int(idx[t, j])
            h = torch.nn.functional.silu(x[t] @ e.w1[ex].T) * (x[t] @ e.w3[ex].T)
            want[t] += w[t, j] * (h @ e.w2[ex].T)
    assert torch.allclose(y, want, atol=1e-5)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dlrover_wuqiong_amd.parallel.moe import MoELayer

        ref, xs = _ref_and_inputs()
        yref = ref(torch.cat(xs))
        (yref.square().sum() + ref.aux_loss * 0).backward()
        layer = MoELayer(16, 32, num_experts=4, top_k=2, ep_group=dist.group.WORLD)
        with torch.no_grad():
            layer.gate.wg.weight.copy_(ref.gate.wg.weight)
            for n in ("w1", "w2", "w3"):
                getattr(layer.experts, n).copy_(getattr(ref.experts, n)[2 * rank:2 * rank + 2])
        y = layer(xs[rank])
        ok = torch.allclose(y, yref[10 * rank:10 * rank + 10], atol=1e-5)
        y.square().sum().backward()
        for n in ("w1", "w2", "w3"):
            ok &= torch.allclose(getattr(layer.experts, n).grad, getattr(ref.experts, n).grad[2 * rank:2 * rank + 2],
                                 atol=1e-4)
        g = layer.gate.wg.weight.grad.clone()
        dist.all_reduce(g)
        ok &= torch.allclose(g, ref.gate.wg.weight.grad, atol=1e-4)
        q.put((rank, bool(ok)))
    except Exception as e:  # pragma: no cover
        import traceback

        traceback.print_exc()
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def test_moe_expert_parallel_two_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=180) for _ in ps)
    for p in ps:
        p.join(timeout=30)
    assert res == [(0, True), (1, True)], res


class _DenseMoE(torch.nn.Module):
    def __init__(self, ep_group=None):
        super().__init__()
        from dlrover_wuqiong_amd.parallel.moe import MoELayer

        self.proj = torch.nn.Linear(16, 16)
        self.moe = MoELayer(16, 32, num_experts=4, top_k=2, ep_group=ep_group)

    def forward(self, x):
        return self.moe(self.proj(x))


def _ddp_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dlrover_wuqiong_amd.parallel.moe_ddp import MoEDistributedDataParallel, expert_data_parallel_group

        torch.manual_seed(0)
        ref = _DenseMoE()
        xs = [torch.randn(10, 16, generator=torch.Generator().manual_seed(50 + r)) for r in range(world)]
        # the objective: mean over the 4 data ranks of each rank's batch-mean loss
        sum(ref(x).square().mean() for x in xs).div(world).backward()
        ep_groups = [dist.new_group([0, 1]), dist.new_group([2, 3])]
        ep = ep_groups[rank // 2]
        edp = expert_data_parallel_group(2)
        m = _DenseMoE(ep_group=ep)
        lo = 2 * (rank % 2)
        with torch.no_grad():
            m.proj.load_state_dict(ref.proj.state_dict())
            m.moe.gate.wg.weight.copy_(ref.moe.gate.wg.weight)
            for n in ("w1", "w2", "w3"):
                getattr(m.moe.experts, n).copy_(getattr(ref.moe.experts, n)[lo:lo + 2])
        ddp = MoEDistributedDataParallel(m, expert_dp_group=edp)
        opt = ddp.attach_optimizer(torch.optim.SGD(m.parameters(), lr=0.0))
        ddp(xs[rank]).square().mean().backward()
        opt.step()  # waits for the expert all-reduces
        ok = torch.allclose(m.proj.weight.grad, ref.proj.weight.grad, atol=1e-5)
        ok &= torch.allclose(m.moe.gate.wg.weight.grad, ref.moe.gate.wg.weight.grad, atol=1e-5)
        for n in ("w1", "w2", "w3"):
            ok &= torch.allclose(getattr(m.moe.experts, n).grad, getattr(ref.moe.experts, n).grad[lo:lo + 2],
                                 atol=1e-5)
        q.put((rank, bool(ok)))
    except Exception as e:  # pragma: no cover
        import traceback

        traceback.print_exc()
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def test_moe_ddp_expert_grads_over_expert_dp_group_four_ranks():
    """EP 2 x DP 2: dense grads averaged over all 4 ranks by DDP, expert
    grads summed over the 2 replicas holding the same experts and scaled by
    1/4 -- both equal the single-process gradient of the mean loss (plain
    DDP over the world would average different experts together)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_ddp_worker, args=(r, 4, port, q)) for r in range(4)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=180) for _ in ps)
    for p in ps:
        p.join(timeout=30)
    assert res == [(r, True) for r in range(4)], res


def test_moe_capacity_drops_overflow_and_matches_reference():
    """Capacity (GShard priority): dropped assignments contribute nothing,
    kept ones equal the dropless layer's per-expert outputs."""
    from dlrover_wuqiong_amd.parallel.moe import MoELayer, capacity_mask

    idx = torch.tensor([[0, 1], [0, 2], [0, 1], [3, 0]])
    keep = capacity_mask(idx, 4, 2)
    # first choices in token order: t0->0, t1->0, t2->0 (3rd: dropped), t3->3;
    # then second choices: t0->1, t1->2, t2->1, t3->0 (expert 0 full)
    assert keep.tolist() == [[True, True], [True, True], [False, True], [True, False]]
    torch.manual_seed(0)
    free = MoELayer(16, 32, num_experts=4, top_k=2)
    capped = MoELayer(16, 32, num_experts=4, top_k=2, capacity_factor=0.5)
    capped.load_state_dict(free.state_dict())
    x = torch.randn(24, 16, requires_grad=True)
    y = capped(x)
    w, idx, _ = free.gate(x)
    keep = capacity_mask(idx, 4, 6)  # capacity ceil(0.5 * 24 * 2 / 4) = 6
    e = free.experts
    want = torch.zeros_like(y)
    for t in range(24):
        for j in range(2):
            if keep[t, j]:
                ex = int(idx[t, j])
                h = torch.nn.functional.silu(x[t] @ e.w1[ex].T) * (x[t] @ e.w3[ex].T)
                want[t] += w[t, j] * (h @ e.w2[ex].T)
    assert int((~keep).sum()) > 0 and torch.allclose(y, want, atol=1e-5)
    y.square().sum().backward()
    assert torch.isfinite(x.grad).all()


def test_replace_with_moe_upcycles_dense_ffn():
    """Upcycled experts are copies of the dense FFN and the router starts
    uniform: the MoE model computes the dense model's output."""
    from dlrover_wuqiong_amd.models.llama import Llama, LlamaConfig, LlamaMLP
    from dlrover_wuqiong_amd.parallel.moe import MoELayer, replace_with_moe

    torch.manual_seed(0)
    cfg = LlamaConfig.named("llama-tiny")
    m = Llama(cfg)
    ids = torch.randint(0, cfg.vocab_size, (2, 16))
    dense = m(ids).detach()
    names = replace_with_moe(m, LlamaMLP, num_experts=4, top_k=2)
    assert len(names) == cfg.num_hidden_layers and all(isinstance(l.mlp, MoELayer) for l in m.layers)
    assert torch.allclose(m(ids), dense, atol=1e-4)


def _empty_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dlrover_wuqiong_amd.parallel.moe import MoELayer

        torch.manual_seed(0)
        layer = MoELayer(16, 32, num_experts=4, top_k=2, ep_group=dist.group.WORLD)
        with torch.no_grad():
            layer.gate.wg.weight.zero_()  # ties: every token to the same 2 experts -> one rank gets nothing
        x = torch.randn(10, 16, requires_grad=True)
        layer(x).square().sum().backward()  # must not desynchronise the inverse all-to-all
        q.put((rank, bool(torch.isfinite(x.grad).all())))
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def test_moe_ep_rank_receiving_no_tokens_two_ranks():
    """An EP rank whose experts get no token still runs the backward's
    inverse all-to-all (the empty expert output keeps its input in the graph)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_empty_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=30)
    assert res == [(0, True), (1, True)], res
