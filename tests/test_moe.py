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
