"""Automatic tensor x pipeline x data sizing (atorch/shard_planner.py;
parity: ATorch shard_planners/dim_planner.py): MI355X cost model decisions
for reference configurations, and ``("mixed_parallel", "auto")`` through
auto_accelerate on 8 gloo ranks."""

import os

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import free_port
from dlrover_wuqiong_amd.atorch.shard_planner import Hardware, ModelShape, estimate, plan_3d

L70 = ModelShape(layers=80, hidden=8192, intermediate=28672, heads=64, kv_heads=8, vocab=128256,
                 params=70_553_706_496)
L8 = ModelShape(layers=32, hidden=4096, intermediate=14336, heads=32, kv_heads=8, vocab=128256,
                params=8_030_261_248)


def test_llama70b_on_one_node_needs_model_parallel():
    plans = plan_3d(None, 8, seq=4096, micro_batch=1, global_batch=32, shape=L70)
    best = plans[0]
    assert best.feasible and best.tensor * best.pipeline > 1  # pure DP cannot hold 70B + Adam
    dp_only = next(p for p in plans if p.tensor == 1 and p.pipeline == 1)
    assert not dp_only.feasible and dp_only.mem_gb > 288
    assert best.mem_gb <= 288 - 24
    # every factorisation of 8 is considered, feasible ones first
    assert {(p.tensor, p.pipeline, p.data) for p in plans} >= {(8, 1, 1), (1, 8, 1), (2, 4, 1), (4, 2, 1)}
    assert all(a.feasible >= b.feasible for a, b in zip(plans, plans[1:]))


def test_llama8b_fits_data_parallel():
    best = plan_3d(None, 8, seq=4096, micro_batch=1, global_batch=32, shape=L8)[0]
    assert best.feasible and (best.tensor, best.pipeline, best.data) == (1, 1, 8)


def test_cost_terms_move_the_right_way():
    hw = Hardware()
    a = estimate(L70, 8, 1, 1, 4096, 1, 32, hw)
    b = estimate(L70, 4, 2, 1, 4096, 1, 32, hw)
    assert a.parts["tp"] > b.parts["tp"] > 0 and b.parts["bubble"] > a.parts["bubble"] == 0
    # more micro-batches shrink the bubble
    c = estimate(L70, 1, 8, 1, 4096, 1, 64, hw)
    d = estimate(L70, 1, 8, 1, 4096, 1, 16, hw)
    assert c.parts["bubble"] / c.parts["compute"] < d.parts["bubble"] / d.parts["compute"]
    # across nodes the data-parallel all-reduce slows down
    e = plan_3d(None, 64, seq=4096, micro_batch=1, global_batch=256, shape=L8)
    assert e[0].feasible


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    torch.set_num_threads(1)
    from dlrover_wuqiong_amd.atorch import distributed as adist

    try:
        from dlrover_wuqiong_amd.atorch.auto_accelerate import auto_accelerate
        from dlrover_wuqiong_amd.models.llama import Llama, LlamaConfig

        adist.init_distributed("gloo")
        cfg = LlamaConfig.named("llama-tiny")
        cfg.num_hidden_layers, cfg.vocab_size = 4, 256
        torch.manual_seed(0)
        # sizes left to the planner (the tiny model fits plain data parallel)
        ok, res, strat = auto_accelerate(Llama(cfg), torch.optim.SGD, optim_args={"lr": 0.1},
                                         fused_optimizer=False,
                                         load_strategy=[("mixed_parallel", {"auto": True, "seq_len": 16,
                                                                            "micro_batch": 1, "global_batch": 8})])
        m = dict(strat.opts)["mixed_parallel"]
        q.put((rank, (m["tensor"], m["pipeline"], m["data"])))
    except Exception as e:  # pragma: no cover
        import traceback

        traceback.print_exc()
        q.put((rank, repr(e)))
    finally:
        adist.reset_distributed()


def test_auto_mixed_parallel_through_auto_accelerate():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_worker, args=(r, 8, port, q)) for r in range(8)]
    for p in ps:
        p.start()
    res = sorted((q.get(timeout=300) for _ in ps), key=lambda x: x[0])
    for p in ps:
        p.join(timeout=60)
    sizes = {r[1] for r in res}
    assert len(sizes) == 1 and isinstance(next(iter(sizes)), tuple), res
    t, p, d = next(iter(sizes))
    assert (t, p, d) == (1, 1, 8)
