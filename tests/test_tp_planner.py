"""Graph-traced tensor-parallel planning (atorch/tp_planner.py): Megatron
column -> row blocks are found by data flow, not by layer names; head counts
hard-coded in views shrink with the shards; the sharded model (2 gloo ranks,
DTensor) computes exactly what the unsharded one does (parity: ATorch
tp_compiler.py graph-traced sharding)."""

import os

import torch
import torch.multiprocessing as mp
import torch.nn as nn
import torch.nn.functional as F

from conftest import free_port


class Attn(nn.Module):
    def __init__(self, h=32, nh=4):
        super().__init__()
        self.nh = nh
        self.to_q, self.to_k, self.to_v, self.out = (nn.Linear(h, h) for _ in range(4))

    def forward(self, x):
        B, S, H = x.shape
        q = self.to_q(x).view(B, S, self.nh, -1).transpose(1, 2)
        k = self.to_k(x).view(B, S, self.nh, -1).transpose(1, 2)
        v = self.to_v(x).view(B, S, self.nh, -1).transpose(1, 2)
        a = F.scaled_dot_product_attention(q, k, v, is_causal=True)
        return self.out(a.transpose(1, 2).reshape(B, S, -1))


class MLP(nn.Module):
    def __init__(self, h=32):
        super().__init__()
        self.alpha, self.gamma = nn.Linear(h, 4 * h), nn.Linear(h, 4 * h)
        self.beta = nn.Linear(4 * h, h)

    def forward(self, x):
        return self.beta(F.silu(self.alpha(x)) * self.gamma(x))


class Block(nn.Module):
    def __init__(self):
        super().__init__()
        self.n1, self.att, self.n2, self.mlp = nn.LayerNorm(32), Attn(), nn.LayerNorm(32), MLP()

    def forward(self, x):
        x = x + self.att(self.n1(x))
        return x + self.mlp(self.n2(x))


class Net(nn.Module):
    def __init__(self):
        super().__init__()
        self.emb = nn.Embedding(50, 32)
        self.blocks = nn.ModuleList([Block(), Block()])
        self.head = nn.Linear(32, 50)

    def forward(self, ids):
        x = self.emb(ids)
        for b in self.blocks:
            x = b(x)
        return self.head(x)


def test_planner_finds_blocks_by_data_flow():
    from dlrover_wuqiong_amd.atorch.tp_planner import trace_tp_plan

    heads = {}
    plan = trace_tp_plan(Net(), heads)
    for i in (0, 1):
        for n in ("to_q", "to_k", "to_v"):
            assert plan[f"blocks.{i}.att.{n}"] == "colwise"
        assert plan[f"blocks.{i}.att.out"] == "rowwise"
        assert plan[f"blocks.{i}.mlp.alpha"] == plan[f"blocks.{i}.mlp.gamma"] == "colwise"
        assert plan[f"blocks.{i}.mlp.beta"] == "rowwise"
    assert "head" not in plan  # fed by the residual stream: stays replicated
    assert heads == {"blocks.0.att": {4}, "blocks.1.att": {4}}


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    from dlrover_wuqiong_amd.atorch import distributed as adist

    try:
        from dlrover_wuqiong_amd.atorch.auto_accelerate import auto_accelerate

        adist.init_distributed("gloo")
        torch.manual_seed(0)
        ref = Net()
        model = Net()
        model.load_state_dict(ref.state_dict())
        ok, res, _s = auto_accelerate(model, load_strategy=[("parallel_mode", ([("tensor", 2)], None)),
                                                            "tensor_parallel"])
        m = res.model.module if hasattr(res.model, "module") else res.model
        ids = torch.randint(0, 50, (2, 9), generator=torch.Generator().manual_seed(1))
        out = res.model(ids)
        same = torch.allclose(out, ref(ids), atol=1e-5)
        sharded = m.blocks[0].mlp.alpha.weight.to_local().shape[0] == 64 and m.blocks[0].att.nh == 2
        q.put((rank, bool(ok and same and sharded)))
    except Exception as e:  # pragma: no cover
        import traceback

        traceback.print_exc()
        q.put((rank, repr(e)))
    finally:
        adist.reset_distributed()


def test_two_rank_auto_tp_matches_unsharded():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(timeout=30)
    assert res == [(0, True), (1, True)], res
