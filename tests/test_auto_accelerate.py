"""auto_accelerate strategies on CPU: single process (module_replace, amp,
checkpoint, planner) and 2 ranks (ddp, fsdp, zero1, tensor_parallel)
(parity: ATorch tests/auto/test_auto_accelerate.py)."""

import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn
import torch.nn.functional as F

from conftest import free_port


class Block(nn.Module):
    def __init__(self, h=32, heads=4):
        super().__init__()
        self.num_heads = heads
        self.norm = nn.LayerNorm(h)
        self.q_proj, self.k_proj, self.v_proj = nn.Linear(h, h), nn.Linear(h, h), nn.Linear(h, h)
        self.o_proj = nn.Linear(h, h)
        self.up_proj, self.down_proj = nn.Linear(h, 4 * h), nn.Linear(4 * h, h)

    def forward(self, x):
        B, S, H = x.shape
        y = self.norm(x)
        q, k, v = (p(y).view(B, S, self.num_heads, -1).transpose(1, 2) for p in (self.q_proj, self.k_proj, self.v_proj))
        a = F.scaled_dot_product_attention(q, k, v, is_causal=True).transpose(1, 2).reshape(B, S, -1)
        x = x + self.o_proj(a)
        return x + self.down_proj(F.gelu(self.up_proj(x)))


class Toy(nn.Module):
    def __init__(self):
        super().__init__()
        self.emb = nn.Embedding(64, 32)
        self.layers = nn.ModuleList([Block(), Block()])
        self.head = nn.Linear(32, 64)

    def forward(self, ids):
        x = self.emb(ids)
        for b in self.layers:
            x = b(x)
        return self.head(x)


class DS(torch.utils.data.Dataset):
    def __len__(self):
        return 32

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(i)
        ids = torch.randint(0, 64, (9,), generator=g)
        return {"ids": ids[:-1], "labels": ids[1:]}


def loss_func(batch, out):
    return F.cross_entropy(out.reshape(-1, 64).float(), batch["labels"].reshape(-1))


def _train(result, steps=4):
    import itertools

    losses = []
    it = itertools.cycle(result.dataloader)
    for _ in range(steps):
        b = result.prepare_input(next(it), result.args["device"])
        loss = result.loss_func(b, result.model(b["ids"]))
        result.optim.zero_grad()
        loss.backward()
        result.optim.step()
        losses.append(float(loss.detach()))
    return losses


def test_single_process_strategies():
    from dlrover_wuqiong_amd.atorch.auto_accelerate import auto_accelerate
    from dlrover_wuqiong_amd.ops.norm import LayerNorm

    torch.manual_seed(0)
    ok, res, strat = auto_accelerate(
        Toy(), torch.optim.AdamW, dataset=DS(), loss_func=loss_func, optim_args={"lr": 1e-2},
        dataloader_args={"batch_size": 8},
        load_strategy=["module_replace", ("amp_native", {"dtype": torch.bfloat16}), "checkpoint"])
    assert ok and strat.names() == ["module_replace", "amp_native", "checkpoint"]
    assert any(isinstance(m, LayerNorm) for m in res.model.modules())
    losses = _train(res, 6)
    assert losses[-1] < losses[0]
    # semi-automatic planner
    ok, res2, strat2 = auto_accelerate(Toy(), torch.optim.SGD, optim_args={"lr": 0.1})
    assert "amp_native" in strat2.names() and res2.optim is not None


def _worker(rank, world, port, strategy, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    try:
        from dlrover_wuqiong_amd.atorch import distributed as adist
        from dlrover_wuqiong_amd.atorch.auto_accelerate import auto_accelerate

        adist.init_distributed("gloo")
        torch.manual_seed(0)
        ok, res, strat = auto_accelerate(Toy(), torch.optim.AdamW, dataset=DS(), loss_func=loss_func,
                                         optim_args={"lr": 1e-2}, dataloader_args={"batch_size": 8},
                                         load_strategy=strategy)
        losses = _train(res, 5)
        good = ok and losses[-1] < losses[0] and len(res.dataloader) == 32 // 8
        q.put((rank, bool(good), strat.names()))
    except Exception as e:  # pragma: no cover
        import traceback

        traceback.print_exc()
        q.put((rank, repr(e), None))
    finally:
        adist.reset_distributed()


def _run(strategy):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, strategy, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted((q.get(timeout=240) for _ in ps), key=lambda x: x[0])
    for p in ps:
        p.join(timeout=30)
    return res


def test_two_rank_ddp_fsdp_zero1():
    for strategy in (["parallel_mode", "ddp"], ["parallel_mode", "fsdp"], ["parallel_mode", "zero1"]):
        res = _run(strategy)
        assert [r[1] for r in res] == [True, True], (strategy, res)


def test_two_rank_tensor_parallel():
    res = _run([("parallel_mode", ([("tensor", 2)], None)), "tensor_parallel"])
    assert [r[1] for r in res] == [True, True], res


def _llama_fsdp_ckpt_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from dlrover_wuqiong_amd.atorch import distributed as adist

    try:
        from torch.distributed.algorithms._checkpoint.checkpoint_wrapper import CheckpointWrapper
        from torch.distributed.fsdp import FSDPModule

        from dlrover_wuqiong_amd.atorch.auto_accelerate import auto_accelerate
        from dlrover_wuqiong_amd.models.llama import Llama, LlamaConfig, LlamaDecoderLayer

        adist.init_distributed("gloo")
        torch.manual_seed(0)
        model = Llama(LlamaConfig.named("llama-tiny"))
        ok, res, _ = auto_accelerate(
            model, torch.optim.AdamW, optim_args={"lr": 1e-3},
            load_strategy=["module_replace", ("amp_native", {"dtype": torch.bfloat16}),
                           ("fsdp", {"wrap_cls": (LlamaDecoderLayer,)}),
                           ("checkpoint", {"wrap_cls": (LlamaDecoderLayer,)})])
        # FSDP must wrap the CheckpointWrapper (inputs cast once, outside the
        # recomputed region), never the layer inside it
        wrapped = [m for m in res.model.modules() if isinstance(m, CheckpointWrapper)]
        nested_ok = bool(wrapped) and all(isinstance(m, FSDPModule) for m in wrapped) and not any(
            isinstance(m, FSDPModule) for m in res.model.modules() if isinstance(m, LlamaDecoderLayer))
        g = torch.Generator().manual_seed(rank)
        ids = torch.randint(0, 1024, (2, 65), generator=g)
        losses = []
        for _ in range(3):
            loss = res.model(ids[:, :-1], ids[:, 1:])
            loss.backward()  # recompute must match the checkpointed forward
            res.optim.step()
            res.optim.zero_grad(set_to_none=True)
            losses.append(float(loss))
        # nested wrap classes: every DecoderLayer AND every MLP inside it is its own FSDP unit
        from dlrover_wuqiong_amd.models.llama import LlamaMLP

        torch.manual_seed(0)
        m2 = Llama(LlamaConfig.named("llama-tiny"))
        ok2, res2, _ = auto_accelerate(m2, torch.optim.AdamW, optim_args={"lr": 1e-3},
                                       load_strategy=[("fsdp", {"wrap_cls": (LlamaDecoderLayer, LlamaMLP)})])
        units = [m for m in res2.model.modules() if isinstance(m, FSDPModule)]
        nlayers = LlamaConfig.named("llama-tiny").num_hidden_layers
        nested_ok = nested_ok and ok2 and sum(isinstance(m, LlamaMLP) for m in units) == nlayers and \
            sum(isinstance(m, LlamaDecoderLayer) for m in units) == nlayers
        loss = res2.model(ids[:, :-1], ids[:, 1:])
        loss.backward()
        res2.optim.step()
        q.put((rank, bool(ok and nested_ok and all(x == x for x in losses))))
    except Exception as e:  # pragma: no cover
        import traceback

        traceback.print_exc()
        q.put((rank, repr(e)))
    finally:
        adist.reset_distributed()


def test_two_rank_llama_fsdp_with_activation_checkpointing():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_llama_fsdp_ckpt_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted((q.get(timeout=240) for _ in ps), key=lambda x: x[0])
    for p in ps:
        p.join(timeout=30)
    assert [r[1] for r in res] == [True, True], res


def _hsdp_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    from dlrover_wuqiong_amd.atorch import distributed as adist

    try:
        from torch.distributed.tensor import Replicate, Shard

        from dlrover_wuqiong_amd.atorch.auto_accelerate import auto_accelerate

        adist.init_distributed("gloo")
        torch.manual_seed(0)
        ok, res, strat = auto_accelerate(
            Toy(), torch.optim.AdamW, dataset=DS(), loss_func=loss_func, optim_args={"lr": 1e-2},
            dataloader_args={"batch_size": 8},
            load_strategy=[("parallel_mode", ([("zero", 2), ("data", 2)], None)), ("fsdp", {"wrap_cls": (Block,)})])
        p = next(res.model.parameters())
        placements_ok = tuple(p.placements) == (Replicate(), Shard(0)) and p.device_mesh.ndim == 2
        losses = _train(res, 5)
        sums = torch.tensor([float(sum(v.full_tensor().double().sum() for v in res.model.state_dict().values()))],
                            dtype=torch.float64)
        allsums = [torch.zeros_like(sums) for _ in range(world)]
        dist.all_gather(allsums, sums)
        same = all(torch.equal(s, allsums[0]) for s in allsums)
        q.put((rank, bool(ok and placements_ok and same and losses[-1] < losses[0] and len(res.dataloader) == 4)))
    except Exception as e:  # pragma: no cover
        import traceback

        traceback.print_exc()
        q.put((rank, repr(e)))
    finally:
        adist.reset_distributed()


def test_four_rank_hsdp():
    """("zero", 2) x ("data", 2): shard within zero groups, replicate across
    data groups (FSDP2 2-D mesh); every rank reads its own quarter of the batch."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_hsdp_worker, args=(r, 4, port, q)) for r in range(4)]
    for p in ps:
        p.start()
    res = sorted((q.get(timeout=240) for _ in ps), key=lambda x: x[0])
    for p in ps:
        p.join(timeout=30)
    assert [r[1] for r in res] == [True] * 4, res


def _sp_worker(rank, world, port, q, mode="sp"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    try:
        from dlrover_wuqiong_amd.atorch import distributed as adist
        from dlrover_wuqiong_amd.atorch.auto_accelerate import auto_accelerate
        from dlrover_wuqiong_amd.models.llama import Llama, LlamaConfig

        adist.init_distributed("gloo")

        class LM(Llama):
            def forward(self, ids, labels=None):
                return super().forward(ids, labels)

        class Tok(torch.utils.data.Dataset):
            def __len__(self):
                return 8

            def __getitem__(self, i):
                g = torch.Generator().manual_seed(i)
                ids = torch.randint(0, 1024, (17,), generator=g)
                return {"ids": ids[:-1], "labels": ids[1:]}

        def split(batch, sp_size, sp_rank):
            n = batch["ids"].shape[1] // sp_size
            return {k: v[:, sp_rank * n:(sp_rank + 1) * n] for k, v in batch.items()}

        torch.manual_seed(0)
        cfg = LlamaConfig.named("llama-tiny")
        full = LM(cfg)
        torch.manual_seed(0)
        ok, res, strat = auto_accelerate(
            LM(cfg), torch.optim.SGD, dataset=Tok(), loss_func=lambda b, out: out, optim_args={"lr": 0.1},
            dataloader_args={"batch_size": 2, "shuffle": False}, model_input_format="unpack_dict",
            load_strategy=["parallel_mode", ("sequence_parallel", {"sp_size": 2, "batch_sp_processing_fn": split})
                           if mode == "sp" else ("context_parallel", {"cp_size": 2})])
        batch = next(iter(res.dataloader))
        shard = res.prepare_input(batch, torch.device("cpu"))
        loss = res.model(**shard)
        # both SP ranks got the same batch; the mean of their shard losses is the full-sequence loss
        lt = loss.detach().clone()
        dist.all_reduce(lt)
        ref = full(batch["ids"], batch["labels"])
        q.put((rank, bool(abs(float(lt) / 2 - float(ref)) < 1e-4 and shard["ids"].shape[1] == 8
                          and len(res.dataloader) == 4), strat.names()))
    except Exception as e:  # pragma: no cover
        import traceback

        traceback.print_exc()
        q.put((rank, repr(e), None))
    finally:
        adist.reset_distributed()


@pytest.mark.parametrize("mode", ["sp", "cp"])
def test_two_rank_sequence_parallel_strategy(mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_sp_worker, args=(r, 2, port, q, mode)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted((q.get(timeout=240) for _ in ps), key=lambda x: x[0])
    for p in ps:
        p.join(timeout=30)
    assert all(r[1] is True for r in res), res
