"""TP x PP x DP in ONE auto_accelerate strategy (8 gloo ranks: tensor 2 x
pipeline 2 x data 2) on a small Llama: the loss of two training steps
matches a single process training the unsplit model on the global batch
(parity: ATorch mixed_parallel_optimization.py:32 / ds_3d_parallel).
And local SGD inside HSDP (4 ranks: 2 replicas x 2 shards): replicas drift
between syncs and agree after each one; the sync applies the outer
optimizer to the averaged pseudo-gradient (ATorch local_sgd/HSDP)."""

import copy
import os

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import free_port


def _llama():
    from dlrover_wuqiong_amd.models.llama import Llama, LlamaConfig

    cfg = LlamaConfig.named("llama-tiny")
    cfg.num_hidden_layers = 4
    cfg.vocab_size = 256
    torch.manual_seed(0)
    return Llama(cfg)


def _batch(step):
    g = torch.Generator().manual_seed(100 + step)
    ids = torch.randint(0, 256, (4, 17), generator=g)
    return ids[:, :-1], ids[:, 1:]


def _mixed_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    from dlrover_wuqiong_amd.atorch import distributed as adist

    try:
        from dlrover_wuqiong_amd.atorch.auto_accelerate import auto_accelerate

        adist.init_distributed("gloo")
        model = _llama()
        ok, res, strat = auto_accelerate(model, torch.optim.SGD, optim_args={"lr": 0.5},
                                         load_strategy=[("ds_3d_parallel", {"tensor": 2, "pipeline": 2, "data": 2,
                                                                            "chunks": 2})],
                                         fused_optimizer=False)
        pipe = res.model
        dr = adist.parallel_rank("data")
        losses = []
        for step in range(2):
            ids, tgt = _batch(step)
            ids, tgt = ids[2 * dr: 2 * dr + 2], tgt[2 * dr: 2 * dr + 2]  # this data replica's half
            res.optim.zero_grad()
            loss = pipe.train_step(ids if pipe.stage == 0 else None, tgt)
            res.optim.step()
            losses.append(float(loss) if pipe.stage == pipe.num_stages - 1 else 0.0)
        t = torch.tensor(losses, dtype=torch.float64)
        dist.all_reduce(t)  # last-stage ranks: 2 tensor x 2 data replicas hold a loss each
        q.put((rank, ("ok", (t / 4).tolist(), "mixed_parallel" in strat.names())))
    except Exception as e:  # pragma: no cover
        import traceback

        traceback.print_exc()
        q.put((rank, repr(e)))
    finally:
        adist.reset_distributed()


def test_eight_rank_tp2_pp2_dp2_loss_parity():
    ref = _llama()
    opt = torch.optim.SGD(ref.parameters(), lr=0.5)
    ref_losses = []
    for step in range(2):
        ids, tgt = _batch(step)
        opt.zero_grad()
        loss = ref(ids, tgt)
        loss.backward()
        opt.step()
        ref_losses.append(float(loss))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_mixed_worker, args=(r, 8, port, q)) for r in range(8)]
    for p in ps:
        p.start()
    res = sorted((q.get(timeout=300) for _ in ps), key=lambda x: x[0])
    for p in ps:
        p.join(timeout=60)
    assert all(isinstance(r[1], tuple) and r[1][0] == "ok" and r[1][2] for r in res), res
    got = res[0][1][1]
    assert all(abs(a - b) < 2e-4 for a, b in zip(got, ref_losses)), (got, ref_losses)
    assert got[1] < got[0]


def _lsgd_worker(rank, world, port, q, warmup=1, per_rank_init=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    from dlrover_wuqiong_amd.atorch import distributed as adist

    try:
        from dlrover_wuqiong_amd.atorch.auto_accelerate import auto_accelerate
        from dlrover_wuqiong_amd.models.llama import LlamaDecoderLayer

        adist.init_distributed("gloo")
        model = _llama()
        if per_rank_init:  # every rank its own random init: the wrapper must sync the replicas
            torch.manual_seed(1000 + rank)
            for p_ in model.parameters():
                p_.data.normal_(0, 0.02)
        ok, res, strat = auto_accelerate(
            model, torch.optim.AdamW, optim_args={"lr": 1e-2}, fused_optimizer=False,
            load_strategy=[("parallel_mode", ([("zero", 2), ("data", 2)], None)),
                           ("fsdp", {"wrap_cls": (LlamaDecoderLayer,), "use_local_sgd": True,
                                     "local_sgd_sync_interval": 2, "local_sgd_warmup_steps": warmup,
                                     "outer_optim_class": torch.optim.SGD,
                                     "outer_optim_kwargs": {"lr": 0.7, "momentum": 0.9, "nesterov": True}})])
        opt = res.optim
        rg = opt.group
        flat = opt._flat()
        other = [torch.zeros_like(flat) for _ in range(dist.get_world_size(rg))]
        dist.all_gather(other, flat, group=rg)
        states = [(0, all(torch.equal(o, other[0]) for o in other), 0, False)]
        for step in range(5):
            ids, tgt = _batch(step)
            ids, tgt = ids[rank: rank + 1], tgt[rank: rank + 1]  # every rank its own sample
            opt.zero_grad()
            res.model(ids, tgt).backward()
            before_sync = None
            if opt.anchor is not None and (opt.step_count + 1 - opt.warmup_steps) % opt.sync_interval == 0:
                # the sync this step will do: outer SGD on the mean pseudo-gradient
                before_sync = opt.anchor.data.clone()
            opt.step()
            flat = opt._flat()
            other = [torch.zeros_like(flat) for _ in range(dist.get_world_size(rg))]
            dist.all_gather(other, flat, group=rg)
            same = all(torch.equal(o, other[0]) for o in other)
            states.append((opt.step_count, same, opt.syncs, before_sync is not None))
        q.put((rank, states))
    except Exception as e:  # pragma: no cover
        import traceback

        traceback.print_exc()
        q.put((rank, repr(e)))
    finally:
        adist.reset_distributed()


def test_four_rank_hsdp_local_sgd():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_lsgd_worker, args=(r, 4, port, q)) for r in range(4)]
    for p in ps:
        p.start()
    res = sorted((q.get(timeout=300) for _ in ps), key=lambda x: x[0])
    for p in ps:
        p.join(timeout=60)
    for _r, states in res:
        assert isinstance(states, list), res
        # step 1: warm-up (HSDP all-reduce) -> replicas equal; then local
        # steps 2 (drift), 3 (sync), 4 (drift), 5 (sync)
        assert [s[1] for s in states] == [True, True, False, True, False, True], states
        assert states[-1][2] == 2


def test_four_rank_hsdp_local_sgd_per_rank_init_no_warmup():
    """warmup_steps=0 and a different random init on every rank: the
    replicas still start from one model and agree after every sync."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_lsgd_worker, args=(r, 4, port, q, 0, True)) for r in range(4)]
    for p in ps:
        p.start()
    res = sorted((q.get(timeout=300) for _ in ps), key=lambda x: x[0])
    for p in ps:
        p.join(timeout=60)
    for _r, states in res:
        assert isinstance(states, list), res
        # init synced; local steps 1 (drift), 2 (sync), 3 (drift), 4 (sync), 5 (drift)
        assert [s[1] for s in states] == [True, False, True, False, True, False], states
