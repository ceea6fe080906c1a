"""Flat-unit FSDP (parallel/flat_fsdp.py) on gloo: training equals one
process on the whole batch (world 1 and 2, with and without resharding after
the forward, global-norm clipping and weight decay), gradient accumulation
under no_sync, the auto_accelerate strategy, and flash checkpoints in the
flat-shard format (in-place memory restore; files resharded to world 1 and
into an unsharded model).  Parity: reference atorch FSDP (FlatParameter)
training / fsdp_save_util tests (behaviour)."""

import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import free_port

STEPS = 3


def _gpt2():
    from dlrover_wuqiong_amd.models.gpt2 import GPT2, GPT2Config

    torch.manual_seed(0)
    cfg = GPT2Config.named("gpt2-tiny")
    return GPT2(cfg), cfg


def _data(cfg, n=STEPS, rows=4):
    g = torch.Generator().manual_seed(1)
    return [torch.randint(0, cfg.vocab_size, (rows, 33), generator=g) for _ in range(n)]


def _reference(micro=1):
    """One process, the whole batch split into ``micro`` accumulated
    micro-batches (one per rank and micro-step of the sharded run),
    FlatParams + FusedAdamW."""
    from dlrover_wuqiong_amd.optimizers.fused import FusedAdamW
    from dlrover_wuqiong_amd.parallel.flat import FlatParams

    m, cfg = _gpt2()
    flat = FlatParams(m)
    opt = FusedAdamW(flat, lr=1e-2, weight_decay=0.05, max_grad_norm=0.5)
    opt.grad_scale = 1.0 / micro
    losses = []
    for x in _data(cfg):
        tot = 0.0
        for xm in x.chunk(micro):
            loss = m(xm[:, :-1], xm[:, 1:])
            loss.backward()
            tot += float(loss.detach())
        opt.step()
        flat.zero_grad()
        losses.append(tot / micro)
    return losses, {n: p.detach().clone() for n, p in m.named_parameters()}


def _train_worker(rank, world, port, reshard, micro, act_ckpt, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dlrover_wuqiong_amd.models.gpt2 import Block
        from dlrover_wuqiong_amd.optimizers.fused import FusedAdamW
        from dlrover_wuqiong_amd.parallel.flat_fsdp import FlatFSDP

        m, cfg = _gpt2()
        if act_ckpt:  # recomputed in the backward, after the unit's storage was released
            from torch.distributed.algorithms._checkpoint.checkpoint_wrapper import (
                apply_activation_checkpointing, checkpoint_wrapper)

            apply_activation_checkpointing(m, checkpoint_wrapper_fn=checkpoint_wrapper,
                                           check_fn=lambda mod: isinstance(mod, Block))
        model = FlatFSDP(m, wrap_cls=(Block,), reshard_after_forward=reshard)
        opt = FusedAdamW(model.shard_flat, lr=1e-2, weight_decay=0.05, max_grad_norm=0.5)
        opt.grad_scale = 1.0 / (world * micro)  # summed over ranks and accumulated micro-batches
        losses = []
        for x in _data(cfg):
            mine = x.chunk(world)[rank].chunk(micro)
            tot = torch.zeros(())
            for j, xm in enumerate(mine):
                if j < len(mine) - 1:
                    with model.no_sync():
                        loss = model(xm[:, :-1], xm[:, 1:])
                        loss.backward()
                else:
                    loss = model(xm[:, :-1], xm[:, 1:])
                    loss.backward()
                tot += loss.detach()
            opt.step()
            opt.zero_grad()
            dist.all_reduce(tot)
            losses.append(float(tot) / (world * micro))
        sd = model.full_state_dict()
        released = [u.released and u.grad_released and u.gfull.untyped_storage().size() == 0
                    for u in model.units if not u.is_root]
        if rank == 0:
            q.put((losses, {k: v.float().numpy() for k, v in sd.items()}, released))
        else:
            q.put(None)
    except Exception as e:  # pragma: no cover
        import traceback

        traceback.print_exc()
        q.put(repr(e))
    finally:
        dist.destroy_process_group()


def _spawn(target, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=target, args=(r, world, port) + args + (q,)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=240) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    errs = [r for r in res if isinstance(r, str)]
    assert not errs, errs
    return [r for r in res if r is not None]


@pytest.mark.parametrize("world,reshard,micro,act_ckpt", [(1, False, 1, False), (2, False, 1, False),
                                                         (2, True, 1, False), (2, True, 2, False),
                                                         (2, True, 1, True), (4, True, 1, False)])
def test_flat_fsdp_matches_one_process(world, reshard, micro, act_ckpt):
    ref_losses, ref_params = _reference(micro=world * micro)
    (losses, params, released), = _spawn(_train_worker, world, reshard, micro, act_ckpt)
    assert losses == pytest.approx(ref_losses, rel=1e-5, abs=1e-5)
    for n, p in ref_params.items():
        torch.testing.assert_close(torch.from_numpy(params[_plain(n, params)]), p, rtol=2e-4, atol=2e-4, msg=n)
    # ZeRO-3: the layers' gathered parameters and unsharded gradients are released between steps
    assert all(released) == (reshard and world > 1)


def _plain(name, params):
    """``name`` as the (possibly activation-checkpoint-wrapped) model spells it."""
    if name in params:
        return name
    for k in params:
        if k.replace("_checkpoint_wrapped_module.", "") == name:
            return k
    raise KeyError(name)


def test_flat_fsdp_world1_is_the_shard():
    """At world 1 the parameters ARE the shard buffer: no extra copy."""
    from dlrover_wuqiong_amd.models.gpt2 import Block
    from dlrover_wuqiong_amd.parallel.flat_fsdp import FlatFSDP

    m, _cfg = _gpt2()
    n_params = sum(p.numel() for p in m.parameters())
    model = FlatFSDP(m, wrap_cls=(Block,))
    base = model.shard_flat.data
    lo, hi = base.data_ptr(), base.data_ptr() + base.numel() * base.element_size()
    for p in m.parameters():
        assert lo <= p.data_ptr() < hi
        assert lo <= p.grad.data_ptr() - (model.shard_flat.grad.data_ptr() - lo) < hi
    assert n_params <= base.numel() < n_params + 64 * (len(model.units) + sum(1 for _ in m.parameters()))
    views, meta = model.flat_shard_tensors()
    assert set(views) == {n for n, _ in m.named_parameters()}
    assert all(mm["dim"] == -1 and mm["offset"] == 0 for mm in meta.values())


def _auto_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dlrover_wuqiong_amd.atorch.auto_accelerate import auto_accelerate
        from dlrover_wuqiong_amd.models.gpt2 import Block
        from dlrover_wuqiong_amd.optimizers.fused import FusedAdamW
        from dlrover_wuqiong_amd.parallel.flat_fsdp import FlatFSDP

        m, cfg = _gpt2()
        ok, res, _s = auto_accelerate(m, torch.optim.AdamW, optim_args={"lr": 1e-3},
                                      load_strategy=[("flat_zero2", {"wrap_cls": (Block,)})])
        assert ok and isinstance(res.model, FlatFSDP) and isinstance(res.optim, FusedAdamW)
        assert res.optim.flat is res.model.shard_flat and res.optim.grad_scale == 1.0 / world
        x = _data(cfg, 1)[0].chunk(world)[rank]
        before = float(res.model(x[:, :-1], x[:, 1:]))
        for _ in range(3):
            loss = res.model(x[:, :-1], x[:, 1:])
            loss.backward()
            res.optim.step()
            res.optim.zero_grad()
        q.put(float(loss) < before)
    except Exception as e:  # pragma: no cover
        import traceback

        traceback.print_exc()
        q.put(repr(e))
    finally:
        dist.destroy_process_group()


def test_auto_accelerate_flat_zero2_two_ranks():
    assert _spawn(_auto_worker, 2) == [True, True]


def _ckpt_worker(rank, world, port, root, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dlrover_wuqiong_amd.atorch import fsdp_flat_ckpt as ffc
        from dlrover_wuqiong_amd.flash_checkpoint.checkpointer import StorageType
        from dlrover_wuqiong_amd.models.gpt2 import Block
        from dlrover_wuqiong_amd.optimizers.fused import FusedAdamW
        from dlrover_wuqiong_amd.parallel.flat_fsdp import FlatFSDP

        m, cfg = _gpt2()
        model = FlatFSDP(m, wrap_cls=(Block,), reshard_after_forward=True)
        opt = FusedAdamW(model.shard_flat, lr=1e-2, weight_decay=0.05, max_grad_norm=0.5)
        data = _data(cfg, 3)

        def step(x):
            x = x.chunk(world)[rank]
            model(x[:, :-1], x[:, 1:]).backward()
            opt.step()
            opt.zero_grad()

        step(data[0])
        step(data[1])
        path = os.path.join(root, "step-2")
        assert ffc.save_checkpoint(2, model, opt, path, storage_type=StorageType.DISK)
        ok = True
        if rank == 0:
            ok = ffc.wait_for_persist(root, 2, timeout=60)
        dist.barrier()
        full = {k: v.clone() for k, v in model.full_state_dict().items()}
        shard = model.shard_flat.data.clone()
        state = [t.clone() for t in (opt.exp_avg, opt.exp_avg_sq)]
        step(data[2])
        after = model.full_state_dict()
        # in-place memory restore of the step-2 snapshot (same world size)
        got = ffc.load_checkpoint(model, opt, path)
        ok = ok and got == 2 and torch.equal(model.shard_flat.data, shard)
        ok = ok and torch.equal(opt.exp_avg, state[0]) and torch.equal(opt.exp_avg_sq, state[1])
        ok = ok and opt.step_count == 2
        if rank == 0:
            torch.save({"full": full, "after": after}, os.path.join(root, "ref.pt"))
        ffc.close_engines()
        q.put(bool(ok))
    except Exception as e:  # pragma: no cover
        import traceback

        traceback.print_exc()
        q.put(repr(e))
    finally:
        dist.destroy_process_group()


def test_flat_fsdp_checkpoint_reshards(tmp_path):
    assert _spawn(_ckpt_worker, 2, str(tmp_path)) == [True, True]
    from safetensors.torch import load_file

    from dlrover_wuqiong_amd.atorch.fsdp_flat_ckpt import ShardTensorUtil
    from dlrover_wuqiong_amd.models.gpt2 import Block
    from dlrover_wuqiong_amd.optimizers.fused import FusedAdamW
    from dlrover_wuqiong_amd.parallel.flat_fsdp import FlatFSDP

    path = str(tmp_path / "step-2")
    ref = torch.load(tmp_path / "ref.pt", weights_only=True)
    s0 = load_file(os.path.join(path, "flat_param.00000-00002"))
    assert all(t.dim() == 1 for t in s0.values())  # element ranges of the flattened parameters
    util = ShardTensorUtil(path)
    for n in ("wte.weight", "h.0.attn.c_attn.weight"):
        torch.testing.assert_close(util.load_tensor_by_name(n), ref["full"][n], rtol=0, atol=0)
    # world 1, flat: parameters + optimizer state resharded; the next step reproduces world 2's
    m, cfg = _gpt2()
    model = FlatFSDP(m, wrap_cls=(Block,))
    opt = FusedAdamW(model.shard_flat, lr=1e-2, weight_decay=0.05, max_grad_norm=0.5)
    util.load_into_model(model)
    util.load_optimizer(model, opt)
    assert opt.step_count == 2
    for k, v in model.full_state_dict().items():
        assert torch.equal(v, ref["full"][k]), k
    x = _data(cfg, 3)[2]
    model(x[:, :-1], x[:, 1:]).backward()
    opt.step()
    for k, v in model.full_state_dict().items():
        torch.testing.assert_close(v, ref["after"][k], rtol=2e-4, atol=2e-4, msg=k)
    # an unsharded model reads the same files (rows of the flattened ranges)
    plain, _cfg = _gpt2()
    with torch.no_grad():
        for p in plain.parameters():
            p.zero_()
    util.load_into_model(plain)
    for n, p in plain.named_parameters():
        assert torch.equal(p, ref["full"][n]), n


def _meta_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dlrover_wuqiong_amd.atorch.auto_accelerate import auto_accelerate
        from dlrover_wuqiong_amd.models.gpt2 import GPT2, Block, GPT2Config

        cfg = GPT2Config.named("gpt2-tiny")
        with torch.device("meta"):
            m = GPT2(cfg)
        ok, res, _s = auto_accelerate(m, torch.optim.AdamW, optim_args={"lr": 1e-3},
                                      load_strategy=[("flat_fsdp", {"wrap_cls": (Block,)})])
        model = res.model
        # nothing of the whole model was built: each rank holds its shard (+ the root unit gathered)
        layers = [u for u in model.units if not u.is_root]
        assert all(u.released for u in layers) and model.shard_flat.numel < sum(u.len for u in model.units) * world
        x = _data(cfg, 1)[0]
        loss = model(x[:, :-1], x[:, 1:])  # every rank the whole batch: the loss of the unsharded model
        loss.backward()
        res.optim.step()
        sd = model.full_state_dict()
        if rank == 0:
            q.put((float(loss), {k: v.float().numpy() for k, v in sd.items()}))
        else:
            q.put(None)
    except Exception as e:  # pragma: no cover
        import traceback

        traceback.print_exc()
        q.put(repr(e))
    finally:
        dist.destroy_process_group()


def test_flat_fsdp_meta_init_materialises_per_shard():
    """A meta-device model: every rank fills only its element ranges from the
    sharding-invariant streams -- the gathered model equals the unsharded
    model under meta_init.deterministic_init_, and it trains the same."""
    from dlrover_wuqiong_amd.atorch.meta_init import deterministic_init_
    from dlrover_wuqiong_amd.optimizers.fused import FusedAdamW
    from dlrover_wuqiong_amd.parallel.flat import FlatParams

    (loss, params), = _spawn(_meta_worker, 2)
    ref, cfg = _gpt2()
    deterministic_init_(ref, seed=0)
    flat = FlatParams(ref)
    opt = FusedAdamW(flat, lr=1e-3)
    x = _data(cfg, 1)[0]
    ref_loss = ref(x[:, :-1], x[:, 1:])
    ref_loss.backward()
    opt.step()
    assert float(ref_loss) == pytest.approx(loss, rel=1e-5)
    for n, p in ref.named_parameters():
        torch.testing.assert_close(torch.from_numpy(params[n]), p.detach(), rtol=2e-4, atol=2e-4, msg=n)


def _hsdp_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dlrover_wuqiong_amd.models.gpt2 import Block
        from dlrover_wuqiong_amd.optimizers.fused import FusedAdamW
        from dlrover_wuqiong_amd.parallel.flat_fsdp import FlatFSDP

        # shard groups {0,1} {2,3}, replicate groups {0,2} {1,3}
        shard = [dist.new_group([0, 1]), dist.new_group([2, 3])][rank // 2]
        rep = [dist.new_group([0, 2]), dist.new_group([1, 3])][rank % 2]
        m, cfg = _gpt2()
        model = FlatFSDP(m, wrap_cls=(Block,), process_group=shard, replicate_group=rep, reshard_after_forward=True)
        opt = FusedAdamW(model.shard_flat, lr=1e-2, weight_decay=0.05, max_grad_norm=0.5)
        assert opt.grad_scale == 0.25
        losses = []
        for x in _data(cfg):
            xm = x.chunk(world)[rank]
            loss = model(xm[:, :-1], xm[:, 1:])
            loss.backward()
            opt.step()
            opt.zero_grad()
            t = loss.detach().clone()
            dist.all_reduce(t)
            losses.append(float(t) / world)
        sd = model.full_state_dict()
        if rank == 0:
            q.put((losses, {k: v.float().numpy() for k, v in sd.items()}))
        else:
            q.put(None)
    except Exception as e:  # pragma: no cover
        import traceback

        traceback.print_exc()
        q.put(repr(e))
    finally:
        dist.destroy_process_group()


def test_flat_fsdp_hybrid_sharding_matches_one_process():
    """HSDP: 2 shard groups x 2 replicas (4 gloo ranks) == one process on
    the whole batch (global-norm clipping over the shard group)."""
    ref_losses, ref_params = _reference(micro=4)
    (losses, params), = _spawn(_hsdp_worker, 4)
    assert losses == pytest.approx(ref_losses, rel=1e-5, abs=1e-5)
    for n, p in ref_params.items():
        torch.testing.assert_close(torch.from_numpy(params[n]), p, rtol=2e-4, atol=2e-4, msg=n)


def _auto_hsdp_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dlrover_wuqiong_amd.atorch.auto_accelerate import auto_accelerate
        from dlrover_wuqiong_amd.models.gpt2 import Block

        m, cfg = _gpt2()
        ok, res, _s = auto_accelerate(m, torch.optim.AdamW, optim_args={"lr": 1e-3},
                                      load_strategy=[("parallel_mode", ([("zero", 2), ("data", 2)], None)),
                                                     ("flat_fsdp", {"wrap_cls": (Block,)})])
        assert ok and res.model.world == 2 and res.model.replicas == 2 and res.optim.grad_scale == 0.25
        x = _data(cfg, 1)[0].chunk(world)[rank]
        for _ in range(2):
            loss = res.model(x[:, :-1], x[:, 1:])
            loss.backward()
            res.optim.step()
            res.optim.zero_grad()
        # replicas hold identical shards
        shard = res.model.shard_flat.data.clone()
        peer = shard.clone()
        dist.broadcast(peer, src=rank % 2, group=res.model.rg)
        q.put(bool(torch.equal(shard, peer)))
    except Exception as e:  # pragma: no cover
        import traceback

        traceback.print_exc()
        q.put(repr(e))
    finally:
        dist.destroy_process_group()


def test_auto_accelerate_flat_fsdp_hybrid():
    assert _spawn(_auto_hsdp_worker, 4) == [True] * 4
