"""Meta-device FSDP initialisation and ``sync_module_states`` through
``auto_accelerate`` (atorch/meta_init.py; parity: ATorch
zero_optimization.py:328-369, utils/fsdp_init_util.py).

* 8 gloo ranks shard a Llama-3-70B-shaped model (hidden 8192, 64/8 heads,
  intermediate 28672, vocab 128256; 2 decoder layers so it fits the CI
  host) built under ``init_empty_weights()``: no rank ever holds more than
  its 1/8 (peak RSS checked) and every shard equals the same rows of the
  unsharded deterministic init.
* 4 ranks: a meta tiny Llama trains with the loss of a single process that
  runs the unsharded model with the same (deterministic) init.
* sync_module_states: per-rank random full models end up as rank 0's; rank
  0 real + other ranks meta -> rank 0's weights are scattered shard-wise.
"""

import os
import resource

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import free_port


def _env(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))


def _cfg70b_2l():
    from dlrover_wuqiong_amd.models.llama import LlamaConfig

    cfg = LlamaConfig.named("llama3-70b")
    cfg.num_hidden_layers = 2
    return cfg


def _run(fn, world, *args, timeout=600):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=fn, args=(r, world, port, q) + args) for r in range(world)]
    for p in ps:
        p.start()
    try:
        res = sorted((q.get(timeout=timeout) for _ in ps), key=lambda x: x[0])
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    return res


def _w70b(rank, world, port, q):
    _env(rank, world, port)
    torch.set_num_threads(1)
    try:
        from accelerate import init_empty_weights

        from dlrover_wuqiong_amd.atorch import distributed as adist
        from dlrover_wuqiong_amd.atorch.auto_accelerate import auto_accelerate
        from dlrover_wuqiong_amd.atorch.meta_init import _fill_counter
        from dlrover_wuqiong_amd.models.llama import Llama, LlamaDecoderLayer

        adist.init_distributed("gloo")
        rss0 = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss << 10
        cfg = _cfg70b_2l()
        with init_empty_weights():
            model = Llama(cfg).to(torch.bfloat16)
        full_bytes = sum(p.numel() for p in model.parameters()) * 2
        ok, res, _ = auto_accelerate(model, None, fused_optimizer=False,
                                     load_strategy=[("fsdp", {"wrap_cls": (LlamaDecoderLayer,)})])
        m = res.model
        local = sum(p.to_local().numel() for p in m.parameters()) * 2
        rss1 = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss << 10
        checks = []
        for name in ("layers.0.self_attn.qkv_proj.weight", "layers.1.self_attn.o_proj.weight", "norm.weight"):
            p = dict(m.named_parameters())[name]
            spec = m.init_spec(name) or (("ones",) if name.endswith("norm.weight") else ("normal", 0.0, 0.02))
            ref = torch.empty(p.shape, dtype=torch.float32)
            _fill_counter(ref, 0, name, 0, spec[0], *(spec[1:] if len(spec) > 1 else (0.0, 0.0)))
            loc = p.to_local()
            rows = loc.shape[0]
            from torch.distributed.tensor._utils import compute_local_shape_and_global_offset

            _s, off = compute_local_shape_and_global_offset(p.shape, p.device_mesh, p.placements)
            want = ref[off[0]: off[0] + rows].to(torch.bfloat16)
            checks.append(bool(torch.equal(loc, want)))
        q.put((rank, ("ok", full_bytes, local, rss1 - rss0, checks, ok)))
    except Exception as e:  # pragma: no cover
        import traceback

        traceback.print_exc()
        q.put((rank, repr(e)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.timeout(900)
def test_eight_rank_llama70b_config_meta_init_shards_only():
    res = _run(_w70b, 8)
    for _r, out in res:
        assert isinstance(out, tuple) and out[0] == "ok", res
        _tag, full_bytes, local, rss_growth, checks, ok = out
        assert ok and all(checks), out
        assert local <= full_bytes / 8 * 1.05 + (1 << 20), (local, full_bytes)
        # never the whole model on a rank: its 1/8 plus working buffers
        assert rss_growth < 0.35 * full_bytes, (rss_growth / 2**30, full_bytes / 2**30)


def _tiny():
    from dlrover_wuqiong_amd.models.llama import LlamaConfig

    cfg = LlamaConfig.named("llama-tiny")
    cfg.num_hidden_layers = 2
    cfg.vocab_size = 256
    return cfg


def _batch(step):
    g = torch.Generator().manual_seed(50 + step)
    ids = torch.randint(0, 256, (4, 17), generator=g)
    return ids[:, :-1], ids[:, 1:]


def _wtrain(rank, world, port, q):
    _env(rank, world, port)
    try:
        from dlrover_wuqiong_amd.atorch import distributed as adist
        from dlrover_wuqiong_amd.atorch.auto_accelerate import auto_accelerate
        from dlrover_wuqiong_amd.models.llama import Llama, LlamaDecoderLayer

        adist.init_distributed("gloo")
        with torch.device("meta"):
            model = Llama(_tiny())
        ok, res, _ = auto_accelerate(model, torch.optim.SGD, optim_args={"lr": 0.5}, fused_optimizer=False,
                                     load_strategy=[("fsdp", {"wrap_cls": (LlamaDecoderLayer,)})])
        losses = []
        for step in range(2):
            ids, tgt = _batch(step)
            res.optim.zero_grad()
            loss = res.model(ids[rank: rank + 1], tgt[rank: rank + 1])
            loss.backward()
            res.optim.step()
            t = loss.detach().clone()
            dist.all_reduce(t)
            losses.append(float(t) / world)
        q.put((rank, ("ok", losses)))
    except Exception as e:  # pragma: no cover
        import traceback

        traceback.print_exc()
        q.put((rank, repr(e)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_four_rank_meta_llama_trains_like_one_process():
    from dlrover_wuqiong_amd.atorch.meta_init import deterministic_init_
    from dlrover_wuqiong_amd.models.llama import Llama

    ref = Llama(_tiny())
    deterministic_init_(ref)  # the same values the shards get
    opt = torch.optim.SGD(ref.parameters(), lr=0.5)
    want = []
    for step in range(2):
        ids, tgt = _batch(step)
        opt.zero_grad()
        # per-rank mean losses averaged == mean over the 4 samples (equal lengths)
        loss = sum(ref(ids[r: r + 1], tgt[r: r + 1]) for r in range(4)) / 4
        loss.backward()
        opt.step()
        want.append(float(loss))
    res = _run(_wtrain, 4)
    for _r, out in res:
        assert isinstance(out, tuple) and out[0] == "ok", res
        assert all(abs(a - b) < 2e-4 for a, b in zip(out[1], want)), (out[1], want)


def _wsync(rank, world, port, q, mode):
    _env(rank, world, port)
    try:
        from dlrover_wuqiong_amd.atorch import distributed as adist
        from dlrover_wuqiong_amd.atorch.auto_accelerate import auto_accelerate
        from dlrover_wuqiong_amd.models.llama import Llama, LlamaDecoderLayer

        adist.init_distributed("gloo")
        if mode == "full" or rank == 0:
            torch.manual_seed(100 + rank)  # every rank a different random model
            model = Llama(_tiny())
        else:
            with torch.device("meta"):
                model = Llama(_tiny())
        # rank 0's weights, known to everyone for the check
        torch.manual_seed(100)
        r0 = {n: p.detach().clone() for n, p in Llama(_tiny()).named_parameters()}
        ok, res, _ = auto_accelerate(model, None, fused_optimizer=False,
                                     load_strategy=[("fsdp", {"wrap_cls": (LlamaDecoderLayer,),
                                                              "sync_module_states": True})])
        same = all(torch.equal(p.full_tensor(), r0[n]) for n, p in res.model.named_parameters())
        q.put((rank, ("ok", same)))
    except Exception as e:  # pragma: no cover
        import traceback

        traceback.print_exc()
        q.put((rank, repr(e)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["full", "rank0_real"])
def test_sync_module_states_rank0_wins(mode):
    res = _run(_wsync, 4, mode)
    for _r, out in res:
        assert isinstance(out, tuple) and out == ("ok", True), res


def _wreject(rank, world, port, q):
    _env(rank, world, port)
    try:
        from dlrover_wuqiong_amd.atorch import distributed as adist
        from dlrover_wuqiong_amd.atorch.auto_accelerate import auto_accelerate
        from dlrover_wuqiong_amd.models.llama import Llama, LlamaDecoderLayer

        adist.init_distributed("gloo")
        if rank == 0:
            model = Llama(_tiny())
        else:
            with torch.device("meta"):
                model = Llama(_tiny())
        try:
            auto_accelerate(model, None, fused_optimizer=False,
                            load_strategy=[("fsdp", {"wrap_cls": (LlamaDecoderLayer,)})])
            q.put((rank, "accepted"))
        except ValueError as e:
            q.put((rank, "rejected" if "sync_module_states" in str(e) else repr(e)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_mixed_meta_without_sync_is_rejected_loudly():
    res = _run(_wreject, 2)
    assert [o for _r, o in res] == ["rejected", "rejected"], res


class _RotaryLike(torch.nn.Module):
    """Parameter-free module with a config-derived, non-persistent buffer
    (the shape of HF rotary embeddings' ``inv_freq``)."""

    def __init__(self, config):
        super().__init__()
        self.config = config
        d = config.hidden_size // config.num_attention_heads
        self.register_buffer("inv_freq", 1.0 / (10000.0 ** (torch.arange(0, d, 2).float() / d)), persistent=False)


def _want_inv_freq(cfg):
    d = cfg.hidden_size // cfg.num_attention_heads
    return 1.0 / (10000.0 ** (torch.arange(0, d, 2).float() / d))


def _wbuf(rank, world, port, q, mode):
    _env(rank, world, port)
    try:
        from dlrover_wuqiong_amd.atorch import distributed as adist
        from dlrover_wuqiong_amd.atorch.auto_accelerate import auto_accelerate
        from dlrover_wuqiong_amd.models.llama import Llama, LlamaDecoderLayer

        adist.init_distributed("gloo")
        cfg = _tiny()
        real = mode == "rank0_real" and rank == 0
        with torch.device("cpu" if real else "meta"):
            model = Llama(cfg)
            model.rot = _RotaryLike(cfg)
        strat = {"wrap_cls": (LlamaDecoderLayer,)}
        if mode == "rank0_real":
            strat["sync_module_states"] = True
        ok, res, _ = auto_accelerate(model, None, fused_optimizer=False, load_strategy=[("fsdp", strat)])
        got = res.model.rot.inv_freq
        q.put((rank, ("ok", bool(torch.equal(got.cpu(), _want_inv_freq(cfg))))))
    except Exception as e:  # pragma: no cover
        import traceback

        traceback.print_exc()
        q.put((rank, repr(e)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["rank0_real", "all_meta"])
def test_meta_buffers_are_initialised(mode):
    """Buffers created on the meta device get real values on every rank:
    rank 0's are broadcast (sync_module_states), or the owning module is
    rebuilt from its config (all ranks meta)."""
    res = _run(_wbuf, 2, mode)
    assert [o for _r, o in res] == [("ok", True), ("ok", True)], res
