"""RL hybrid engine: KV-cached generation from the training weights (CPU
reference math here; the HIP decode kernel + graph path in
test_hybrid_engine_gpu.py) and FSDP2 gather/reshard around a rollout."""

import os

import torch
import torch.multiprocessing as mp

from conftest import free_port
from dlrover_wuqiong_amd.atorch.rl.hybrid_engine import HybridEngine
from dlrover_wuqiong_amd.atorch.rl.trainer import sample
from dlrover_wuqiong_amd.models.llama import Llama, LlamaConfig
from dlrover_wuqiong_amd.ops.attention import decode_attention_reference


def test_greedy_generation_matches_full_forward_sampling():
    torch.manual_seed(0)
    m = Llama(LlamaConfig.named("llama-tiny")).eval()
    p = torch.randint(0, 1024, (3, 7))
    ref = sample(m, p, 8, temperature=0)
    eng = HybridEngine(m, 4, 32)
    assert eng.generate(p, 8, temperature=0).tolist() == ref.tolist()
    # a second rollout reuses the cache
    p2 = torch.randint(0, 1024, (3, 5))
    assert eng.generate(p2, 4, temperature=0).tolist() == sample(m, p2, 4, temperature=0).tolist()
    assert m.training is False


def test_decode_reference_matches_dense_attention():
    torch.manual_seed(1)
    B, H, HKV, D, S = 2, 4, 2, 16, 9
    q = torch.randn(B, H, D)
    kc, vc = torch.randn(B, S, HKV, D), torch.randn(B, S, HKV, D)
    lens = torch.tensor([9, 5], dtype=torch.int32)
    out = decode_attention_reference(q, kc, vc, lens)
    for b in range(B):
        n = int(lens[b])
        k = kc[b, :n].repeat_interleave(2, 1).transpose(0, 1)
        v = vc[b, :n].repeat_interleave(2, 1).transpose(0, 1)
        ref = torch.nn.functional.scaled_dot_product_attention(q[b][:, None], k, v)[:, 0]
        torch.testing.assert_close(out[b], ref, atol=1e-5, rtol=1e-5)


def test_ppo_trainer_uses_hybrid_engine():
    from dlrover_wuqiong_amd.atorch.rl.config import PPOConfig
    from dlrover_wuqiong_amd.atorch.rl.engine import ModelEngine, ValueModel
    from dlrover_wuqiong_amd.atorch.rl.trainer import PPOTrainer

    torch.manual_seed(0)
    cfg = LlamaConfig.named("llama-tiny")
    actor, ref = Llama(cfg), Llama(cfg)
    critic = ValueModel(Llama(cfg), cfg.vocab_size)

    class Reward(torch.nn.Module):
        def forward(self, ids):
            return (ids[:, -4:] % 7 == 0).float().mean(-1)

    eng = ModelEngine(actor, critic, ref, Reward(), actor_lr=1e-4, critic_lr=1e-4)
    prompts = torch.randint(0, cfg.vocab_size, (8, 6))
    pc = PPOConfig(max_new_tokens=4, rollout_batch_size=4, mini_batch_size=4, ppo_epochs=1)
    tr = PPOTrainer(eng, prompts, pc)
    stats = tr.train(1)
    assert tr._hy is not None and tr._hy.cache.k.shape[2] == 10 and stats


def _fsdp_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    from torch.distributed.fsdp import fully_shard

    try:
        dist.init_process_group("gloo")
        torch.manual_seed(0)
        full = Llama(LlamaConfig.named("llama-tiny")).eval()
        torch.manual_seed(0)
        m = Llama(LlamaConfig.named("llama-tiny")).eval()
        for layer in m.layers:
            fully_shard(layer)
        fully_shard(m)
        p = torch.randint(0, 1024, (2, 6), generator=torch.Generator().manual_seed(5))
        out = HybridEngine(m, 2, 16).generate(p, 5, temperature=0)
        ref = sample(full, p, 5, temperature=0)
        # parameters are sharded again after the rollout
        from torch.distributed.tensor import DTensor

        resharded = all(isinstance(x, DTensor) for x in m.layers[0].parameters())
        q.put((rank, out.tolist() == ref.tolist() and resharded))
    except Exception as e:  # pragma: no cover
        import traceback

        traceback.print_exc()
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def test_fsdp_actor_gathered_for_generation():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_fsdp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=180) for _ in ps)
    for p in ps:
        p.join(30)
    assert all(r[1] is True for r in res), res


def _tp_worker(rank, world, port, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dlrover_wuqiong_amd.models.llama import shard_llama_state_dict

        torch.manual_seed(0)
        cfg = LlamaConfig.named("llama-tiny")
        full = Llama(cfg).eval()
        p = torch.randint(0, 1024, (2, 6), generator=torch.Generator().manual_seed(3))
        ref = sample(full, p, 6, temperature=0)
        tp = Llama(cfg, tp_group=dist.group.WORLD)
        tp.load_state_dict(shard_llama_state_dict(full.state_dict(), cfg, rank, world))
        eng = HybridEngine(tp, 2, 16)
        out = eng.generate(p, 6, temperature=0)
        # sampled (temperature 1): both TP ranks must emit the same tokens
        out2 = eng.generate(p, 5, temperature=1.0, generator=torch.Generator().manual_seed(rank))
        both = [torch.zeros_like(out2) for _ in range(world)]
        dist.all_gather(both, out2)
        q.put((rank, out.tolist() == ref.tolist() and torch.equal(both[0], both[1]) and eng.cache.k.shape[3] == 1))
    except Exception as e:  # pragma: no cover
        import traceback

        traceback.print_exc()
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def test_tensor_parallel_actor_generation():
    """A TP=2 actor generates exactly what the unsharded model generates: each
    rank caches its KV heads, logits are gathered over the vocab shards and
    the sample is shared within the TP group."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_tp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=180) for _ in ps)
    for p in ps:
        p.join(30)
    assert all(r[1] is True for r in res), res
