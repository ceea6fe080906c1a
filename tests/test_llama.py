"""Llama family on CPU: forward/backward, GQA, MoE variant; tensor parallel
(2 ranks) and Ulysses sequence parallel (2 ranks) match the single-device
model."""

import os

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import free_port


def test_llama_tiny_trains_and_moe():
    from dlrover_wuqiong_amd.models.llama import Llama, LlamaConfig

    for name in ("llama-tiny", "llama-moe-tiny"):
        torch.manual_seed(0)
        m = Llama(LlamaConfig.named(name))
        ids = torch.randint(0, 1024, (2, 33))
        opt = torch.optim.AdamW(m.parameters(), lr=3e-3)
        losses = []
        for _ in range(8):
            loss = m(ids[:, :-1], ids[:, 1:])
            opt.zero_grad()
            loss.backward()
            opt.step()
            losses.append(float(loss))
        assert losses[-1] < losses[0] - 0.5, (name, losses)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dlrover_wuqiong_amd.models.llama import Llama, LlamaConfig, shard_llama_state_dict

        cfg = LlamaConfig.named("llama-tiny")
        torch.manual_seed(0)
        ref = Llama(cfg)
        ids = torch.randint(0, 1024, (2, 17))
        ref_loss = ref(ids[:, :-1], ids[:, 1:])
        ref_loss.backward()
        ok = True
        # tensor parallel
        torch.manual_seed(1)
        tpm = Llama(cfg, tp_group=dist.group.WORLD)
        tpm.load_state_dict(shard_llama_state_dict(ref.state_dict(), cfg, rank, world))
        loss = tpm(ids[:, :-1], ids[:, 1:])
        ok &= torch.allclose(loss, ref_loss, atol=1e-5)
        loss.backward()
        g = tpm.layers[0].self_attn.o_proj.weight.grad
        per = g.shape[1]
        ok &= torch.allclose(g, ref.layers[0].self_attn.o_proj.weight.grad[:, rank * per:(rank + 1) * per], atol=1e-5)
        # Ulysses sequence parallel: each rank holds half of the sequence
        spm = Llama(cfg, sp_group=dist.group.WORLD)
        spm.load_state_dict(ref.state_dict())
        S = 16
        x, y = ids[:, :-1], ids[:, 1:]
        part = slice(rank * S // world, (rank + 1) * S // world)
        logits = spm(x[:, part])
        full = ref(x)
        ok &= torch.allclose(logits, full[:, part], atol=1e-4)
        q.put((rank, bool(ok)))
    except Exception as e:  # pragma: no cover
        import traceback

        traceback.print_exc()
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def test_llama_tp_and_sp_two_ranks():
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
