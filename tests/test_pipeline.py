"""Pipeline parallelism on CPU/gloo: GPipe, 1F1B and interleaved-1F1B
schedules must reproduce the single-process loss and every gradient
(including the tied embedding / LM head) of GPT-2 and Llama.

Parity: reference ``atorch/tests/.../test_pipe_compiler.py`` /
``test_pipeline_parallel_optimization.py`` check that the PiPPy-compiled
model trains; here each stage's gradients are compared to the unsplit model."""

import copy
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import free_port


def test_partition_layers_balances_head_cost():
    from dlrover_wuqiong_amd.parallel.pipeline import partition_layers

    b = partition_layers(48, 4, embed_cost=0.1, head_cost=2.8)
    assert b[0][0] == 0 and b[-1][1] == 48
    assert all(b[i][1] == b[i + 1][0] for i in range(3))
    sizes = [e - s for s, e in b]
    assert sizes[-1] < sizes[1]  # the LM-head stage gets fewer layers
    assert partition_layers(4, 4) == [(0, 1), (1, 2), (2, 3), (3, 4)]
    with pytest.raises(ValueError):
        partition_layers(3, 4)


def _model(kind):
    if kind == "gpt2":
        from dlrover_wuqiong_amd.models.gpt2 import GPT2, GPT2Config

        return GPT2(GPT2Config(vocab_size=64, n_positions=16, n_layer=8, n_head=2, n_embd=32))
    from dlrover_wuqiong_amd.models.llama import Llama, LlamaConfig

    cfg = LlamaConfig.named("llama-tiny")
    cfg.num_hidden_layers = 8
    cfg.tie_word_embeddings = True
    return Llama(cfg)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    try:
        from dlrover_wuqiong_amd.parallel import state
        from dlrover_wuqiong_amd.parallel.pipeline import PipelineModule

        dist.init_process_group("gloo", rank=rank, world_size=world)
        state.initialize_model_parallel(pipeline_model_parallel_size=world)
        ok = []
        for kind in ("gpt2", "llama"):
            for sched, v in (("gpipe", 1), ("1f1b", 1), ("interleaved", 2)):
                torch.manual_seed(0)
                model = _model(kind)
                vocab = 64 if kind == "gpt2" else model.cfg.vocab_size
                ref = copy.deepcopy(model)
                g = torch.Generator().manual_seed(1)
                ids = torch.randint(0, vocab, (8, 12), generator=g)
                tgt = torch.randint(0, vocab, (8, 12), generator=g)
                ref_loss = ref(ids, tgt)
                ref_loss.backward()
                pipe = PipelineModule(model, world, rank, num_microbatches=4, schedule=sched, virtual_stages=v,
                                      group=state.get_pipeline_model_parallel_group(),
                                      embedding_group=state.get_embedding_group())
                loss = pipe.train_step(ids if rank == 0 else None, tgt)
                good = abs(float(loss) - float(ref_loss)) < 1e-5
                ref_named = dict(ref.named_parameters())
                layers_attr = "h" if kind == "gpt2" else "layers"
                for chunk in pipe.chunks:
                    for i, layer in enumerate(getattr(chunk, layers_attr)):
                        rl = getattr(ref, layers_attr)[chunk.start + i]
                        for (n, p), (_, rp) in zip(layer.named_parameters(), rl.named_parameters()):
                            good &= torch.allclose(p.grad, rp.grad, atol=1e-5, rtol=1e-4)
                    emb = "wte.weight" if kind == "gpt2" else "embed_tokens.weight"
                    for p in chunk.tied_parameters():
                        good &= torch.allclose(p.grad, ref_named[emb].grad, atol=1e-5, rtol=1e-4)
                ok.append((kind, sched, bool(good)))
        q.put((rank, ok))
    except Exception as e:  # pragma: no cover
        import traceback

        traceback.print_exc()
        q.put((rank, repr(e)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_pipeline_schedules_match_unsplit_model(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(timeout=30)
    for rank, ok in res:
        assert isinstance(ok, list), ok
        assert all(g for *_, g in ok), (rank, ok)


def _auto_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        from dlrover_wuqiong_amd.atorch import distributed as adist
        from dlrover_wuqiong_amd.atorch.auto_accelerate import auto_accelerate

        adist.init_distributed("gloo")
        torch.manual_seed(0)
        model = _model("gpt2")
        ref = copy.deepcopy(model)
        g = torch.Generator().manual_seed(1)
        ids = torch.randint(0, 64, (8, 12), generator=g)
        tgt = torch.randint(0, 64, (8, 12), generator=g)
        # data rank d trains on half d of the batch; reference = mean over both halves
        ref_loss = (ref(ids[:4], tgt[:4]) + ref(ids[4:], tgt[4:])) / 2
        ref_loss.backward()
        ok, res, strat = auto_accelerate(
            model, torch.optim.SGD, optim_args={"lr": 0.1},
            load_strategy=[("parallel_mode", ([("pipeline", 2), ("data", 2)], None)),
                           ("pipeline_parallel", {"chunks": 2, "schedule": "1f1b"})])
        pipe = res.model
        d = adist.parallel_rank("data")
        loss = pipe.train_step(ids[4 * d:4 * d + 4], tgt[4 * d:4 * d + 4])
        good = "pipeline_parallel" in strat.names() and "ddp" in strat.names()
        # per-data-rank losses differ; grads are averaged over the data group
        for i, layer in enumerate(pipe.chunks[0].h):
            rl = ref.h[pipe.chunks[0].start + i]
            for p, rp in zip(layer.parameters(), rl.parameters()):
                good &= torch.allclose(p.grad, rp.grad, atol=1e-5, rtol=1e-4)
        before = [p.detach().clone() for p in pipe.parameters()]
        res.optim.step()
        good &= any(not torch.equal(b, p) for b, p in zip(before, pipe.parameters()))
        good &= bool(torch.isfinite(loss))
        q.put((rank, bool(good)))
    except Exception as e:  # pragma: no cover
        import traceback

        traceback.print_exc()
        q.put((rank, repr(e)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_auto_accelerate_pipeline_with_data_parallel():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_auto_worker, args=(r, 4, port, q)) for r in range(4)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(timeout=30)
    assert res == [(r, True) for r in range(4)], res
