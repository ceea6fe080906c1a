"""Tensor parallelism for encoder families (ATorch's Megatron TP layers for
Bert / CLIP, modules/distributed_modules/transformer.py) through
``auto_accelerate``'s ``mixed_parallel`` (tensor 2 x data 2, no pipeline) on
4 gloo ranks: HF BertForMaskedLM and CLIPTextModel train with the loss of one
process on the global batch.  Attention blocks fx cannot trace come from the
layer-grouped name table (Bert: query / key / value -> attention.output.dense,
intermediate.dense -> output.dense)."""

import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import free_port

V = 128


def _model(family):
    import transformers as tf

    torch.manual_seed(0)
    if family == "bert":
        m = tf.BertForMaskedLM(tf.BertConfig(vocab_size=V, hidden_size=64, num_hidden_layers=2,
                                             num_attention_heads=4, intermediate_size=128,
                                             hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0))
    else:
        m = tf.CLIPTextModel(tf.CLIPTextConfig(vocab_size=V, hidden_size=64, num_hidden_layers=2,
                                               num_attention_heads=4, intermediate_size=128))
    m.config._attn_implementation = "sdpa"
    return m.float()


def _loss(family, model, ids):
    import torch.nn.functional as F

    if family == "bert":
        return model(input_ids=ids, labels=ids).loss
    h = model(input_ids=ids).last_hidden_state
    return F.mse_loss(h, torch.zeros_like(h))


def _batch(step):
    g = torch.Generator().manual_seed(300 + step)
    return torch.randint(0, V, (4, 12), generator=g)


def _worker(rank, world, port, q, family):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    torch.set_num_threads(1)
    from dlrover_wuqiong_amd.atorch import distributed as adist

    try:
        from dlrover_wuqiong_amd.atorch.auto_accelerate import auto_accelerate

        adist.init_distributed("gloo")
        ok, res, _ = auto_accelerate(_model(family), torch.optim.SGD, optim_args={"lr": 0.5},
                                     fused_optimizer=False,
                                     load_strategy=[("mixed_parallel", {"tensor": 2, "pipeline": 1, "data": 2})])
        n_tp = sum(bool(getattr(p, "tensor_model_parallel", False)) for p in res.model.parameters())
        dr = adist.parallel_rank("data")
        losses = []
        for step in range(2):
            ids = _batch(step)[2 * dr: 2 * dr + 2]
            res.optim.zero_grad()
            loss = _loss(family, res.model, ids)
            loss.backward()
            res.optim.step()
            t = loss.detach().reshape(1).double()
            dist.all_reduce(t)
            losses.append(float(t) / world)
        q.put((rank, ("ok", losses, n_tp)))
    except Exception as e:  # pragma: no cover
        import traceback

        traceback.print_exc()
        q.put((rank, repr(e)))
    finally:
        adist.reset_distributed()


@pytest.mark.timeout(400)
@pytest.mark.parametrize("family", ["bert", "clip"])
def test_encoder_tp2_dp2_matches_one_process(family):
    model = _model(family)
    opt = torch.optim.SGD(model.parameters(), lr=0.5)
    ref = []
    for step in range(2):
        ids = _batch(step)
        opt.zero_grad()
        # each data replica's loss is the mean over its 2 samples; the
        # replicas' average equals the 4-sample mean here (equal lengths)
        loss = (_loss(family, model, ids[:2]) + _loss(family, model, ids[2:])) / 2
        loss.backward()
        opt.step()
        ref.append(float(loss))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_worker, args=(r, 4, port, q, family)) for r in range(4)]
    for p in ps:
        p.start()
    res = sorted((q.get(timeout=300) for _ in ps), key=lambda x: x[0])
    for p in ps:
        p.join(timeout=60)
    assert all(isinstance(r[1], tuple) and r[1][0] == "ok" for r in res), res
    # attention (q, k, v, out) and MLP (2) of both layers
    assert all(r[1][2] == 12 for r in res), res
    got = res[0][1][1]
    assert all(abs(a - b) < 2e-4 for a, b in zip(got, ref)), (family, got, ref)
