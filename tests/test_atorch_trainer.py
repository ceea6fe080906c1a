"""AtorchTrainer: auto_accelerate-built training loop with HF callbacks,
flash-checkpoint saves, rotation and exact resume.
Parity: reference atorch/tests/.../test_atorch_trainer.py."""

import os

import pytest
import torch


class _DS(torch.utils.data.Dataset):
    def __init__(self, n=48, seq=16, vocab=64):
        g = torch.Generator().manual_seed(0)
        self.x = torch.randint(0, vocab, (n, seq + 1), generator=g)

    def __len__(self):
        return len(self.x)

    def __getitem__(self, i):
        return {"idx": self.x[i, :-1], "targets": self.x[i, 1:]}


def _model():
    from dlrover_wuqiong_amd.models.gpt2 import GPT2, GPT2Config

    torch.manual_seed(0)
    return GPT2(GPT2Config(vocab_size=64, n_positions=16, n_layer=2, n_head=2, n_embd=32))


def _args(out, **kw):
    from dlrover_wuqiong_amd.atorch.trainer import AtorchTrainingArgs

    base = dict(output_dir=str(out), per_device_train_batch_size=4, max_steps=6, save_steps=3, logging_steps=2,
                learning_rate=1e-3, shuffle=False, atorch_opt="none", atorch_module_replace=False,
                disable_tqdm=True, save_total_limit=1, seed=7, use_cpu=True, flash_checkpoint=True)
    base.update(kw)
    return AtorchTrainingArgs(**base)


@pytest.mark.parametrize("flash", [True, False])
def test_trainer_trains_saves_rotates_and_resumes_exactly(tmp_path, flash):
    from transformers import TrainerCallback

    from dlrover_wuqiong_amd.atorch.trainer import AtorchTrainer

    events = []

    class Rec(TrainerCallback):
        def on_save(self, args, state, control, **kw):
            events.append(("save", state.global_step))

        def on_log(self, args, state, control, logs=None, **kw):
            events.append(("log", state.global_step))

    a = AtorchTrainer(_model(), _args(tmp_path / "a", flash_checkpoint=flash), train_dataset=_DS(),
                      callbacks=[Rec()])
    m = a.train()
    assert m["global_step"] == 6
    assert ("save", 3) in events and ("save", 6) in events and ("log", 2) in events
    a.close()
    cks = sorted(os.listdir(tmp_path / "a"))
    assert "checkpoint-6" in cks and "checkpoint-3" not in cks  # save_total_limit=1
    assert any(h.get("loss") is not None for h in a.state.log_history)
    final_a = {k: v.clone() for k, v in a.model.state_dict().items()}

    # run b: stop at step 3 (checkpoint), then resume in a fresh trainer to step 6
    class Stop(TrainerCallback):
        def on_step_end(self, args, state, control, **kw):
            if state.global_step == 3:
                control.should_training_stop = True

    b = AtorchTrainer(_model(), _args(tmp_path / "b", save_total_limit=None, flash_checkpoint=flash),
                      train_dataset=_DS(), callbacks=[Stop()])
    assert b.train()["global_step"] == 3
    b.close()
    c = AtorchTrainer(_model(), _args(tmp_path / "b", flash_checkpoint=flash), train_dataset=_DS())
    c.train(resume_from_checkpoint=True)
    c.close()
    for k, v in c.model.state_dict().items():
        assert torch.allclose(v, final_a[k], atol=1e-6), k
    c.save_model(str(tmp_path / "final"))
    from safetensors.torch import load_file

    w = load_file(str(tmp_path / "final" / "model.safetensors"))
    assert torch.equal(w["wte.weight"], final_a["wte.weight"])


# ------------------------------------------------ distributed evaluation
class _ClsDS(torch.utils.data.Dataset):
    """37 samples: not a multiple of ranks x batch, so the sampler pads."""

    def __init__(self, n=37):
        g = torch.Generator().manual_seed(3)
        self.x = torch.randn(n, 8, generator=g)
        self.y = (self.x.sum(-1) > 0).long()

    def __len__(self):
        return len(self.x)

    def __getitem__(self, i):
        return {"x": self.x[i], "labels": self.y[i]}


class _Cls(torch.nn.Module):
    def __init__(self):
        super().__init__()
        torch.manual_seed(0)
        self.lin = torch.nn.Linear(8, 2)

    def forward(self, x, labels=None):
        logits = self.lin(x)
        out = {"logits": logits}
        if labels is not None:
            out["loss"] = torch.nn.functional.cross_entropy(logits, labels)
        return out


def _metrics(p):
    import numpy as np

    pred = p.predictions.argmax(-1)
    return {"acc": float((pred == p.label_ids).mean()), "n": int(len(p.label_ids)),
            "label_sum": int(np.sum(p.label_ids)), "logit_sum": float(np.sum(p.predictions))}


def _cls_args(out, **kw):
    base = dict(per_device_train_batch_size=4, per_device_eval_batch_size=3, max_steps=6, save_steps=2,
                logging_steps=100, atorch_opt="ddp", learning_rate=0.5, flash_checkpoint=False)
    base.update(kw)
    return _args(out, **base)


def _eval_worker(rank, world, port, q, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    import torch.distributed as dist

    try:
        from dlrover_wuqiong_amd.atorch.trainer import AtorchTrainer

        dist.init_process_group("gloo")
        t = AtorchTrainer(_Cls(), _cls_args(out), train_dataset=_ClsDS(), eval_dataset=_ClsDS(),
                          compute_metrics=_metrics)
        m = t.evaluate()
        pr = t.predict(_ClsDS())
        q.put((rank, ("ok", m, pr.predictions.tolist(), pr.num_samples)))
        t.close()
    except Exception as e:  # pragma: no cover
        import traceback

        traceback.print_exc()
        q.put((rank, repr(e)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_four_rank_evaluation_equals_single_process(tmp_path):
    import torch.multiprocessing as mp

    from conftest import free_port
    from dlrover_wuqiong_amd.atorch.trainer import AtorchTrainer

    single = AtorchTrainer(_Cls(), _cls_args(tmp_path / "s", atorch_opt="none"), train_dataset=_ClsDS(),
                           eval_dataset=_ClsDS(), compute_metrics=_metrics)
    want = single.evaluate()
    want_pred = single.predict(_ClsDS()).predictions
    assert want["eval_n"] == 37
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_eval_worker, args=(r, 4, port, q, str(tmp_path / "d"))) for r in range(4)]
    for p in ps:
        p.start()
    res = sorted((q.get(timeout=300) for _ in ps), key=lambda x: x[0])
    for p in ps:
        p.join(timeout=60)
    for _r, out in res:
        assert isinstance(out, tuple) and out[0] == "ok", res
        m = out[1]
        # global metrics over exactly the 37 samples (padding stripped), equal to one process
        assert m["eval_n"] == 37 and m["eval_label_sum"] == want["eval_label_sum"]
        assert abs(m["eval_acc"] - want["eval_acc"]) < 1e-9
        assert abs(m["eval_loss"] - want["eval_loss"]) < 1e-5
        assert abs(m["eval_logit_sum"] - want["eval_logit_sum"]) < 1e-3
        assert out[3] == 37 and torch.allclose(torch.tensor(out[2]), want_pred, atol=1e-5)


class _LMDS(torch.utils.data.Dataset):
    """Token sequences for a vocab-sized-logits model."""

    def __init__(self, n, seq=12, vocab=512):
        g = torch.Generator().manual_seed(5)
        self.x = torch.randint(0, vocab, (n, seq), generator=g)

    def __len__(self):
        return len(self.x)

    def __getitem__(self, i):
        return {"x": self.x[i], "labels": self.x[i]}


class _LM(torch.nn.Module):
    def __init__(self, vocab=512):
        super().__init__()
        torch.manual_seed(0)
        self.emb = torch.nn.Embedding(vocab, 16)
        self.head = torch.nn.Linear(16, vocab)

    def forward(self, x, labels=None):
        logits = self.head(self.emb(x))
        out = {"logits": logits}
        if labels is not None:
            out["loss"] = torch.nn.functional.cross_entropy(logits.flatten(0, 1), labels.flatten())
        return out


def _argmax(logits, labels):
    return logits.argmax(-1)


def _tok_metrics(p):
    import numpy as np

    return {"tok_acc": float((p.predictions == p.label_ids).mean()), "rows": int(len(p.label_ids)),
            "pred_sum": int(np.sum(p.predictions))}


def _lm_eval(rank, world, port, q, out, sizes, eas):
    if world > 1:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    import torch.distributed as dist

    try:
        from dlrover_wuqiong_amd.atorch.trainer import AtorchTrainer

        if world > 1:
            dist.init_process_group("gloo")
        res = []
        for n in sizes:
            t = AtorchTrainer(_LM(), _cls_args(out, per_device_eval_batch_size=2, eval_accumulation_steps=eas,
                                               atorch_opt="ddp" if world > 1 else "none"),
                              train_dataset=_LMDS(8), eval_dataset=_LMDS(n), compute_metrics=_tok_metrics,
                              preprocess_logits_for_metrics=_argmax)
            m = t.evaluate()
            res.append((m, t.eval_peak_accum_bytes))
            t.close()
        q.put((rank, ("ok", res)))
    except Exception as e:  # pragma: no cover
        import traceback

        traceback.print_exc()
        q.put((rank, repr(e)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _spawn_eval(world, target, args):
    import torch.multiprocessing as mp

    from conftest import free_port

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted((q.get(timeout=300) for _ in ps), key=lambda x: x[0])
    for p in ps:
        p.join(timeout=60)
    return res


def test_bounded_eval_with_logit_preprocessing_matches_single_process(tmp_path):
    """Vocab-sized logits reduced to argmax ids per batch, moved to the host
    every 2 batches on 4 gloo ranks: the metrics equal one process's, and
    the device-side accumulation is bounded whatever the dataset length."""
    import queue

    q = queue.Queue()
    _lm_eval(0, 1, 0, q, str(tmp_path / "s"), (37, 150), None)
    _r, single = q.get()
    assert single[0] == "ok", single
    res = _spawn_eval(4, _lm_eval, (str(tmp_path / "d"), (37, 150), 2))
    for _r, out in res:
        assert isinstance(out, tuple) and out[0] == "ok", res
        for (m, peak), (want, _p) in zip(out[1], single[1]):
            assert m["eval_rows"] == want["eval_rows"] and m["eval_pred_sum"] == want["eval_pred_sum"]
            assert abs(m["eval_tok_acc"] - want["eval_tok_acc"]) < 1e-12
            assert abs(m["eval_loss"] - want["eval_loss"]) < 1e-5
        (_m37, peak37), (_m150, peak150) = out[1]
        # at most 2 batches of int64 ids + labels (2 x 12 tokens x 8 B each) on the device
        assert peak37 == peak150 <= 2 * 2 * (2 * 12 * 8), (peak37, peak150)


def _few_batches_eval(rank, world, port, q, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    import torch.distributed as dist

    try:
        from dlrover_wuqiong_amd.atorch.trainer import AtorchTrainer

        dist.init_process_group("gloo")
        # 9 samples, eval batch 3: 3 batches on 4 ranks -- rank 3 has only a padding batch
        t = AtorchTrainer(_Cls(), _cls_args(out), train_dataset=_ClsDS(), eval_dataset=_ClsDS(9),
                          compute_metrics=_metrics)
        m = t.evaluate()
        pr = t.predict(_ClsDS(9))
        q.put((rank, ("ok", m, pr.num_samples, tuple(pr.predictions.shape))))
        t.close()
    except Exception as e:  # pragma: no cover
        import traceback

        traceback.print_exc()
        q.put((rank, repr(e)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_eval_with_more_ranks_than_batches(tmp_path):
    """A rank whose whole share is padding still enters every gather (no
    deadlock) and the result covers exactly the dataset."""
    res = _spawn_eval(4, _few_batches_eval, (str(tmp_path / "d"),))
    for _r, out in res:
        assert isinstance(out, tuple) and out[0] == "ok", res
        assert out[1]["eval_n"] == 9 and out[2] == 9 and out[3] == (9, 2)


def test_load_best_model_at_end(tmp_path):
    from dlrover_wuqiong_amd.atorch.trainer import AtorchTrainer

    snaps = {}
    holder = {}

    def metrics(p):
        step = holder["t"].state.global_step
        snaps[step] = {k: v.clone() for k, v in holder["t"].model.state_dict().items()}
        return {"score": -abs(step - 4)}  # best at step 4 of 2, 4, 6

    t = AtorchTrainer(_Cls(), _cls_args(tmp_path / "b", atorch_opt="none", eval_strategy="steps", eval_steps=2,
                                        load_best_model_at_end=True, metric_for_best_model="score",
                                        greater_is_better=True, save_total_limit=1),
                      train_dataset=_ClsDS(), eval_dataset=_ClsDS(), compute_metrics=metrics)
    holder["t"] = t
    t.train()
    assert t.state.best_model_checkpoint.endswith("checkpoint-4") and t.state.best_metric == 0
    assert os.path.isdir(t.state.best_model_checkpoint)  # kept despite save_total_limit=1
    for k, v in t.model.state_dict().items():
        assert torch.equal(v, snaps[4][k]), k
    assert not torch.equal(snaps[4]["lin.weight"], snaps[6]["lin.weight"])
    t.close()
