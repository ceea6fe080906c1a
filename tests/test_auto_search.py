"""Strategy search: analyser, dry runner, exhaustive and BO-guided search.
Parity: reference atorch/tests/.../test_dry_runner.py, test_analyser.py,
test_bo_sg.py (strategy generation with Bayesian optimisation)."""

import torch


def _model_fn():
    from dlrover_wuqiong_amd.models.gpt2 import GPT2, GPT2Config

    torch.manual_seed(0)
    return GPT2(GPT2Config(vocab_size=64, n_positions=16, n_layer=2, n_head=2, n_embd=32))


def _batch():
    g = torch.Generator().manual_seed(0)
    x = torch.randint(0, 64, (4, 17), generator=g)
    return (x[:, :-1], x[:, 1:])


def _loss(batch, out):
    return out


def test_analyser_and_dry_runner():
    from dlrover_wuqiong_amd.atorch.auto_search import DryRunner, analyse_model

    a = analyse_model(_model_fn(), world=4)
    assert a["block_classes"] == ["Block"] and a["params"] > 0
    assert a["state_bytes"]["fsdp"] < a["state_bytes"]["zero2"] < a["state_bytes"]["zero1"] < a["state_bytes"]["ddp"]
    r = DryRunner.profile(_model_fn, ["module_replace"], torch.optim.AdamW, {"lr": 1e-3}, _batch(), _loss,
                          model_input_format="unpack_sequence")
    assert r.ok and r.throughput > 0 and r.step_time > 0
    bad = DryRunner.profile(_model_fn, ["no_such_opt"], torch.optim.AdamW, {"lr": 1e-3}, _batch(), _loss,
                            model_input_format="unpack_sequence")
    assert not bad.ok and "no_such_opt" in bad.error


def test_search_strategy_exhaustive_and_bo():
    from dlrover_wuqiong_amd.atorch.auto_search import search_strategy

    best, rep = search_strategy(_model_fn, torch.optim.AdamW, {"lr": 1e-3}, _batch(), _loss,
                                model_input_format="unpack_sequence")
    assert len(rep.results) == 4 and all(r.ok for r in rep.results)
    assert best in [r.strategy for r in rep.results]
    best2, rep2 = search_strategy(_model_fn, torch.optim.AdamW, {"lr": 1e-3}, _batch(), _loss, max_trials=3,
                                  model_input_format="unpack_sequence")
    assert len(rep2.results) == 3
    # pruning: a tiny HBM budget rules everything out
    try:
        search_strategy(_model_fn, torch.optim.AdamW, {"lr": 1e-3}, _batch(), _loss, hbm_bytes=1,
                        model_input_format="unpack_sequence")
        raise AssertionError("expected failure")
    except RuntimeError:
        pass


def test_auto_accelerate_search_mode():
    from dlrover_wuqiong_amd.atorch.auto_accelerate import auto_accelerate

    ok, res, strat = auto_accelerate(_model_fn(), torch.optim.AdamW, optim_args={"lr": 1e-3}, loss_func=_loss,
                                     load_strategy="search", model_fn=_model_fn, sample_batch=_batch(),
                                     max_trials=2, model_input_format="unpack_sequence")
    assert ok and "module_replace" in strat.names()
    x, y = _batch()
    res.model(x, y).backward()
    res.optim.step()
