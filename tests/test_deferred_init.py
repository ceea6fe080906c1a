"""flash_checkpoint/deferred_init.py: on a restart the model's torch.nn.init
calls are recorded, not run; replay() reproduces the normal init exactly
(also through FlatParams' re-pointed storage)."""

import torch

from dlrover_wuqiong_amd.flash_checkpoint.deferred_init import deferred_init
from dlrover_wuqiong_amd.models.gpt2 import GPT2, GPT2Config
from dlrover_wuqiong_amd.parallel.flat import FlatParams


def _cfg():
    return GPT2Config(vocab_size=64, n_positions=16, n_layer=2, n_head=2, n_embd=32)


def test_noop_outside_restart(monkeypatch):
    monkeypatch.delenv("TORCHELASTIC_RESTART_COUNT", raising=False)
    torch.manual_seed(0)
    ref = GPT2(_cfg())
    torch.manual_seed(0)
    with deferred_init() as di:
        m = GPT2(_cfg())
    assert not di.active and di.replay() == 0
    for a, b in zip(ref.parameters(), m.parameters()):
        assert torch.equal(a, b)


def test_restart_defers_and_replays_through_flat_params(monkeypatch):
    monkeypatch.setenv("TORCHELASTIC_RESTART_COUNT", "1")
    torch.manual_seed(0)
    with deferred_init(active=False):
        ref = GPT2(_cfg())
    torch.manual_seed(0)
    with deferred_init() as di:
        m = GPT2(_cfg())
    assert di.active and len(di.calls) > 0
    flat = FlatParams(m)  # parameters now view the flat buffer
    assert m.h[0].attn.c_attn.weight.data_ptr() >= flat.data.data_ptr()
    torch.manual_seed(0)
    # the replay consumes the generator in the same order as the eager init
    n = di.replay()
    assert n > 0 and di.replay() == 0
    # (the parameters are views of the flat buffer: the replay wrote there)
    for (na, a), (nb, b) in zip(ref.named_parameters(), m.named_parameters()):
        assert torch.equal(a, b), na


def test_disabled_by_env(monkeypatch):
    monkeypatch.setenv("TORCHELASTIC_RESTART_COUNT", "2")
    monkeypatch.setenv("DWAMD_DEFER_INIT", "0")
    with deferred_init() as di:
        GPT2(_cfg())
    assert not di.active and not di.calls


def test_restart_build_holds_the_collector_until_the_restore():
    import gc

    from dlrover_wuqiong_amd.flash_checkpoint import deferred_init as dim

    assert gc.isenabled()
    with dim.deferred_init(active=True) as d:
        torch.nn.Linear(4, 4)
        assert not gc.isenabled()
    assert not gc.isenabled()  # still held: the model build continues until the restore
    d.discard()
    assert gc.isenabled()
    with dim.deferred_init(active=False):
        assert gc.isenabled()
    with dim.deferred_init(active=True) as d:
        pass
    d.replay()
    assert gc.isenabled()
    gc.unfreeze()
