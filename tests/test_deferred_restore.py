"""CPU: which checkpoint leaves a restore may let land behind the first step
(flash_checkpoint/deferred_restore.py), and the optimizer step pre-hook that
orders every optimizer step after pending deferred copies."""

import types

import torch

from dlrover_wuqiong_amd.flash_checkpoint import deferred_restore as dr
from dlrover_wuqiong_amd.flash_checkpoint.engine import CheckpointEngine
from dlrover_wuqiong_amd.flash_checkpoint.layout import TensorMeta


def _tm(n=4):
    return TensorMeta(shape=(n,), dtype=torch.float32, element_size=4, numel=n, device="cuda")


def test_late_leaf_flags_follow_optimizer_keys(monkeypatch):
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    tree = {"model_states": {"model": {"w": _tm(), "optimizer_like_param_name": {"x": _tm()}},
                             "optimizer": {"state": {0: {"exp_avg": _tm(), "step": 3}}, "param_groups": [{"lr": 1}]},
                             "step": 7, "rng": [_tm(), _tm()]}}
    eng = types.SimpleNamespace(defer_optimizer_restore=True)
    flags = CheckpointEngine._late_leaf_flags(eng, tree)
    # leaves in iter_leaves order: w, x (model), exp_avg (optimizer), 2 x rng
    assert flags == [False, False, True, False, False]
    eng.defer_optimizer_restore = False
    assert CheckpointEngine._late_leaf_flags(eng, tree) is None
    eng.defer_optimizer_restore = True
    monkeypatch.setenv("DWAMD_DEFER_OPTIM_RESTORE", "0")
    assert CheckpointEngine._late_leaf_flags(eng, tree) is None
    monkeypatch.delenv("DWAMD_DEFER_OPTIM_RESTORE")
    assert CheckpointEngine._late_leaf_flags(eng, {"model": {"w": _tm()}}) is None
    assert dr.is_deferred_key("opt") and dr.is_deferred_key("Optimizer") and not dr.is_deferred_key("model")


class _Fake:
    device = torch.device("cpu")

    def __init__(self):
        self.waits = 0
        self.done = False

    def wait(self, stream=None):
        self.waits += 1

    def ready_event(self):
        return None

    @property
    def complete(self):
        return self.done


def test_every_optimizer_step_waits_for_pending_restores():
    from dlrover_wuqiong_amd.optimizers.fused import FusedAdamW
    from dlrover_wuqiong_amd.parallel.flat import FlatParams

    f = _Fake()
    dr.add(f)
    try:
        m = torch.nn.Linear(4, 4)
        torch.optim.SGD(m.parameters(), lr=0.1).step()
        assert f.waits == 1
        flat = FlatParams(torch.nn.Linear(4, 4), dtype=torch.float32)
        for p in flat.params:
            p.grad = torch.zeros_like(p)
        FusedAdamW(flat, lr=1e-3).step()
        assert f.waits == 2
        f.done = True  # landed: pruned, later steps do not wait
        torch.optim.SGD(m.parameters(), lr=0.1).step()
        assert f.waits == 2 and not dr.pending()
    finally:
        f.done = True
        dr.pending()


def test_deferred_state_prefix_from_ring_progress():
    """The deferred state write-back (optimizers/fused.py) defers exactly the
    flat elements whose master / exp_avg / exp_avg_sq the ring snapshot reads
    but has not copied yet (address arithmetic only; CPU tensors)."""
    from dlrover_wuqiong_amd.optimizers.fused import FusedAdamW
    from dlrover_wuqiong_amd.parallel.flat import FlatParams

    m = torch.nn.Sequential(torch.nn.Linear(64, 64), torch.nn.Linear(64, 64)).to(torch.bfloat16)
    flat = FlatParams(m)
    opt = FusedAdamW(flat, lr=1e-3)
    n = flat.numel
    bufs = [opt.exp_avg, opt.exp_avg_sq, opt.master]

    class Ring:
        def __init__(self, src, staged):
            self.src, self.stg = src, staged

        def ring_sources(self):
            return self.src

        def ring_staged(self):
            return self.stg

    whole = [(b.data_ptr(), b.data_ptr() + 4 * n) for b in bufs]
    assert opt._dsw_first_unstaged(Ring(whole, [])) == 0  # nothing copied: everything deferred
    assert opt._dsw_first_unstaged(Ring(whole, whole)) == n  # all copied: nothing deferred
    # exp_avg fully copied, exp_avg_sq up to element 3000, master up to 5000
    part = [whole[0], (whole[1][0], whole[1][0] + 4 * 3000), (whole[2][0], whole[2][0] + 4 * 5000)]
    assert opt._dsw_first_unstaged(Ring(whole, sorted(part))) == 3000
    # state the snapshot does not read at all never needs protecting
    assert opt._dsw_first_unstaged(Ring([whole[0]], [])) == 0
    assert opt._dsw_first_unstaged(Ring([whole[0]], [whole[0]])) == n
    assert opt._dsw_supported()  # FusedAdamW supports it
