"""Lazy gradient zeroing of FlatParams (parallel/flat.py, opt-in
``lazy_zero_grad=True``; ``DWAMD_LAZY_ZERO_GRAD`` overrides): zero_grad() only
opens a generation, the first contribution overwrites, autograd-accumulated
parameters are zeroed just before their first accumulation, and unused
parameters are zeroed when the backward ends."""

import torch
import torch.nn as nn

from dlrover_wuqiong_amd.parallel.flat import FlatParams


class _Net(nn.Module):
    def __init__(self):
        super().__init__()
        self.emb = nn.Embedding(10, 8)
        self.fc = nn.Linear(8, 8)
        self.unused = nn.Linear(8, 8)
        self.head = nn.Linear(8, 3)

    def forward(self, ids):
        return self.head(torch.relu(self.fc(self.emb(ids)))).pow(2).mean()


def _grads(flat):
    return [p.grad.clone() for p in flat.params]


def test_lazy_zero_matches_eager(monkeypatch):
    torch.manual_seed(0)
    ids = torch.randint(0, 10, (4, 5))
    ref_net = _Net()
    net = _Net()
    net.load_state_dict(ref_net.state_dict())
    monkeypatch.delenv("DWAMD_LAZY_ZERO_GRAD", raising=False)
    ref = FlatParams(ref_net, dtype=torch.float32)  # eager: the default
    flat = FlatParams(net, dtype=torch.float32, lazy_zero_grad=True)
    assert flat.lazy_zero and not ref.lazy_zero
    for it in range(3):
        for f, m in ((ref, ref_net), (flat, net)):
            f.zero_grad()
            if f is flat:
                f.grad.fill_(123.0)  # stale values a lazy generation must never expose
                f._fresh = True      # (fill_ above is after zero_grad: still the open generation)
            m(ids).backward()
            if it == 2:  # gradient accumulation: a second backward adds
                m(ids).backward()
        for a, b in zip(_grads(flat), _grads(ref)):
            torch.testing.assert_close(a, b)
        # the unused parameter: zeroed at the end of the backward, not 123
        i = flat.index_of(net.unused.weight)
        assert torch.count_nonzero(flat.params[i].grad) == 0
        assert not flat._fresh


def test_claim_outside_backward_and_finalize(monkeypatch):
    monkeypatch.delenv("DWAMD_LAZY_ZERO_GRAD", raising=False)
    net = _Net()
    flat = FlatParams(net, dtype=torch.float32, lazy_zero_grad=True)
    flat.grad.fill_(5.0)
    flat.zero_grad()
    i = flat.index_of(net.fc.weight)
    assert flat.claim(i) is True      # first writer of the generation: overwrite
    assert flat.claim(i) is False     # a second contribution accumulates
    flat.params[i].grad.fill_(1.0)    # the "overwrite"
    flat.finalize_grads()             # the rest was never written: zeroed
    for j, p in enumerate(flat.params):
        assert torch.all(p.grad == (1.0 if j == i else 0.0))
    assert flat.claim(i) is False     # generation closed: accumulate


def test_env_overrides(monkeypatch):
    monkeypatch.setenv("DWAMD_LAZY_ZERO_GRAD", "0")
    assert not FlatParams(_Net(), dtype=torch.float32, lazy_zero_grad=True).lazy_zero
    monkeypatch.setenv("DWAMD_LAZY_ZERO_GRAD", "1")
    assert FlatParams(_Net(), dtype=torch.float32).lazy_zero
    monkeypatch.delenv("DWAMD_LAZY_ZERO_GRAD")
    assert not FlatParams(_Net(), dtype=torch.float32).lazy_zero
