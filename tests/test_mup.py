"""muP: infshapes from base/delta models, parameter classes, optimizer lr
scaling and the coordinate check (update size independent of width) --
parity: ATorch atorch/mup and its tests."""

import torch
import torch.nn as nn


def _mlp(width, mup=True):
    from dlrover_wuqiong_amd.atorch.mup import MupLinear, MupModule, MuReadout

    class M(MupModule):
        def __init__(self):
            super().__init__()
            self.fc1 = MupLinear(16, width, sampler="kaiming_normal")
            self.fc2 = MupLinear(width, width, sampler="kaiming_normal")
            self.out = MuReadout(width, 4, readout_zero_init=False) if mup else nn.Linear(width, 4)

        def forward(self, x):
            return self.out(torch.relu(self.fc2(torch.relu(self.fc1(x)))))

    return M()


def test_infshapes_and_param_groups(tmp_path):
    from dlrover_wuqiong_amd.atorch import mup

    base, delta, target = _mlp(8), _mlp(16), _mlp(64)
    mup.set_base_shapes(target, base, delta=delta, savefile=str(tmp_path / "s.yaml"))
    sh = mup.get_infshapes(target)
    assert sh["fc2.weight"].ninf() == 2 and sh["fc2.weight"].width_mult() == 8.0
    assert sh["fc1.weight"].ninf() == 1 and sh["fc1.bias"].ninf() == 1
    assert sh["out.weight"].ninf() == 1 and sh["out.bias"].ninf() == 0
    # the saved base shapes reproduce the same infshapes
    t2 = _mlp(64)
    mup.set_base_shapes(t2, str(tmp_path / "s.yaml"))
    assert mup.get_infshapes(t2)["fc2.weight"] == sh["fc2.weight"]
    opt = mup.MuAdam(target.parameters(), lr=1e-2, weight_decay=0.1)
    lrs = {id(p): g["lr"] for g in opt.param_groups for p in g["params"]}
    wds = {id(p): g["weight_decay"] for g in opt.param_groups for p in g["params"]}
    assert abs(lrs[id(target.fc2.weight)] - 1e-2 / 8) < 1e-12 and lrs[id(target.fc1.weight)] == 1e-2
    assert abs(wds[id(target.fc2.weight)] - 0.8) < 1e-12
    sgd = mup.MuSGD(target.parameters(), lr=0.1)
    lrs = {id(p): g["lr"] for g in sgd.param_groups for p in g["params"]}
    assert abs(lrs[id(target.fc1.weight)] - 0.8) < 1e-9 and abs(lrs[id(target.fc2.weight)] - 0.1) < 1e-9


def _delta_logits(width, use_mup, lr=1e-3):
    from dlrover_wuqiong_amd.atorch import mup

    torch.manual_seed(0)
    m = _mlp(width, mup=use_mup)
    mup.set_base_shapes(m, _mlp(32, mup=use_mup) if use_mup else None, delta=_mlp(64, mup=use_mup) if use_mup else None)
    m.mup_initial("mup" if use_mup else "sp")
    opt = mup.MuAdam(m.parameters(), lr=lr) if use_mup else torch.optim.AdamW(m.parameters(), lr=lr)
    g = torch.Generator().manual_seed(1)
    x, y = torch.randn(256, 16, generator=g), torch.randn(256, 4, generator=g)
    y0 = m(x).detach()
    for _ in range(3):
        loss = (m(x) - y).square().mean()
        opt.zero_grad()
        loss.backward()
        opt.step()
    return (m(x).detach() - y0).abs().mean().item()


def test_coordinate_check_update_size_width_independent():
    """After a few Adam steps at a fixed lr the change of the logits stays
    O(1) across widths under muP, while under SP it blows up with width."""
    mu = [_delta_logits(w, True) for w in (256, 1024, 4096)]
    sp = [_delta_logits(w, False) for w in (256, 1024, 4096)]
    assert max(mu) / min(mu) < 1.5, mu
    assert sp[-1] / sp[0] > 5.0, sp
