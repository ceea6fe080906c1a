"""elastic_agent/warm_profile.py: the live worker's step recorded once (GEMM
signatures + other aten ops, no random / sync / view ops), replayed on
scratch tensors by a standby (CPU stand-in for the device)."""

import torch
import torch.nn as nn
import torch.nn.functional as F

from dlrover_wuqiong_amd.elastic_agent import warm_profile as wp


def _step(model, x, y):
    loss = F.cross_entropy(model(x), y)
    loss.backward()
    return loss


def test_record_and_replay_on_cpu():
    torch.manual_seed(0)
    model = nn.Sequential(nn.Embedding(50, 16), nn.Linear(16, 32), nn.GELU(), nn.Dropout(0.1), nn.Linear(32, 50))
    x = torch.randint(0, 50, (4, 8))
    y = torch.randint(0, 50, (4, 8))

    def fwd(inp):
        return model(inp).reshape(-1, 50)

    rec = wp._make_recorder("cpu")
    with rec:
        loss = F.cross_entropy(fwd(x), y.reshape(-1))
        loss.backward()
    gemm_ops = {g["op"] for g in rec.seen.values()}
    other = {g["op"] for g in rec.other.values()}
    assert gemm_ops & {"mm", "addmm"}
    assert "embedding" in other or "index_select" in other
    assert not any(w in o for o in other for w in ("rand", "bernoulli", "dropout", "native_dropout"))
    assert not other & wp._VIEW_OPS
    prof = {"gemms": list(rec.seen.values()), "ops": list(rec.other.values())}
    r = wp.replay(prof, device=torch.device("cpu"))
    assert r["gemms"] == len(prof["gemms"]) and r["ops"] >= 0.8 * len(prof["ops"]), r


def test_integer_operands_replay_as_zeros():
    e = wp._enc(torch.tensor([[3, 7]]), "cpu")
    t = wp._dec(e, torch.device("cpu"))
    assert t.dtype == torch.int64 and t.shape == (1, 2) and int(t.abs().sum()) == 0
