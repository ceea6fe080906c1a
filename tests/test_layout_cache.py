"""LayoutCache fast path: the one-pass hit must rebuild exactly the tree a
full re-plan builds, and any changed tensor leaf must force a re-plan."""

import collections

import torch

from dlrover_wuqiong_amd.flash_checkpoint.layout import LayoutCache, TensorMeta, plan_layout

NT = collections.namedtuple("NT", "a b")


def _state(w, step):
    return {"model": collections.OrderedDict(w=w, b=w[:3]),
            "optimizer": {"state": {0: {"exp_avg": w * 0 + 1, "step": step}},
                          "param_groups": [{"params": [0, 1, 2], "lr": 0.1, "betas": (0.9, 0.95), "nt": NT(1, 2)}]},
            "step": step, "extra": [w, None, "x", (1, 2.0)]}




def test_hit_rebuilds_same_tree_and_misses_on_change():
    w = torch.arange(10.0)
    avg = torch.ones(10)
    cache = LayoutCache()
    sd1 = _state(w, 1)
    sd1["optimizer"]["state"][0]["exp_avg"] = avg
    lay1, _ = cache.plan(sd1)
    sd2 = _state(w, 2)
    sd2["optimizer"]["state"][0]["exp_avg"] = avg
    lay2, tens = cache.plan(sd2)
    ref, _ = plan_layout(sd2)
    assert lay2.meta_tree == ref.meta_tree and lay2.extents is lay1.extents
    assert isinstance(lay2.meta_tree["model"], collections.OrderedDict)
    assert lay2.meta_tree["step"] == 2 and lay2.meta_tree["optimizer"]["state"][0]["step"] == 2
    assert lay2.meta_tree["optimizer"]["param_groups"][0]["nt"] == NT(1, 2)
    assert isinstance(lay2.meta_tree["extra"][0], TensorMeta) and lay2.meta_tree["extra"][3] == (1, 2.0)
    assert len(tens) == 4
    # a different tensor (new storage) -> full re-plan
    sd3 = _state(torch.arange(10.0), 3)
    sd3["optimizer"]["state"][0]["exp_avg"] = avg
    lay3, _ = cache.plan(sd3)
    assert lay3.extents is not lay1.extents
    # non-contiguous leaves are never served from the cache
    sd4 = {"t": torch.arange(12.0).view(3, 4).t()}
    a, _ = cache.plan(sd4)
    b, _ = cache.plan(sd4)
    assert a.extents is not b.extents


def test_device_storages_first_and_gpu_end(monkeypatch):
    """plan_layout puts every device storage before every host one (the
    staging flush writes [0, gpu_end) only); the order inside each group is
    first appearance.  Device tensors are faked by their storage key."""
    import torch

    from dlrover_wuqiong_amd.flash_checkpoint import layout as L

    a, s, b = torch.zeros(1000), torch.tensor(3.0), torch.zeros(500)
    fake_dev = {a.untyped_storage().data_ptr(), b.untyped_storage().data_ptr()}
    orig = L._storage_key

    def key(t):
        k = orig(t)
        return ("cuda", 0, k[2]) if k[2] in fake_dev else k

    monkeypatch.setattr(L, "_storage_key", key)
    lay, _ = L.plan_layout({"a": a, "step": s, "b": b})
    devs = [e.device for e in lay.extents]
    assert devs == ["cuda", "cuda", "cpu"], devs  # the host scalar after both device tensors
    assert lay.gpu_end == max(e.offset + e.nbytes for e in lay.extents if e.device == "cuda")
    assert all(e.offset >= lay.gpu_end for e in lay.cpu_extents())
    metas = lay.meta_tree
    assert metas["a"].offset < metas["b"].offset < metas["step"].offset
