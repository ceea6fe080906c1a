"""Multi-tensor fused AdamW / AGD (``optimizers/multi_tensor.py``,
``csrc/kernels/optim_multi.hip``): CPU reference math vs torch.optim / ATorch
AGD, state-dict layout, auto_accelerate wiring incl. FSDP2 (gloo, 2 ranks)
with a flash-checkpoint round trip; GPU kernel vs the fp32 reference."""

import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import free_port, gpu_available
from dlrover_wuqiong_amd.optimizers.agd import AGD
from dlrover_wuqiong_amd.optimizers.multi_tensor import MultiTensorAdamW, MultiTensorAGD, fused_equivalent


def _params(dtype=torch.float32, device="cpu", seed=0):
    g = torch.Generator().manual_seed(seed)
    shapes = [(37, 19), (1000,), (3, 5, 7), (64, 64), (1,)]
    return [torch.randn(s, generator=g).to(device=device, dtype=dtype).requires_grad_() for s in shapes]


def _grads(ps, step):
    g = torch.Generator().manual_seed(100 + step)
    return [torch.randn(p.shape, generator=g).to(p.device) for p in ps]


def _groups(ps, **extra):
    return [{"params": ps[:3]}, {"params": ps[3:], "weight_decay": 0.0, **extra}]


@pytest.mark.parametrize("adamw", [True, False])
def test_adam_matches_torch(adamw):
    ps, ref = _params(), _params()
    o = MultiTensorAdamW(_groups(ps), lr=1e-2, weight_decay=0.1, adamw=adamw)
    cls = torch.optim.AdamW if adamw else torch.optim.Adam
    r = cls(_groups(ref), lr=1e-2, weight_decay=0.1)
    for s in range(6):
        for a, b, g in zip(ps, ref, _grads(ps, s)):
            a.grad, b.grad = g.clone(), g.clone()
        o.step()
        r.step()
    for a, b in zip(ps, ref):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


def test_agd_matches_reference():
    ps, ref = _params(), _params()
    o = MultiTensorAGD(_groups(ps, clip=0.5), lr=1e-2, weight_decay=0.05, delta=1e-5)
    r = AGD(_groups(ref, clip=0.5), lr=1e-2, weight_decay=0.05, delta=1e-5)
    for s in range(6):
        for a, b, g in zip(ps, ref, _grads(ps, s)):
            a.grad, b.grad = g.clone(), g.clone()
        o.step()
        r.step()
    for a, b in zip(ps, ref):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


def test_bf16_params_keep_fp32_master():
    ps = _params(torch.bfloat16)
    ref = [p.detach().float().clone().requires_grad_() for p in ps]
    o = MultiTensorAdamW(ps, lr=1e-3, weight_decay=0.1)
    r = torch.optim.AdamW(ref, lr=1e-3, weight_decay=0.1)
    assert all("master_param" in o.state[p] for p in ps)
    for s in range(5):
        for a, b, g in zip(ps, ref, _grads(ps, s)):
            a.grad, b.grad = g.to(torch.bfloat16), g.to(torch.bfloat16).float()
        o.step()
        r.step()
    for a, b in zip(ps, ref):
        torch.testing.assert_close(o.state[a]["master_param"], b.detach(), rtol=1e-5, atol=1e-6)
        assert torch.equal(a.detach(), b.detach().to(torch.bfloat16))


def test_grad_clipping_matches_clip_grad_norm():
    ps, ref = _params(), _params()
    o = MultiTensorAdamW(ps, lr=1e-2, max_grad_norm=0.5)
    r = torch.optim.AdamW(ref, lr=1e-2)
    for s in range(4):
        for a, b, g in zip(ps, ref, _grads(ps, s)):
            a.grad, b.grad = 3 * g, 3 * g
        o.step()
        nrm = torch.nn.utils.clip_grad_norm_(ref, 0.5)
        r.step()
        assert abs(float(o.last_grad_norm) - float(nrm)) < 1e-3 * float(nrm)
    for a, b in zip(ps, ref):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


def test_state_is_flat_views_and_load_keeps_them():
    ps = _params()
    o = MultiTensorAdamW(ps, lr=1e-2)
    for a, g in zip(ps, _grads(ps, 0)):
        a.grad = g
    o.step()
    flat = o.flat_state_buffers()[torch.device("cpu")]
    base = flat["exp_avg"].data_ptr()
    ptrs = [o.state[p]["exp_avg"].data_ptr() for p in ps]
    assert all(base <= x < base + flat["exp_avg"].numel() * 4 for x in ptrs)
    sd = o.state_dict()
    saved = {i: {k: (v.clone() if torch.is_tensor(v) else v) for k, v in s.items()} for i, s in sd["state"].items()}
    for a, g in zip(ps, _grads(ps, 1)):
        a.grad = g
    o.step()
    o.load_state_dict({"state": saved, "param_groups": sd["param_groups"]})
    assert [o.state[p]["exp_avg"].data_ptr() for p in ps] == ptrs
    assert o.step_count == 1
    for i, p in enumerate(ps):
        assert torch.equal(o.state[p]["exp_avg"], saved[i]["exp_avg"])


def test_fused_equivalent_mapping():
    assert fused_equivalent(torch.optim.AdamW, {})[0] is MultiTensorAdamW
    cls, args = fused_equivalent(torch.optim.Adam, {"lr": 1.0})
    assert cls is MultiTensorAdamW and args["adamw"] is False and args["weight_decay"] == 0.0
    assert fused_equivalent(torch.optim.AdamW, {"amsgrad": True})[0] is None
    assert fused_equivalent(AGD, {"clip": 1.0})[0] is MultiTensorAGD
    assert fused_equivalent(AGD, {"win": True})[0] is None
    assert fused_equivalent(torch.optim.SGD, {})[0] is None


def test_auto_accelerate_uses_fused_optimizer():
    from dlrover_wuqiong_amd.atorch.auto_accelerate import auto_accelerate

    model = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 4))
    ok, res, _ = auto_accelerate(model, torch.optim.AdamW, optim_args={"lr": 1e-3}, load_strategy=["half"])
    assert ok and isinstance(res.optim, MultiTensorAdamW)
    assert all("master_param" in s for s in res.optim.state.values())
    ok, res, _ = auto_accelerate(model, torch.optim.AdamW, optim_args={"lr": 1e-3}, load_strategy=[],
                                 fused_optimizer=False)
    assert type(res.optim) is torch.optim.AdamW


# ----------------------------------------------------------- FSDP2 (gloo)
def _fsdp_worker(rank, world, port, root, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from torch.distributed.fsdp import fully_shard

        from dlrover_wuqiong_amd.flash_checkpoint.checkpointer import StorageType
        from dlrover_wuqiong_amd.flash_checkpoint.fsdp import FsdpShardCheckpointer

        torch.manual_seed(0)
        model = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 5))
        ref = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 5))
        ref.load_state_dict(model.state_dict())
        for m in model:
            if isinstance(m, torch.nn.Linear):
                fully_shard(m)
        fully_shard(model)
        opt = MultiTensorAdamW(model.parameters(), lr=1e-2, weight_decay=0.1, max_grad_norm=1.0)
        ropt = torch.optim.AdamW(ref.parameters(), lr=1e-2, weight_decay=0.1)

        def train(seed):
            g = torch.Generator().manual_seed(seed)
            x = torch.randn(4, 8, generator=g)
            model(x).pow(2).sum().backward()
            opt.step()
            opt.zero_grad()
            # the replicated reference sees the mean over ranks of the same batch
            ref(x).pow(2).sum().backward()
            torch.nn.utils.clip_grad_norm_(ref.parameters(), 1.0)
            ropt.step()
            ropt.zero_grad()

        for s in range(3):
            train(s)
        full = {k: v.full_tensor() for k, v in model.state_dict().items()}
        ok = all(torch.allclose(full[k], v, rtol=1e-5, atol=1e-6) for k, v in ref.state_dict().items())
        ck = FsdpShardCheckpointer(root)
        assert ck.save_checkpoint(3, model, opt, storage_type=StorageType.MEMORY)
        ck.wait_latest_checkpoint()
        want = {k: v.to_local().clone() for k, v in model.state_dict().items()}
        want_m = [opt.state[p]["exp_avg"].to_local().clone() for p in model.parameters()]
        train(7)
        ck.load_checkpoint(model, opt)
        ok = ok and all(torch.equal(v.to_local(), want[k]) for k, v in model.state_dict().items())
        ok = ok and all(torch.equal(opt.state[p]["exp_avg"].to_local(), w)
                        for p, w in zip(model.parameters(), want_m))
        ok = ok and opt.step_count == 3
        ck.close()
        q.put((rank, bool(ok)))
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback

        q.put((rank, traceback.format_exc() + repr(e)))
    finally:
        dist.destroy_process_group()


def test_fsdp2_multi_tensor_matches_replicated_and_flash_ckpt(tmp_path):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_fsdp_worker, args=(r, 2, port, str(tmp_path), q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {0: True, 1: True}, res


# ----------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("pdtype,gdtype,agd", [(torch.float32, torch.float32, False),
                                               (torch.bfloat16, torch.bfloat16, False),
                                               (torch.bfloat16, torch.float32, False),
                                               (torch.bfloat16, torch.bfloat16, True)])
def test_gpu_kernel_matches_cpu_reference(pdtype, gdtype, agd):
    assert gpu_available()
    dev = torch.device("cuda:0")
    # include a misaligned view (scalar path) and a multi-chunk tensor
    big = torch.randn(3 * 16384 + 77, generator=torch.Generator().manual_seed(3))
    shapes = [(37, 19), (1000,), (64, 64), (1,)]
    g0 = torch.Generator().manual_seed(5)
    cpu = [torch.randn(s, generator=g0) for s in shapes] + [big]
    store = torch.zeros(cpu[1].numel() + 1, dtype=pdtype, device=dev)
    gp = []
    for i, c in enumerate(cpu):
        if i == 1:  # element offset 1: not 16-byte aligned
            v = store[1:].view(c.shape)
            v.data.copy_(c.to(pdtype))
            gp.append(torch.nn.Parameter(v))
        else:
            gp.append(torch.nn.Parameter(c.to(device=dev, dtype=pdtype)))
    rp = [torch.nn.Parameter(p.detach().float().cpu()) for p in gp]
    kw = dict(lr=1e-2, weight_decay=0.1, max_grad_norm=2.0)
    groups = lambda ps: [{"params": ps[:3]}, {"params": ps[3:], "weight_decay": 0.0}]  # noqa: E731
    if agd:
        o, r = MultiTensorAGD(groups(gp), clip=1.0, **kw), MultiTensorAGD(groups(rp), clip=1.0, **kw)
    else:
        o, r = MultiTensorAdamW(groups(gp), **kw), MultiTensorAdamW(groups(rp), **kw)
    for s in range(5):
        for a, b, g in zip(gp, rp, _grads(rp, s)):
            gq = g.to(gdtype)
            if gdtype != pdtype and hasattr(a, "grad_dtype"):
                a.grad_dtype = None  # fp32 grads on bf16 params (e.g. FSDP2 reduce_dtype=fp32)
            a.grad = gq.to(dev)
            b.grad = gq.float()
        o.step()
        r.step()
    torch.cuda.synchronize()
    for a, b in zip(gp, rp):
        w = o.state[a]["master_param"] if "master_param" in o.state[a] else a
        wr = r.state[b]["master_param"] if "master_param" in r.state[b] else b
        torch.testing.assert_close(w.detach().float().cpu(), wr.detach(), rtol=2e-5, atol=2e-5)
        torch.testing.assert_close(o.state[a]["exp_avg_sq"].cpu(), r.state[b]["exp_avg_sq"], rtol=1e-4, atol=1e-7)
    assert abs(float(o.last_grad_norm) - float(r.last_grad_norm)) < 1e-3 * float(r.last_grad_norm)


@pytest.mark.gpu
def test_gpu_multi_tensor_vs_torch_adamw_fp32():
    assert gpu_available()
    dev = torch.device("cuda:0")
    ps = _params(device=dev)
    ref = [p.detach().float().cpu().clone().requires_grad_() for p in ps]
    o = MultiTensorAdamW(ps, lr=3e-3, betas=(0.9, 0.95), weight_decay=0.1)
    r = torch.optim.AdamW(ref, lr=3e-3, betas=(0.9, 0.95), weight_decay=0.1)
    for s in range(8):
        for a, b, g in zip(ps, ref, _grads(ref, s)):
            a.grad, b.grad = g.to(dev), g.clone()
        o.step()
        r.step()
    for a, b in zip(ps, ref):
        torch.testing.assert_close(a.detach().cpu(), b.detach(), rtol=1e-5, atol=1e-5)
