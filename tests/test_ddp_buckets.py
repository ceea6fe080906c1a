"""FlatDDP bucket readiness (CPU, gloo, 2 ranks).

The fused ops write flat gradients themselves and return ``None`` to
autograd, which still fires the post-accumulate hook; a parameter can also be
used twice, or be unused in one step and used in the next (MoE experts).  A
bucket must never be reduced before every gradient in it has landed: every
launched all-reduce is recorded with a snapshot of its slice, and the
snapshot must equal the finished local gradient.
"""

import os

import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn

from conftest import free_port
from dlrover_wuqiong_amd.ops._grad import notify


class _DirectMul(torch.autograd.Function):
    """Like the fused ops: accumulates into ``w.grad`` and returns None."""

    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x)
        ctx.w = w
        return x * w

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        ctx.w.grad.add_((g * x).sum(0))
        notify(ctx.w)
        return g * ctx.w.detach(), None


class _Net(nn.Module):
    def __init__(self):
        super().__init__()
        self.a = nn.Parameter(torch.randn(64))   # direct-grad op
        self.b = nn.Parameter(torch.randn(64))   # used twice (autograd)
        self.c = nn.Parameter(torch.randn(64))   # used only when use_c
        self.d = nn.Parameter(torch.randn(64))   # direct op, applied twice

    def forward(self, x, use_c):
        h = _DirectMul.apply(x, self.a)
        h = h * self.b + torch.tanh(h) * self.b
        h = _DirectMul.apply(_DirectMul.apply(h, self.d), self.d)
        if use_c:
            h = h * self.c
        return (h ** 2).mean()


def _worker(rank, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        from dlrover_wuqiong_amd.parallel.ddp import FlatDDP
        from dlrover_wuqiong_amd.parallel.flat import FlatParams

        dist.init_process_group("gloo", rank=rank, world_size=2)
        torch.manual_seed(0)
        net = _Net()
        flat = FlatParams(net)
        ddp = FlatDDP(net, flat, bucket_mb=1)
        early = []  # (start, end, snapshot) of every bucket launched from a hook
        real = dist.all_reduce

        def recording(t, group=None, async_op=False):
            early.append((t.data_ptr(), t.clone()))
            return real(t, group=group, async_op=async_op)

        dist.all_reduce = recording
        errors = []
        for step, use_c in enumerate([False, True, True, False]):
            early.clear()
            flat.zero_grad()
            x = torch.randn(8, 64, generator=torch.Generator().manual_seed(10 * step + rank))
            ddp(x, use_c).backward()
            local = flat.grad.clone()
            ddp.finish_gradient_sync()
            for ptr, snap in early:
                off = (ptr - flat.grad.data_ptr()) // flat.grad.element_size()
                if not torch.equal(snap, local[off:off + snap.numel()]):
                    errors.append(f"step {step}: bucket at {off} reduced before its gradients landed")
            ref = local.clone()
            real(ref)
            if not torch.allclose(ref, flat.grad):
                errors.append(f"step {step}: reduced gradient differs from the sum")
        dist.all_reduce = real
        q.put((rank, errors))
    except Exception as e:  # pragma: no cover
        q.put((rank, [repr(e)]))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_flat_ddp_buckets_launch_only_when_complete():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=30)
    assert all(not errs for _, errs in res), res


def _qworker(rank, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        from dlrover_wuqiong_amd.parallel.ddp import FlatDDP
        from dlrover_wuqiong_amd.parallel.flat import FlatParams

        dist.init_process_group("gloo", rank=rank, world_size=2)
        torch.manual_seed(0)
        net = nn.Sequential(nn.Linear(64, 256), nn.Tanh(), nn.Linear(256, 64))
        import copy

        ref_net = copy.deepcopy(net)
        flat = FlatParams(net)
        ddp = FlatDDP(net, flat, bucket_mb=1, grad_comm_bits=8)
        errs = []
        for step in range(3):
            flat.zero_grad()
            ref_net.zero_grad()
            x = torch.randn(16, 64, generator=torch.Generator().manual_seed(10 * step + rank))
            (ddp(x) ** 2).mean().backward()
            (ref_net(x) ** 2).mean().backward()
            ddp.finish_gradient_sync()
            got = torch.cat([p.grad.reshape(-1) for p in net.parameters()])
            ref = torch.cat([p.grad.reshape(-1) for p in ref_net.parameters()])
            dist.all_reduce(ref)
            rel = float((got - ref).abs().max() / ref.abs().max())
            if rel > 2 / 128:
                errs.append(f"step {step}: quantized reduce error {rel:.4f}")
        # both replicas hold the same (quantized) sum
        g = flat.grad.clone()
        other = [torch.empty_like(g) for _ in range(2)]
        dist.all_gather(other, g)
        if not torch.equal(other[0], other[1]):
            errs.append("replicas differ")
        q.put((rank, errs))
    except Exception as e:  # pragma: no cover
        q.put((rank, [repr(e)]))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_flat_ddp_quantized_grad_reduce():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_qworker, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=30)
    assert all(not errs for _, errs in res), res
