"""Group-wise int8/int4 quantization + quantized collectives.

CPU: the reference math (ATorch test_quantize.py formula) round-trips
within half a quantization step, int4 packing is high-nibble-first, the
adaptive group rule, and qwZ all-gather / qgZ reduce-scatter / all-reduce
at 2 and 4 gloo ranks against exact sums.  GPU: the HIP kernels against
the fp32 reference (codes equal up to rare rounding ties, params equal)."""

import os

import pytest
import torch

from dlrover_wuqiong_amd.common.rpc import find_free_port
from dlrover_wuqiong_amd.ops.quantization import (Quantizer, choose_groups, dequant_reduce, dequantize,
                                                  dequantize_reference, quantize, quantize_reference)


@pytest.mark.parametrize("bits", [8, 4])
@pytest.mark.parametrize("sym", [True, False])
def test_reference_roundtrip(bits, sym):
    torch.manual_seed(0)
    groups, gs = 16, 256
    x = torch.randn(groups * gs) * torch.linspace(0.1, 10, groups).repeat_interleave(gs)
    c, p = quantize_reference(x, groups, bits, sym)
    assert c.dtype == torch.int8 and c.numel() == x.numel() // (8 // bits) and p.shape == (groups, 2)
    y = dequantize_reference(c, p, groups, bits)
    step = p[:, 0].repeat_interleave(gs)  # 1/scale = one quantization step
    # half a step, except the top of the range: 2^bits codes over [min, max] (or
    # [-absmax, absmax]) map the maximum to qmax + 1, clamped: one step
    err = (y - x).abs()
    assert (err <= step * (1 + 1e-4) + 1e-6).all()
    assert float((err > 0.5 * step + 1e-6).float().mean()) < 0.01


def test_int4_packing_order():
    x = torch.tensor([-8.0, 7.0, 1.0, -1.0, 0.0, 3.0, -3.0, 2.0]) * 1.0
    c, p = quantize_reference(x, 1, 4, symmetric=True)
    codes = torch.round(x * p[0, 0].reciprocal()).clamp(-8, 7).to(torch.int32)
    assert int(c[0].to(torch.int32) & 0xFF) == ((int(codes[0]) & 0xF) << 4 | (int(codes[1]) & 0xF))


def test_choose_groups_and_quantizer():
    assert choose_groups(8000) == 1
    g = choose_groups(1600 * 6400)
    assert (1600 * 6400) % (8 * g) == 0 and (1600 * 6400) / g <= 16000
    q = Quantizer()
    x = torch.randn(4096 * 3)
    c, p = q.quantize(x)
    y = q.dequantize(c, p)
    assert (y - x).abs().max() <= p[:, 0].max() + 1e-6


def _coll_worker(rank, world, port, out_q, bits):
    import torch.distributed as dist

    from dlrover_wuqiong_amd.parallel.quantized_comm import (quantized_all_gather, quantized_all_reduce,
                                                             quantized_reduce_scatter)

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.manual_seed(rank)
        x = torch.randn(world * 1024)
        allx = [torch.empty_like(x) for _ in range(world)]
        dist.all_gather(allx, x)
        exact_sum = torch.stack(allx).sum(0)
        step = 1.0 / (2 ** (bits - 1))
        # qwZ all-gather of a shard
        shard = x[:1024]
        g = quantized_all_gather(shard, bits=bits, group_size=256)
        ref = torch.cat([a[:1024] for a in allx])
        e_ag = float(((g - ref).abs().view(-1, 256).amax(-1) / ref.abs().view(-1, 256).amax(-1)).max())
        # qgZ reduce-scatter
        rs = quantized_reduce_scatter(x, bits=bits, group_size=256)
        ref_rs = exact_sum[rank * 1024:(rank + 1) * 1024]
        scale = torch.stack(allx)[:, rank * 1024:(rank + 1) * 1024].abs().amax()
        e_rs = float((rs - ref_rs).abs().max() / scale)
        # all-reduce (mean)
        y = x.clone()
        quantized_all_reduce(y, bits=bits, group_size=256, average=True)
        e_ar = float((y - exact_sum / world).abs().max() / torch.stack(allx).abs().amax())
        out_q.put((rank, e_ag, e_rs, e_ar, step))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,bits", [(2, 8), (4, 8), (2, 4)])
def test_quantized_collectives(world, bits):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = find_free_port()
    ps = [ctx.Process(target=_coll_worker, args=(r, world, port, q, bits)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=180) for _ in ps]
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    for rank, e_ag, e_rs, e_ar, step in res:
        assert e_ag <= step * 1.001, (rank, e_ag)
        assert e_rs <= world * step, (rank, e_rs)
        assert e_ar <= 2 * step, (rank, e_ar)


@pytest.mark.gpu
@pytest.mark.parametrize("bits", [8, 4])
@pytest.mark.parametrize("sym", [True, False])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_quant_kernels_gpu(bits, sym, dtype):
    torch.manual_seed(1)
    groups, gs = 300, 2048
    x = (torch.randn(groups * gs, device="cuda") *
         torch.linspace(0.01, 50, groups, device="cuda").repeat_interleave(gs)).to(dtype)
    x[:gs] = 0.0  # a constant group
    c, p = quantize(x, groups, bits, sym)
    c_ref, p_ref = quantize_reference(x.cpu(), groups, bits, sym)
    torch.cuda.synchronize()
    assert torch.allclose(p.cpu(), p_ref, rtol=1e-5, atol=1e-4)  # zero points: fp32 rounding of qmin - min*scale
    if bits == 8:
        diff = (c.cpu().to(torch.int32) - c_ref.to(torch.int32)).abs()
    else:
        from dlrover_wuqiong_amd.ops.quantization import _unpack4

        diff = (_unpack4(c.cpu()) - _unpack4(c_ref)).abs()
    # ties at x*scale + zp = k + 0.5 round either way under fp32 evaluation-order differences
    assert int(diff.max()) <= 1 and float((diff > 0).float().mean()) < 1e-3
    y = dequantize(c, p, groups, bits, sym, dtype=torch.float32)
    y_ref = dequantize_reference(c.cpu(), p.cpu(), groups, bits)
    assert torch.allclose(y.cpu(), y_ref, rtol=1e-6, atol=1e-6)
    # dequant-reduce of 3 chunks (the qgZ receive side) + accumulate, bf16 out
    n_src, elems = 3, 8 * gs
    srcs = [torch.randn(elems, device="cuda", dtype=dtype) for _ in range(n_src)]
    qs = [quantize(s, elems // gs, bits, sym) for s in srcs]
    codes = torch.stack([a for a, _ in qs])
    params = torch.stack([b for _, b in qs])
    out = torch.ones(elems, device="cuda", dtype=torch.bfloat16)
    dequant_reduce(codes, params, n_src, elems, gs, bits, out=out, accumulate=True)
    ref = 1.0 + sum(dequantize_reference(a.cpu(), b.cpu(), elems // gs, bits) for a, b in qs)
    assert torch.allclose(out.float().cpu(), ref, rtol=1e-2, atol=1e-2)


def _rccl_worker(rank, world, port, out_q):
    import torch.distributed as dist

    from dlrover_wuqiong_amd.parallel.quantized_comm import (quantized_all_gather, quantized_all_reduce,
                                                             quantized_reduce_scatter)

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=world)
    try:
        x = torch.randn(1 << 20, device="cuda", dtype=torch.bfloat16)
        g = quantized_all_gather(x, bits=8)
        rs = quantized_reduce_scatter(x, bits=8)
        y = x.float().clone()
        quantized_all_reduce(y, bits=4)
        torch.cuda.synchronize()
        amax = float(x.float().abs().max())
        out_q.put((float((g.float() - x.float()).abs().max()) / amax, float((rs.float() - x.float()).abs().max()) / amax,
                   float((y - x.float()).abs().max()) / amax))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_quantized_collectives_rccl_single_rank():
    """The RCCL code paths (all_gather_into_tensor / all_to_all_single) and
    the HIP kernels together, in a one-rank RCCL world (one GPU per box)."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(0, 1, find_free_port(), q))
    p.start()
    e_ag, e_rs, e_ar = q.get(timeout=120)
    p.join(60)
    assert p.exitcode == 0
    assert e_ag <= 1 / 128 * 1.01 and e_rs <= 1 / 128 * 1.01 and e_ar <= 2 / 8 * 1.01, (e_ag, e_rs, e_ar)
