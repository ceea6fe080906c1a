"""GPT-style MLP (c_fc -> bias + tanh-GELU -> c_proj) with the bias and the
GELU gradient fused into hipBLASLt GEMM epilogues
(``csrc/kernels/gemm_epilogue.hip``):

  forward   pre = x W1^T + b1                 (bias epilogue writes the pre-activation)
            g = gelu_tanh(pre)                (one read, one write)
            y = g W2^T + b2                   (bias epilogue)
  backward  dW2 += dy^T g, db2 += colsum(dy)
            dh (, db1) = DGELU[_BGRAD](dy W2, pre)   (epilogue forms), or
                         dy W2, then one gelu_bwd + colsum pass (default)
            dW1 += dh^T x, dx = dh W1

Gradients of flat-buffer parameters accumulate in place (``_grad.py``).

Measured on the GPT2-1.5B MLP (8192 x 1600 -> 6400 -> 1600, 1x MI355X,
``scripts/bench_mlp.py``, ``profiles/r2/bench_mlp.jsonl``): the forward
(bias epilogue + GELU-only pass) takes 0.315 ms vs 0.40 for GEMM + bias-GELU
kernel; in the backward hipBLASLt's DGELU / DGELU_BGRAD epilogue kernels are
SLOWER than the plain dgrad GEMM + ``gelu_bwd`` + ``colsum`` (1.66-1.73 vs
1.12 ms fwd+bwd), so the backward defaults to the unfused kernels;
``DWAMD_MLP_BWD_EPILOGUE=bgrad|dgelu`` selects the epilogue forms (per GEMM
shape they fall back when hipBLASLt has no algorithm:
``profiles/r2/hipblaslt_epilogue_probe.txt``).

Parity: ATorch fused bias-GELU MLP (``atorch/modules/transformer/layers.py``
``MLPLayer`` with fused dense-gelu) / Megatron ``bias_gelu_fusion``.
"""

import os

import torch
import torch.nn.functional as F

from . import _hip
from ._grad import claim, direct_grad, notify

_EPI_UNSUPPORTED = -100
_BWD_MODE = {}  # (M, N1, N2) -> "bgrad" | "dgelu" | "unfused"
_BWD_DEFAULT = os.environ.get("DWAMD_MLP_BWD_EPILOGUE", "unfused")


def _acc(param, grad_fn):
    """Write into the flat gradient of ``param`` or return the grad.
    ``grad_fn(g, overwrite)``: g is the flat view (None: return the grad);
    overwrite on the first contribution since a lazy zero_grad."""
    g = direct_grad(param)
    if g is not None:
        grad_fn(g, claim(param))
        notify(param)
        return None
    return grad_fn(None, False)


def _mm_into(g, a, b, overwrite):
    return torch.mm(a, b, out=g) if overwrite else g.addmm_(a, b)


class _FusedMLPFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2):
        shape = x.shape
        x2 = x.reshape(-1, shape[-1]).contiguous()
        N1 = w1.shape[0]
        pre = F.linear(x2, w1, b1)  # hipBLASLt bias epilogue
        g = torch.empty_like(pre)
        _hip.check(_hip.lib().dw_bias_gelu_fwd(_hip.ptr(pre), None, _hip.ptr(g), None, pre.numel(), N1,
                                               _hip.stream()), "gelu_fwd")
        y = F.linear(g, w2, b2)
        ctx.save_for_backward(x2, w1, pre, g, w2)
        ctx.params = (w1, b1, w2, b2)
        ctx.shape = shape
        ctx.out_bias, ctx.out_bias_folded = b2, False  # see ops/linear.py
        return y.view(*shape[:-1], w2.shape[0])

    @staticmethod
    def backward(ctx, dy):
        from .activation import colsum

        x2, w1, pre, g, w2 = ctx.saved_tensors
        p_w1, p_b1, p_w2, p_b2 = ctx.params
        N2, N1 = w2.shape
        dy2 = dy.reshape(-1, N2).contiguous().to(x2.dtype)
        M = dy2.shape[0]
        dw2 = _acc(p_w2, lambda gb, ow: _mm_into(gb, dy2.t(), g, ow) if gb is not None else dy2.t() @ g)
        db2 = None if ctx.out_bias_folded else _acc(
            p_b2, lambda gb, ow: colsum(dy2, out=gb, accumulate=not ow) if gb is not None else colsum(dy2, p_b2.dtype))
        key = (M, N1, N2)
        dh = torch.empty(M, N1, device=dy.device, dtype=x2.dtype)
        db1_f = None
        db1_done = False
        mode = _BWD_MODE.get(key, _BWD_DEFAULT)
        if mode == "bgrad":
            db1_f = torch.empty(N1, device=dy.device, dtype=torch.float32)
            rc = _hip.lib().dw_gemm_dgelu_bgrad(_hip.ptr(dy2), _hip.ptr(w2), _hip.ptr(pre), _hip.ptr(dh),
                                                _hip.ptr(db1_f), M, N1, N2, _hip.stream())
            if rc == _EPI_UNSUPPORTED:
                mode = _BWD_MODE[key] = "dgelu"
                db1_f = None
            else:
                _hip.check(rc, "gemm_dgelu_bgrad")
        if mode == "dgelu":
            rc = _hip.lib().dw_gemm_dgelu(_hip.ptr(dy2), _hip.ptr(w2), _hip.ptr(pre), _hip.ptr(dh), M, N1, N2,
                                          _hip.stream())
            if rc == _EPI_UNSUPPORTED:
                mode = _BWD_MODE[key] = "unfused"
            else:
                _hip.check(rc, "gemm_dgelu")
        if mode == "unfused":
            # dgrad GEMM, then ONE pass: dh = dg * gelu'(pre) and db1 = colsum(dh)
            dg = (dy2 @ w2).contiguous()
            ws = _hip.zeroed_workspace(N1 + (N1 + 511) // 512, dy.device)
            gb1 = direct_grad(p_b1)
            if gb1 is not None and gb1.dtype in (torch.bfloat16, torch.float32):
                # the finish kernel adds db1 into the flat gradient itself (no
                # fp32 temporary + cast + add_ launches)
                _hip.check(_hip.lib().dw_gelu_bwd_dbias(_hip.ptr(dg), _hip.ptr(pre), _hip.ptr(dh), M, N1,
                                                        _hip.ptr(ws), _hip.ptr(gb1),
                                                        int(gb1.dtype == torch.float32), int(not claim(p_b1)),
                                                        _hip.stream(), _hip.det_scratch(M, N1, 1, dy.device)),
                           "gelu_bwd_dbias")
                notify(p_b1)
                db1_done = True
            else:
                db1_f = torch.empty(N1, device=dy.device, dtype=torch.float32)
                _hip.check(_hip.lib().dw_gelu_bwd_dbias(_hip.ptr(dg), _hip.ptr(pre), _hip.ptr(dh), M, N1,
                                                        _hip.ptr(ws), _hip.ptr(db1_f), 1, 0, _hip.stream(),
                                                        _hip.det_scratch(M, N1, 1, dy.device)),
                           "gelu_bwd_dbias")
        _BWD_MODE.setdefault(key, mode)
        db1 = None
        if not db1_done:
            if db1_f is None:
                db1_f = colsum(dh, torch.float32)
            db1 = _acc(p_b1, lambda gb, ow: (gb.copy_ if ow else gb.add_)(db1_f.to(gb.dtype))
                       if gb is not None else db1_f.to(p_b1.dtype))
        dw1 = _acc(p_w1, lambda gb, ow: _mm_into(gb, dh.t(), x2, ow) if gb is not None else dh.t() @ x2)
        dx = (dh @ w1).view(ctx.shape)
        return dx, dw1, db1, dw2, db2


def fused_gelu_mlp(x, fc, proj):
    """``proj(gelu_tanh(fc(x)))`` for two ``nn.Linear``-like modules with
    biases; HIP epilogue-fused on the GPU, plain PyTorch elsewhere."""
    if _hip.use_hip(x) and x.dtype == torch.bfloat16 and fc.bias is not None and proj.bias is not None \
            and fc.weight.dtype == torch.bfloat16 and proj.weight.dtype == torch.bfloat16:
        return _FusedMLPFn.apply(x, fc.weight, fc.bias, proj.weight, proj.bias)
    return proj(F.gelu(fc(x), approximate="tanh"))
