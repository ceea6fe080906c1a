"""Megatron-style tensor parallelism (+ sequence parallelism) over RCCL.

Layers: ``ColumnParallelLinear`` (weight split along the output dim),
``RowParallelLinear`` (split along the input dim, partial sums reduced),
``VocabParallelEmbedding`` and ``vocab_parallel_cross_entropy`` (logits stay
sharded over the vocabulary: only [tokens] max / sum-exp / target-logit
vectors are all-reduced, never the [tokens, vocab] logits).

With ``sequence_parallel=True`` activations between TP regions are sharded
along the sequence (dim 0 of [S, B, H] / flattened tokens): the column layer
all-gathers its input and the row layer reduce-scatters its output, replacing
the all-reduce (same bytes on the wire, 1/tp of the activation memory for
norms / dropout / residuals).

MI355X notes: TP groups come innermost from ``parallel.state`` /
``atorch.distributed`` so they span GPUs of one node; every GPU pair of an
MI355X node has a direct xGMI link, and RCCL rings over them run at per-link
bandwidth, so TP=8 in-node is the natural maximum.

Parity: ATorch ``atorch/modules/distributed_modules/layers.py``
(``ColumnParallelLinear``, ``RowParallelLinear``, ``VocabParallelEmbedding``)
and ``mappings.py`` (copy / reduce / scatter / gather regions), Megatron
``core/tensor_parallel``.
"""

import os
from typing import Optional

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F


def _ws(group) -> int:
    return dist.get_world_size(group) if dist.is_initialized() else 1


def _rk(group) -> int:
    return dist.get_rank(group) if dist.is_initialized() else 0


# ------------------------------------------------------------- mappings
def _reduce(x, group):
    if _ws(group) == 1:
        return x
    x = x.contiguous()
    dist.all_reduce(x, group=group)
    return x


def _split_last(x, group):
    n = _ws(group)
    if n == 1:
        return x
    return torch.tensor_split(x, n, dim=-1)[_rk(group)].contiguous()


def _gather_last(x, group):
    n = _ws(group)
    if n == 1:
        return x
    x = x.contiguous()
    out = [torch.empty_like(x) for _ in range(n)]
    dist.all_gather(out, x, group=group)
    return torch.cat(out, dim=-1)


def _gather_first(x, group):
    n = _ws(group)
    if n == 1:
        return x
    x = x.contiguous()
    out = torch.empty((n * x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    dist.all_gather_into_tensor(out, x, group=group)
    return out


def _reduce_scatter_first(x, group):
    n = _ws(group)
    if n == 1:
        return x
    x = x.contiguous()
    assert x.shape[0] % n == 0, f"sequence dim {x.shape[0]} not divisible by tp {n}"
    out = torch.empty((x.shape[0] // n,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    dist.reduce_scatter_tensor(out, x, group=group)
    return out


def _split_first(x, group):
    n = _ws(group)
    if n == 1:
        return x
    return torch.tensor_split(x, n, dim=0)[_rk(group)].contiguous()


class _CopyToRegion(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return x

    @staticmethod
    def backward(ctx, g):
        return _reduce(g, ctx.group), None


class _ReduceFromRegion(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        return _reduce(x, group)

    @staticmethod
    def backward(ctx, g):
        return g, None


class _ScatterToRegion(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return _split_last(x, group)

    @staticmethod
    def backward(ctx, g):
        return _gather_last(g, ctx.group), None


class _GatherFromRegion(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return _gather_last(x, group)

    @staticmethod
    def backward(ctx, g):
        return _split_last(g, ctx.group), None


class _GatherFromSequenceRegion(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group, grad_reduce_scatter=True):
        ctx.group, ctx.rs = group, grad_reduce_scatter
        return _gather_first(x, group)

    @staticmethod
    def backward(ctx, g):
        return (_reduce_scatter_first(g, ctx.group) if ctx.rs else _split_first(g, ctx.group)), None, None


class _ReduceScatterToSequenceRegion(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return _reduce_scatter_first(x, group)

    @staticmethod
    def backward(ctx, g):
        return _gather_first(g, ctx.group), None


class _ScatterToSequenceRegion(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return _split_first(x, group)

    @staticmethod
    def backward(ctx, g):
        return _gather_first(g, ctx.group), None


def copy_to_tensor_parallel_region(x, group=None):
    return _CopyToRegion.apply(x, group)


def reduce_from_tensor_parallel_region(x, group=None):
    return _ReduceFromRegion.apply(x, group)


def scatter_to_tensor_parallel_region(x, group=None):
    return _ScatterToRegion.apply(x, group)


def gather_from_tensor_parallel_region(x, group=None):
    return _GatherFromRegion.apply(x, group)


def gather_from_sequence_parallel_region(x, group=None, tensor_parallel_output_grad=True):
    return _GatherFromSequenceRegion.apply(x, group, tensor_parallel_output_grad)


def reduce_scatter_to_sequence_parallel_region(x, group=None):
    return _ReduceScatterToSequenceRegion.apply(x, group)


def scatter_to_sequence_parallel_region(x, group=None):
    return _ScatterToSequenceRegion.apply(x, group)


class _ColumnLinearOverlap(torch.autograd.Function):
    """Column-parallel Linear with its communication overlapped with GEMMs
    (ATorch ``LinearWithGradAccumulationAndAsyncCommunication``,
    ``modules/distributed_modules/layers.py:90-158``; Megatron's
    ``async_tensor_model_parallel_allreduce``).

    Forward, sequence parallel: the all-gather of the sequence shards is
    issued async and this rank's own rows are multiplied while the other
    ranks' rows are in flight; the rest follows once they landed.
    Backward: dX = dY W is computed first and its all-reduce (or, with SP,
    reduce-scatter) is issued async; the weight-gradient GEMM dW = dY^T X
    (plus db) runs underneath it -- on MI355X the RCCL kernel on its own
    stream shares the CUs with the hipBLASLt GEMM instead of serialising.
    With SP the input is re-gathered in backward (only the local shard is
    saved: 1/tp of the activation memory), that gather overlapping dX."""

    @staticmethod
    def forward(ctx, x, weight, bias, group, sp):
        ctx.group, ctx.sp, ctx.has_bias = group, sp, bias is not None
        if sp:
            n, r = _ws(group), _rk(group)
            xc = x.contiguous()
            full = torch.empty((n * xc.shape[0],) + tuple(xc.shape[1:]), dtype=xc.dtype, device=xc.device)
            work = dist.all_gather_into_tensor(full, xc, group=group, async_op=True)
            rows = xc.shape[0]
            y_own = F.linear(xc, weight, bias)  # under the gather
            work.wait()
            y = torch.empty((full.shape[0],) + tuple(y_own.shape[1:]), dtype=y_own.dtype, device=y_own.device)
            y[r * rows:(r + 1) * rows] = y_own
            if r > 0:
                y[:r * rows] = F.linear(full[:r * rows], weight, bias)
            if r < n - 1:
                y[(r + 1) * rows:] = F.linear(full[(r + 1) * rows:], weight, bias)
            ctx.save_for_backward(xc, weight)
            return y
        ctx.save_for_backward(x, weight)
        return F.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, g):
        x, weight = ctx.saved_tensors
        group, sp = ctx.group, ctx.sp
        g = g.contiguous()
        gather = None
        if sp:
            n = _ws(group)
            total = torch.empty((n * x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
            gather = dist.all_gather_into_tensor(total, x, group=group, async_op=True)
        else:
            total = x
        # (under autocast the forward GEMMs ran in g's dtype: so do these)
        dx = g.matmul(weight.to(g.dtype))
        if gather is not None:
            gather.wait()
        if sp:
            out = torch.empty((dx.shape[0] // _ws(group),) + tuple(dx.shape[1:]), dtype=dx.dtype, device=dx.device)
            red = dist.reduce_scatter_tensor(out, dx.contiguous(), group=group, async_op=True)
        else:
            out = dx
            red = dist.all_reduce(dx, group=group, async_op=True)
        g2 = g.reshape(-1, g.shape[-1])
        dw = g2.t().matmul(total.reshape(-1, total.shape[-1]).to(g2.dtype))  # under the collective
        db = g2.sum(0) if ctx.has_bias else None
        red.wait()
        return (out.to(x.dtype), dw.to(weight.dtype), (db.to(weight.dtype) if db is not None else None), None,
                None)


def column_parallel_linear(x, weight, bias, group, sequence_parallel=False):
    """Y = X W^T (+ b) for a column shard W, communication overlapped with
    the GEMMs (see :class:`_ColumnLinearOverlap`)."""
    if _ws(group) == 1:
        return F.linear(x, weight, bias)
    return _ColumnLinearOverlap.apply(x, weight, bias, group, sequence_parallel)


def _default_tp_group():
    from . import state

    return state.get_tensor_model_parallel_group()


# --------------------------------------------------------------- layers
class ColumnParallelLinear(nn.Module):
    """Y = X A^T with A split along the output features: rank r holds rows
    [r*out/tp, (r+1)*out/tp).  ``gather_output`` all-gathers Y."""

    def __init__(self, in_features: int, out_features: int, bias: bool = True, gather_output: bool = False,
                 sequence_parallel: bool = False, group=None, dtype=None, device=None,
                 init_method=nn.init.xavier_normal_, skip_bias_add: bool = False):
        super().__init__()
        self.group = group if group is not None else _default_tp_group()
        self.tp = _ws(self.group)
        assert out_features % self.tp == 0, f"out_features {out_features} not divisible by tp {self.tp}"
        self.in_features, self.out_features = in_features, out_features
        self.out_per_rank = out_features // self.tp
        self.gather_output = gather_output
        self.sequence_parallel = sequence_parallel
        self.skip_bias_add = skip_bias_add
        # comm / GEMM overlap (DWAMD_TP_OVERLAP=0: the plain blocking mappings)
        self.overlap_comm = os.environ.get("DWAMD_TP_OVERLAP", "1") == "1"
        self.weight = nn.Parameter(torch.empty(self.out_per_rank, in_features, dtype=dtype, device=device))
        self.bias = nn.Parameter(torch.zeros(self.out_per_rank, dtype=dtype, device=device)) if bias else None
        init_method(self.weight)
        self.weight.tensor_model_parallel = True
        self.weight.partition_dim = 0

    @classmethod
    def from_linear(cls, lin: nn.Linear, group=None, **kw) -> "ColumnParallelLinear":
        m = cls(lin.in_features, lin.out_features, lin.bias is not None, group=group, dtype=lin.weight.dtype,
                device=lin.weight.device, init_method=lambda w: None, **kw)
        r = _rk(m.group)
        with torch.no_grad():
            m.weight.copy_(lin.weight[r * m.out_per_rank:(r + 1) * m.out_per_rank])
            if m.bias is not None:
                m.bias.copy_(lin.bias[r * m.out_per_rank:(r + 1) * m.out_per_rank])
        return m

    def forward(self, x):
        bias = None if self.skip_bias_add else self.bias
        if self.overlap_comm and torch.is_grad_enabled():
            y = column_parallel_linear(x, self.weight, bias, self.group, self.sequence_parallel)
        else:
            if self.sequence_parallel:
                x = gather_from_sequence_parallel_region(x, self.group)
            else:
                x = copy_to_tensor_parallel_region(x, self.group)
            y = F.linear(x, self.weight, bias)
        if self.gather_output:
            y = gather_from_tensor_parallel_region(y, self.group)
        return (y, self.bias) if self.skip_bias_add else y


class RowParallelLinear(nn.Module):
    """Y = X A^T with A split along the input features; partial products are
    all-reduced (or reduce-scattered along the sequence with SP)."""

    def __init__(self, in_features: int, out_features: int, bias: bool = True, input_is_parallel: bool = True,
                 sequence_parallel: bool = False, group=None, dtype=None, device=None,
                 init_method=nn.init.xavier_normal_, skip_bias_add: bool = False):
        super().__init__()
        self.group = group if group is not None else _default_tp_group()
        self.tp = _ws(self.group)
        assert in_features % self.tp == 0, f"in_features {in_features} not divisible by tp {self.tp}"
        self.in_features, self.out_features = in_features, out_features
        self.in_per_rank = in_features // self.tp
        self.input_is_parallel = input_is_parallel
        self.sequence_parallel = sequence_parallel
        self.skip_bias_add = skip_bias_add
        self.weight = nn.Parameter(torch.empty(out_features, self.in_per_rank, dtype=dtype, device=device))
        self.bias = nn.Parameter(torch.zeros(out_features, dtype=dtype, device=device)) if bias else None
        init_method(self.weight)
        self.weight.tensor_model_parallel = True
        self.weight.partition_dim = 1
        if self.bias is not None and sequence_parallel:
            self.bias.sequence_parallel = True  # its grad must be all-reduced across TP

    @classmethod
    def from_linear(cls, lin: nn.Linear, group=None, **kw) -> "RowParallelLinear":
        m = cls(lin.in_features, lin.out_features, lin.bias is not None, group=group, dtype=lin.weight.dtype,
                device=lin.weight.device, init_method=lambda w: None, **kw)
        r = _rk(m.group)
        with torch.no_grad():
            m.weight.copy_(lin.weight[:, r * m.in_per_rank:(r + 1) * m.in_per_rank])
            if m.bias is not None:
                m.bias.copy_(lin.bias)
        return m

    def forward(self, x):
        if not self.input_is_parallel:
            x = scatter_to_tensor_parallel_region(x, self.group)
        y = F.linear(x, self.weight)
        if self.sequence_parallel:
            y = reduce_scatter_to_sequence_parallel_region(y, self.group)
        else:
            y = reduce_from_tensor_parallel_region(y, self.group)
        if self.skip_bias_add:
            return y, self.bias
        return y + self.bias if self.bias is not None else y


class VocabParallelEmbedding(nn.Module):
    """Embedding table split along the vocabulary; out-of-range tokens give
    zeros locally and the partial lookups are all-reduced."""

    def __init__(self, num_embeddings: int, embedding_dim: int, group=None, dtype=None, device=None,
                 init_method=nn.init.normal_):
        super().__init__()
        self.group = group if group is not None else _default_tp_group()
        self.tp = _ws(self.group)
        r = _rk(self.group)
        per = (num_embeddings + self.tp - 1) // self.tp
        self.vocab_start = r * per
        self.vocab_end = min(num_embeddings, (r + 1) * per)
        self.num_embeddings, self.embedding_dim = num_embeddings, embedding_dim
        self.weight = nn.Parameter(torch.empty(per, embedding_dim, dtype=dtype, device=device))
        init_method(self.weight)
        self.weight.tensor_model_parallel = True
        self.weight.partition_dim = 0

    @classmethod
    def from_embedding(cls, emb: nn.Embedding, group=None) -> "VocabParallelEmbedding":
        m = cls(emb.num_embeddings, emb.embedding_dim, group=group, dtype=emb.weight.dtype,
                device=emb.weight.device, init_method=lambda w: None)
        with torch.no_grad():
            m.weight.zero_()
            n = m.vocab_end - m.vocab_start
            m.weight[:n].copy_(emb.weight[m.vocab_start:m.vocab_end])
        return m

    def forward(self, ids):
        if self.tp == 1:
            return F.embedding(ids, self.weight)
        mask = (ids < self.vocab_start) | (ids >= self.vocab_end)
        local = (ids - self.vocab_start).masked_fill(mask, 0)
        out = F.embedding(local, self.weight)
        out = out.masked_fill(mask.unsqueeze(-1), 0.0)
        return reduce_from_tensor_parallel_region(out, self.group)


class _VocabParallelCrossEntropy(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, group, vocab_start, label_smoothing, ignore_index):
        # logits [N, V_local] (any float dtype; math in fp32)
        x = logits.float()
        lmax = x.max(dim=-1).values
        if _ws(group) > 1:
            dist.all_reduce(lmax, op=dist.ReduceOp.MAX, group=group)
        x = x - lmax.unsqueeze(-1)
        v_local = x.shape[-1]
        valid = target != ignore_index
        tloc = target - vocab_start
        in_range = (tloc >= 0) & (tloc < v_local) & valid
        tidx = tloc.clamp(0, v_local - 1)
        tlogit = x.gather(-1, tidx.unsqueeze(-1)).squeeze(-1) * in_range
        ex = x.exp()
        sumexp = ex.sum(-1)
        sum_x = x.sum(-1) if label_smoothing > 0 else None
        stats = torch.stack([tlogit, sumexp] + ([sum_x] if sum_x is not None else []), 0)
        if _ws(group) > 1:
            dist.all_reduce(stats, group=group)
        tlogit, sumexp = stats[0], stats[1]
        logz = sumexp.log()
        loss = logz - tlogit
        vocab = v_local * _ws(group)
        if label_smoothing > 0:
            mean_logp = stats[2] / vocab - logz
            loss = (1 - label_smoothing) * loss - label_smoothing * mean_logp
        loss = loss * valid
        softmax = ex / sumexp.unsqueeze(-1)
        ctx.save_for_backward(softmax, tidx, in_range, valid)
        ctx.ls, ctx.vocab = label_smoothing, vocab
        ctx.dtype = logits.dtype
        return loss

    @staticmethod
    def backward(ctx, g):
        softmax, tidx, in_range, valid = ctx.saved_tensors
        grad = softmax
        ls = ctx.ls
        if ls > 0:
            grad = grad - ls / ctx.vocab
        grad.scatter_add_(-1, tidx.unsqueeze(-1), -(1 - ls) * in_range.float().unsqueeze(-1))
        grad = grad * (g * valid).unsqueeze(-1)
        return grad.to(ctx.dtype), None, None, None, None, None


def vocab_parallel_cross_entropy(logits: torch.Tensor, target: torch.Tensor, group=None, vocab_start: int = -1,
                                 label_smoothing: float = 0.0, ignore_index: int = -100) -> torch.Tensor:
    """Per-token loss from vocab-sharded logits [..., V/tp]."""
    group = group if group is not None else _default_tp_group()
    if vocab_start < 0:
        vocab_start = _rk(group) * logits.shape[-1]
    shp = target.shape
    loss = _VocabParallelCrossEntropy.apply(logits.reshape(-1, logits.shape[-1]), target.reshape(-1), group,
                                            vocab_start, label_smoothing, ignore_index)
    return loss.view(shp)


def allreduce_sequence_parallel_grads(module: nn.Module, group=None):
    """Grads of parameters replicated across TP ranks but fed by
    sequence-sharded activations (norm weights, row-parallel biases) are
    partial: all-reduce them across the TP group (call before the optimizer)."""
    group = group if group is not None else _default_tp_group()
    if _ws(group) == 1:
        return
    grads = [p.grad for p in module.parameters() if getattr(p, "sequence_parallel", False) and p.grad is not None]
    if not grads:
        return
    flat = torch.cat([g.reshape(-1) for g in grads])
    dist.all_reduce(flat, group=group)
    o = 0
    for g in grads:
        g.copy_(flat[o:o + g.numel()].view_as(g))
        o += g.numel()


def mark_sequence_parallel(module: nn.Module):
    """Tag norm parameters inside a sequence-parallel region."""
    for m in module.modules():
        if isinstance(m, (nn.LayerNorm,)) or type(m).__name__ in ("LayerNorm", "RMSNorm", "AtorchLayerNorm"):
            for p in m.parameters(recurse=False):
                p.sequence_parallel = True
