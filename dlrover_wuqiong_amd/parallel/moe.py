"""Mixture-of-Experts layer with expert parallelism (dropless, top-k).

Token path (per MoE layer):
  1. router logits -> top-k experts + renormalised weights (aux load-balance
     loss and router z-loss are recorded on the module);
  2. the T*k (token, expert) assignments are sorted by expert -- one gather
     builds a contiguous, expert-grouped activation buffer;
  3. expert parallel: the buffer is exchanged with ONE variable-split
     ``all_to_all_single`` over the EP group (RCCL; the per-expert counts go
     first in a tiny all_to_all; the split sizes are the layer's only host
     read) and regrouped by local expert in ONE permutation launch driven by
     the device counts (``csrc/kernels/moe_permute.hip``);
  4. the local experts run as grouped GEMMs over the contiguous groups
     (``grouped_mlp`` -> ``ops.grouped_gemm``: one MFMA launch per projection
     for all experts, group offsets on the device -- no host sync, no
     padding, no capacity drop);
  5. the inverse exchange + un-permute + weighted sum over k.

MI355X sizing: with 288 GB per GPU experts can stay resident at high EP
degrees; keep EP within a node (xGMI all-to-all is per-link bound: every
GPU talks to 7 peers over 7 links concurrently) and put DP across nodes.

Parity: ATorch ``atorch/modules/moe`` (``MOELayer``, ``TopkGate``,
``Experts``, ``_AllToAll``; grouped-GEMM experts) -- re-designed dropless.
"""

import math
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F


def _ws(group) -> int:
    return dist.get_world_size(group) if (dist.is_initialized() and group is not None) else 1


class _AllToAllV(torch.autograd.Function):
    """Variable-split all_to_all_single along dim 0 (autograd: inverse split)."""

    @staticmethod
    def forward(ctx, x, out_splits: List[int], in_splits: List[int], group):
        ctx.group, ctx.out_splits, ctx.in_splits = group, out_splits, in_splits
        out = x.new_empty((sum(out_splits),) + tuple(x.shape[1:]))
        dist.all_to_all_single(out, x.contiguous(), out_splits, in_splits, group=group)
        return out

    @staticmethod
    def backward(ctx, g):
        gin = g.new_empty((sum(ctx.in_splits),) + tuple(g.shape[1:]))
        dist.all_to_all_single(gin, g.contiguous(), ctx.in_splits, ctx.out_splits, group=ctx.group)
        return gin, None, None, None


def all_to_all_v(x, out_splits, in_splits, group):
    return _AllToAllV.apply(x, out_splits, in_splits, group)


def _regroup_index(counts: torch.Tensor, n: int) -> torch.Tensor:
    """dst[i] of every received row i (torch ops; the CPU path and the
    reference of ``csrc/kernels/moe_permute.hip``)."""
    ep, L = counts.shape
    flat = counts.reshape(-1)
    src_off = torch.cumsum(flat, 0) - flat                       # (s, e) source-major
    t = counts.t().reshape(-1)
    exp_off = (torch.cumsum(t, 0) - t).view(L, ep).t().reshape(-1)  # [s * L + e] expert-major
    seg = torch.repeat_interleave(torch.arange(ep * L, device=counts.device), flat, output_size=n)
    return exp_off[seg] + torch.arange(n, device=counts.device) - src_off[seg]


def _regroup(x: torch.Tensor, counts: torch.Tensor, direction: int) -> torch.Tensor:
    from ..ops import _hip

    n = x.shape[0]
    row_bytes = x[0].numel() * x.element_size() if n else 0
    if _hip.use_hip(x) and x.is_contiguous() and row_bytes % 16 == 0 and counts.numel() <= 1024:
        import ctypes

        out = torch.empty_like(x)
        c = counts.to(torch.int64).contiguous()
        _hip.check(_hip.lib().dw_moe_regroup(_hip.ptr(x), _hip.ptr(out), _hip.ptr(c), counts.shape[0],
                                             counts.shape[1], ctypes.c_longlong(n), row_bytes, direction,
                                             _hip.stream()), "moe_regroup")
        return out
    dst = _regroup_index(counts, n)
    if direction == 0:
        return torch.empty_like(x).index_copy_(0, dst, x)
    return x.index_select(0, dst)


class _Regroup(torch.autograd.Function):
    """(source rank, expert) -> (expert, source rank) row order and back; the
    backward is the opposite direction of the same permutation."""

    @staticmethod
    def forward(ctx, x, counts, direction: int):
        ctx.save_for_backward(counts)
        ctx.direction = direction
        return _regroup(x.contiguous(), counts, direction)

    @staticmethod
    def backward(ctx, g):
        (counts,) = ctx.saved_tensors
        return _regroup(g.contiguous(), counts, 1 - ctx.direction), None, None


def moe_regroup(x: torch.Tensor, counts: torch.Tensor, direction: int = 0) -> torch.Tensor:
    """``counts`` [ep, L] rows per (source rank, local expert), on the device.
    direction 0: received order -> expert-grouped; 1: back."""
    return _Regroup.apply(x, counts, direction)


class TopKGate(nn.Module):
    def __init__(self, hidden: int, num_experts: int, top_k: int = 2, z_loss_coef: float = 1e-3,
                 aux_loss_coef: float = 1e-2, norm_topk: bool = True, dtype=None, device=None):
        super().__init__()
        self.num_experts, self.top_k = num_experts, top_k
        self.z_loss_coef, self.aux_loss_coef = z_loss_coef, aux_loss_coef
        self.norm_topk = norm_topk
        self.wg = nn.Linear(hidden, num_experts, bias=False, dtype=dtype, device=device)

    def forward(self, x):
        logits = self.wg(x).float()
        probs = logits.softmax(-1)
        w, idx = probs.topk(self.top_k, dim=-1)
        if self.norm_topk:
            w = w / w.sum(-1, keepdim=True)
        # Switch/GShard load balance: E * sum_e f_e * p_e
        frac = torch.zeros(self.num_experts, device=x.device, dtype=torch.float32)
        frac.scatter_add_(0, idx.reshape(-1), torch.ones(idx.numel(), device=x.device))
        frac = frac / idx.numel()
        aux = self.num_experts * (frac * probs.mean(0)).sum() * self.aux_loss_coef
        z = torch.logsumexp(logits, -1).square().mean() * self.z_loss_coef
        return w, idx, aux + z


def grouped_mlp(x: torch.Tensor, counts, w1: torch.Tensor, w2: torch.Tensor,
                w3: Optional[torch.Tensor] = None, activation: str = "silu") -> torch.Tensor:
    """Expert FFN over contiguous groups: rows [off_e, off_e + counts[e]) go
    through expert e.  w1/w3 [E, F, H] (w3: SwiGLU gate), w2 [E, H, F].
    ``counts``: per-expert row counts (device tensor or host list).  On a GPU
    every projection is ONE grouped-GEMM launch over all experts with the
    offsets on the device (no host sync); on the CPU a per-expert loop."""
    from ..ops import _hip

    E = w1.shape[0]
    # Few large experts (Mixtral-style, >= 2048 rows each): hipBLASLt's tuned
    # per-expert GEMMs beat the grouped kernel 1.8x and the one host read of
    # the counts is noise next to ms-long GEMMs.  Many small experts
    # (fine-grained MoE): the grouped kernel wins 2.5-10x
    # (profiles/r2/grouped_gemm_bench.jsonl).
    few_large = E <= 16 and x.shape[0] >= 2048 * E
    if _hip.use_hip(x) and x.dtype == torch.bfloat16 and not few_large:
        from ..ops.grouped_gemm import grouped_linear, offsets_from_counts

        offs = offsets_from_counts(counts, x.device)
        h = grouped_linear(x, w1, offs)
        if w3 is not None:
            h = F.silu(h) * grouped_linear(x, w3, offs) if activation == "silu" else F.gelu(h) * grouped_linear(
                x, w3, offs)
        else:
            h = F.silu(h) if activation == "silu" else F.gelu(h)
        return grouped_linear(h, w2, offs)
    if torch.is_tensor(counts):
        counts = counts.tolist()
    outs = []
    off = 0
    act = F.silu if activation == "silu" else F.gelu
    for e, n in enumerate(counts):
        if n == 0:
            continue
        xe = x[off:off + n]
        h = F.linear(xe, w1[e])
        h = act(h) * F.linear(xe, w3[e]) if w3 is not None else act(h)
        outs.append(F.linear(h, w2[e]))
        off += n
    if not outs:
        # no rows for any local expert (EP: this rank received nothing): keep
        # x AND the weights in the graph, so the backward still runs the
        # inverse all-to-all every EP peer waits for
        return x.new_zeros((0, w2.shape[1])) + 0 * (x.sum() + w1.sum() + w2.sum() +
                                                    (w3.sum() if w3 is not None else 0))
    return torch.cat(outs, 0)


class Experts(nn.Module):
    def __init__(self, num_local_experts: int, hidden: int, ffn: int, swiglu: bool = True, dtype=None, device=None):
        super().__init__()
        self.num_local_experts = num_local_experts
        self.w1 = nn.Parameter(torch.empty(num_local_experts, ffn, hidden, dtype=dtype, device=device))
        self.w2 = nn.Parameter(torch.empty(num_local_experts, hidden, ffn, dtype=dtype, device=device))
        self.w3 = nn.Parameter(torch.empty(num_local_experts, ffn, hidden, dtype=dtype, device=device)) \
            if swiglu else None
        for p in (self.w1, self.w2, self.w3):
            if p is not None:
                nn.init.normal_(p, std=1.0 / math.sqrt(p.shape[-1]))
                p.expert_parallel = True  # grads reduced over the expert-data-parallel group only

    def forward(self, x, counts: List[int]):
        return grouped_mlp(x, counts, self.w1, self.w2, self.w3, "silu" if self.w3 is not None else "gelu")


def capacity_mask(idx: torch.Tensor, num_experts: int, capacity: int) -> torch.Tensor:
    """[T, k] keep-mask of top-k assignments under a per-expert capacity
    (GShard / Switch priority: every token's first choice before any second
    choice, earlier tokens first); computed on the device."""
    T, k = idx.shape
    pri = idx.t().reshape(-1)  # k-major: first choices first
    oh = F.one_hot(pri, num_experts)
    pos = (oh.cumsum(0) * oh).sum(-1) - 1  # position of each assignment in its expert's queue
    return (pos < capacity).view(k, T).t()


class MoELayer(nn.Module):
    """``num_experts`` global experts split evenly over ``ep_group``.

    ``capacity_factor`` > 0: GShard / Switch capacity -- each expert takes at
    most ceil(factor * T * k / E) assignments of a batch (T tokens on this
    rank), the rest are dropped (their weight is 0; with a residual around
    the layer the token passes through unchanged).  Dropped assignments go
    to a sentinel bucket past the last expert: never sent, never computed.
    Default 0: dropless."""

    def __init__(self, hidden: int, ffn: int, num_experts: int, top_k: int = 2, ep_group=None,
                 swiglu: bool = True, dtype=None, device=None, aux_loss_coef: float = 1e-2,
                 capacity_factor: float = 0.0, norm_topk: bool = True):
        super().__init__()
        self.ep_group = ep_group
        self.ep = _ws(ep_group)
        assert num_experts % self.ep == 0, f"{num_experts} experts not divisible by EP {self.ep}"
        self.num_experts, self.top_k = num_experts, top_k
        self.num_local = num_experts // self.ep
        self.capacity_factor = float(capacity_factor)
        self.gate = TopKGate(hidden, num_experts, top_k, aux_loss_coef=aux_loss_coef, norm_topk=norm_topk,
                             dtype=dtype, device=device)
        self.experts = Experts(self.num_local, hidden, ffn, swiglu, dtype=dtype, device=device)
        self.aux_loss = torch.zeros(())

    def forward(self, x):
        shape = x.shape
        x = x.reshape(-1, shape[-1])
        T, k, E = x.shape[0], self.top_k, self.num_experts
        w, idx, self.aux_loss = self.gate(x)
        keep = None
        if self.capacity_factor > 0:
            cap = max(1, math.ceil(self.capacity_factor * T * k / E))
            keep = capacity_mask(idx, E, cap)
            idx = torch.where(keep, idx, torch.full_like(idx, E))  # sentinel bucket E
            w = w * keep
        flat = idx.reshape(-1)
        order = torch.argsort(flat, stable=True)
        counts = torch.bincount(flat, minlength=E + (keep is not None))[:E]
        xs = x.index_select(0, order // k)
        if keep is not None:
            # the grouped GEMMs leave rows past the last group (the sentinel
            # bucket) unwritten in y and dx: mask them out both ways
            valid = (flat.index_select(0, order) < E).unsqueeze(-1)
            xs = torch.where(valid, xs, xs.new_zeros(()))
        if self.ep > 1:
            send_counts = counts.view(self.ep, self.num_local)  # [dst rank, local expert]
            recv_counts = torch.empty_like(send_counts)
            dist.all_to_all_single(recv_counts, send_counts.contiguous(), group=self.ep_group)
            # the ONE host read per layer: the all-to-all split sizes
            in_splits, out_splits = torch.stack([send_counts.sum(1), recv_counts.sum(1)]).tolist()
            xr = all_to_all_v(xs[:sum(in_splits)] if keep is not None else xs, out_splits, in_splits,
                              self.ep_group)
            # received rows are (src rank, expert)-ordered: one permutation
            # launch (device counts) groups them by local expert
            y = self.experts(moe_regroup(xr, recv_counts, 0), recv_counts.sum(0))
            y = all_to_all_v(moe_regroup(y, recv_counts, 1), in_splits, out_splits, self.ep_group)
        else:
            y = self.experts(xs, counts)  # device counts: no host sync on the GPU path
        if keep is not None:
            # dropped (sentinel) rows: never computed -- zero, whatever the buffer holds
            if y.shape[0] < xs.shape[0]:
                y = torch.cat([y, y.new_zeros(xs.shape[0] - y.shape[0], y.shape[-1])])
            y = torch.where(valid, y, y.new_zeros(()))
        # un-permute and combine the k expert outputs per token
        out = torch.zeros(T * k, y.shape[-1], dtype=y.dtype, device=y.device)
        out = out.index_copy(0, order, y)
        out = (out.view(T, k, -1) * w.to(y.dtype).unsqueeze(-1)).sum(1)
        return out.view(shape[:-1] + (out.shape[-1],))


class SwitchGate(TopKGate):
    """Switch Transformer router: top-1, the output scaled by the expert's
    raw gate probability (reference switch_gating.py; use with a
    ``MoELayer(top_k=1, capacity_factor=..., norm_topk=False)``)."""

    def __init__(self, hidden: int, num_experts: int, **kw):
        kw.setdefault("norm_topk", False)
        super().__init__(hidden, num_experts, top_k=1, **kw)


def replace_with_moe(model: nn.Module, layer_class, num_experts: int, top_k: int = 2, ep_group=None,
                     capacity_factor: float = 0.0, noise_std: float = 0.0) -> List[str]:
    """Sparse upcycling (reference modules/moe/inject.py ``replace_with_moe``):
    every ``layer_class`` SwiGLU FFN of ``model`` becomes a ``MoELayer`` whose
    experts start as copies of the dense weights (optionally + Gaussian
    noise) and whose router starts small and random (balanced routing; the
    renormalised top-k weights sum to 1 over identical experts) -- without
    noise the MoE model initially computes exactly the dense model's
    function.  Supported FFNs:
    this framework's ``LlamaMLP`` (fused ``gate_up_proj``) and HF-style
    ``gate_proj`` / ``up_proj`` / ``down_proj``.  With ``ep_group`` this
    rank keeps its slice of the experts.  Returns the replaced names."""
    done = []
    for name, mod in list(model.named_modules()):
        for cname, child in list(mod.named_children()):
            if not isinstance(child, layer_class):
                continue
            if hasattr(child, "gate_up_proj"):
                gu = child.gate_up_proj.weight
                F_ = gu.shape[0] // 2
                gate_w, up_w = gu[:F_], gu[F_:]
            elif hasattr(child, "gate_proj") and hasattr(child, "up_proj"):
                gate_w, up_w = child.gate_proj.weight, child.up_proj.weight
            else:
                raise TypeError(f"{type(child).__name__}: not a SwiGLU FFN (gate/up/down projections)")
            down_w = child.down_proj.weight
            H, F_ = down_w.shape
            moe = MoELayer(H, F_, num_experts, top_k, ep_group=ep_group, capacity_factor=capacity_factor,
                           dtype=down_w.dtype, device=down_w.device)
            lo = moe.num_local * (dist.get_rank(ep_group) if moe.ep > 1 else 0)
            with torch.no_grad():
                # a zero router ties every expert and top-k then sends all
                # tokens to the same k experts (one EP rank gets everything)
                gen = torch.Generator(device="cpu").manual_seed(1234)
                moe.gate.wg.weight.copy_(torch.randn(moe.gate.wg.weight.shape, generator=gen) * (0.1 / H ** 0.5))
                for e in range(moe.num_local):
                    for dst, src in ((moe.experts.w1, gate_w), (moe.experts.w3, up_w), (moe.experts.w2, down_w)):
                        dst[e].copy_(src)
                        if noise_std > 0:
                            g = torch.Generator(device="cpu").manual_seed(lo + e)
                            dst[e].add_(torch.randn(dst[e].shape, generator=g).to(dst) * noise_std)
            setattr(mod, cname, moe)
            done.append(f"{name}.{cname}" if name else cname)
    return done


def moe_aux_loss(model: nn.Module) -> torch.Tensor:
    losses = [m.aux_loss for m in model.modules() if isinstance(m, MoELayer)]
    return sum(losses) if losses else torch.zeros(())
