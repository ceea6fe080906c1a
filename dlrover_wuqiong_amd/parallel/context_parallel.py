"""Context parallelism: attention over a sequence sharded across ranks, with
load-balanced (zig-zag) causal sharding and an all-gather of K/V.

Sharding.  The global sequence of S tokens is cut into 2N chunks of
c = S / 2N; rank r holds chunks r and 2N-1-r (``zigzag_split``).  Under a
causal mask chunk a attends to the (a+1)c-token prefix, so every rank's two
chunks see (r+1)c + (2N-r)c = (2N+1)c keys: equal attention work on every
rank, which a contiguous split (rank r sees (r+1)/N of the keys) does not
give.

Attention.  K and V (GQA: Hkv/H of Q's size -- 1/8 on Llama-3) are
all-gathered once per layer in ONE collective over the CP group, reordered
into global sequence order, and each local query chunk runs the
variable-length MFMA flash kernel against its key prefix with bottom-right
causal alignment (``flash_attn_varlen_func``: q length c, k length (a+1)c).
The backward of the gather is a reduce-scatter of dK/dV.  Compared with a
ring (N-1 point-to-point K/V hops interleaved with N partial attentions and
an LSE merge), the all-gather keeps one large collective per layer -- what
RCCL's xGMI rings move at full per-link bandwidth -- and one kernel launch
per chunk; the gathered K/V of a 128k-token Llama-3-8B layer is 256 MB,
small next to 288 GB of HBM.

RoPE uses global positions (``zigzag_positions``).  Parameters are
replicated across the CP group: their gradients are averaged over it like a
data-parallel group (fold CP into the DP group of DDP/FSDP).

Parity: ATorch sequence-sharded attention
``atorch/modules/distributed_transformer/distributed_attention.py``
(DistributedSelfAttention: local queries against the whole sequence's keys,
AllGatherQMicro / ReduceScatterContext in ``commu_utils.py``).
"""

from typing import Optional

import torch
import torch.distributed as dist


def _ws(group) -> int:
    return dist.get_world_size(group) if (group is not None and dist.is_initialized()) else 1


def _rank(group) -> int:
    return dist.get_rank(group) if (group is not None and dist.is_initialized()) else 0


def zigzag_chunks(rank: int, world: int):
    return rank, 2 * world - 1 - rank


def zigzag_split(x: torch.Tensor, group, dim: int = 1) -> torch.Tensor:
    """This rank's two zig-zag chunks of a full-sequence tensor."""
    n = _ws(group)
    if n == 1:
        return x
    a, b = zigzag_chunks(_rank(group), n)
    ch = x.chunk(2 * n, dim=dim)
    return torch.cat([ch[a], ch[b]], dim=dim)


def zigzag_positions(seq_local: int, group, device=None) -> torch.Tensor:
    """Global token positions of this rank's local (zig-zag) tokens."""
    n = _ws(group)
    if n == 1:
        return torch.arange(seq_local, device=device)
    c = seq_local // 2
    a, b = zigzag_chunks(_rank(group), n)
    return torch.cat([torch.arange(a * c, (a + 1) * c, device=device), torch.arange(b * c, (b + 1) * c, device=device)])


def _global_order(n: int):
    """Index i of the gathered [N, 2, ...] chunk list that holds global chunk g."""
    src = [0] * (2 * n)
    for j in range(n):
        a, b = zigzag_chunks(j, n)
        src[a], src[b] = 2 * j, 2 * j + 1
    return src


class _GatherKV(torch.autograd.Function):
    """[2, B, S_local, Hkv, D] (k, v stacked) -> [N, 2, B, S_local, Hkv, D];
    backward: reduce-scatter (sum) of the gathered gradient."""

    @staticmethod
    def forward(ctx, kv, group):
        ctx.group = group
        n = _ws(group)
        out = torch.empty((n,) + tuple(kv.shape), dtype=kv.dtype, device=kv.device)
        kv = kv.contiguous()
        if dist.get_backend(group) == "gloo":
            dist.all_gather(list(out.unbind(0)), kv, group=group)
        else:
            dist.all_gather_into_tensor(out.view(-1), kv.view(-1), group=group)
        return out

    @staticmethod
    def backward(ctx, g):
        group = ctx.group
        g = g.contiguous()
        if dist.get_backend(group) == "gloo":  # gloo has no reduce-scatter
            dist.all_reduce(g, group=group)
            return g[_rank(group)].clone(), None
        out = torch.empty(g.shape[1:], dtype=g.dtype, device=g.device)
        dist.reduce_scatter_tensor(out.view(-1), g.view(-1), group=group)
        return out, None


def gather_kv_global(k: torch.Tensor, v: torch.Tensor, group):
    """All-gather this rank's zig-zag K/V shards ([B, S_local, Hkv, D]) and
    return the full-sequence K, V ([B, S, Hkv, D], global order)."""
    n = _ws(group)
    kv = _GatherKV.apply(torch.stack([k, v]), group)          # [N, 2, B, 2c, Hkv, D]
    N, _, B, S2, Hk, D = kv.shape
    c = S2 // 2
    chunks = kv.view(N, 2, B, 2, c, Hk, D).permute(0, 3, 1, 2, 4, 5, 6).reshape(2 * N, 2, B, c, Hk, D)
    full = chunks[_global_order(n)]                            # [2N, 2, B, c, Hkv, D]
    full = full.permute(1, 2, 0, 3, 4, 5).reshape(2, B, 2 * N * c, Hk, D)
    return full[0], full[1]


def context_parallel_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, group,
                               causal: bool = True, softmax_scale: Optional[float] = None) -> torch.Tensor:
    """q [B, S_local, H, D], k/v [B, S_local, Hkv, D]: this rank's zig-zag
    shard (S_local = 2c).  Returns this rank's attention output
    [B, S_local, H, D] over the WHOLE sequence."""
    from ..ops.attention import flash_attn_func, flash_attn_varlen_func

    n = _ws(group)
    if n == 1:
        return flash_attn_func(q, k, v, causal=causal, softmax_scale=softmax_scale)
    B, S2, H, D = q.shape
    assert S2 % 2 == 0, "context parallel needs an even local sequence (two zig-zag chunks)"
    c = S2 // 2
    kf, vf = gather_kv_global(k, v, group)
    S = kf.shape[1]
    Hk = kf.shape[2]
    outs = []
    for i, a in enumerate(zigzag_chunks(_rank(group), n)):
        L = (a + 1) * c if causal else S
        qa = q[:, i * c:(i + 1) * c].reshape(B * c, H, D)
        ka = kf[:, :L].reshape(B * L, Hk, D)
        va = vf[:, :L].reshape(B * L, Hk, D)
        cu_q = torch.arange(0, (B + 1) * c, c, dtype=torch.int32, device=q.device)
        cu_k = torch.arange(0, (B + 1) * L, L, dtype=torch.int32, device=q.device)
        o = flash_attn_varlen_func(qa, ka, va, cu_q, cu_k, c, L, softmax_scale=softmax_scale, causal=causal)
        outs.append(o.view(B, c, H, D))
    return torch.cat(outs, dim=1)
