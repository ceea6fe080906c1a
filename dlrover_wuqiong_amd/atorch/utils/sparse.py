"""All-reduce of sparse COO tensors (embedding gradients): every rank's
(indices, values) are all-gathered -- padded to the largest nnz, one
collective for the indices and one for the values -- summed and coalesced.

Parity: ATorch ``atorch/utils/sparse.py`` (all_reduce_sparse).
"""

import torch
import torch.distributed as dist


def all_reduce_sparse(sparse_tensor: torch.Tensor, group=None) -> torch.Tensor:
    t = sparse_tensor.coalesce()
    world = dist.get_world_size(group)
    idx, val = t.indices(), t.values()
    dev = val.device
    nnz = torch.tensor([idx.shape[1]], device=dev, dtype=torch.long)
    all_nnz = [torch.zeros_like(nnz) for _ in range(world)]
    dist.all_gather(all_nnz, nnz, group=group)
    counts = [int(n) for n in all_nnz]
    m = max(counts)
    pad = m - idx.shape[1]
    idx_p = torch.cat([idx, idx.new_zeros(idx.shape[0], pad)], dim=1) if pad else idx
    val_p = torch.cat([val, val.new_zeros((pad,) + tuple(val.shape[1:]))]) if pad else val
    idx_all = [torch.empty_like(idx_p) for _ in range(world)]
    val_all = [torch.empty_like(val_p) for _ in range(world)]
    dist.all_gather(idx_all, idx_p.contiguous(), group=group)
    dist.all_gather(val_all, val_p.contiguous(), group=group)
    indices = torch.cat([i[:, :c] for i, c in zip(idx_all, counts)], dim=1)
    values = torch.cat([v[:c] for v, c in zip(val_all, counts)])
    return torch.sparse_coo_tensor(indices, values, t.shape).coalesce()
