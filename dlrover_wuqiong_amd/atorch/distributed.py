"""ATorch-style distributed context: init + named N-D parallel groups.

``create_parallel_group(([("tensor", 4), ("pipeline", 2), ("data", 2)], None))``
slices the ranks with the FIRST dimension innermost (consecutive ranks), so
"tensor" groups are {0..3}, {4..7} ... -- on an MI355X node the innermost
group stays on the node's fully connected xGMI mesh.  Groups use the default
backend (RCCL on GPU); ``seq_all_to_all`` is the Ulysses sequence-parallel
exchange.

Parity: reference ``atorch/distributed/distributed.py`` (``init_distributed``
:664, ``create_parallel_group`` :323, ``parallel_group/rank/group_size``
:85-125, ``create_sequence_parallel_group`` :435, ``seq_all_to_all`` :474-502,
``destroy_parallel_group`` :414).  Coworker / pippy-RPC plumbing of the
reference is not carried over (pipeline stages here communicate with
point-to-point RCCL sends, see ``parallel/pipeline.py``).
"""

import os
from datetime import timedelta
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist


class _DistributedContext:
    INITIALIZED = False
    PARALLEL_CONFIG = None
    PARALLEL_CONFIGS: Dict[str, object] = {}  # per group-name prefix (ParallelGroupContextManager)
    PG_NAME_PREFIX = ""
    PARALLEL_GROUP: Dict[str, object] = {}
    PARALLEL_GROUPS_AND_RANKS: Dict[str, List[Tuple[object, List[int]]]] = {}
    PARALLEL_RANK: Dict[str, int] = {}
    PARALLEL_GROUP_SIZE: Dict[str, int] = {}
    PARALLEL_INSTANCE_NUM = 1
    PARALLEL_INSTANCE_INDEX = 0
    SEQUENCE_PARALLEL_GROUP = None
    SEQUENCE_PARALLEL_SIZE = 1


def local_rank() -> int:
    return int(os.getenv("LOCAL_RANK", "0"))


def rank() -> int:
    return dist.get_rank() if dist.is_initialized() else 0


def world_size() -> int:
    return dist.get_world_size() if dist.is_initialized() else 1


def is_distributed() -> bool:
    return dist.is_initialized()


def backend() -> Optional[str]:
    return dist.get_backend() if dist.is_initialized() else None


def nproc_per_node() -> int:
    return int(os.getenv("LOCAL_WORLD_SIZE", "1"))


def node_size() -> int:
    return max(1, world_size() // max(1, nproc_per_node()))


def init_distributed(backend: str = "nccl", set_cuda_device_using_local_rank: bool = True,
                     timeout: Optional[timedelta] = None, **kwargs) -> bool:
    """``backend="nccl"`` is RCCL on ROCm; falls back to gloo without a GPU."""
    if dist.is_initialized():
        _DistributedContext.INITIALIZED = True
        return True
    if backend == "nccl" and not torch.cuda.is_available():
        backend = "gloo"
    dev = None
    if torch.cuda.is_available() and set_cuda_device_using_local_rank:
        dev = torch.device("cuda", local_rank())
        torch.cuda.set_device(dev)
    kw = {"timeout": timeout} if timeout else {}
    if backend == "nccl" and dev is not None:
        kw["device_id"] = dev
    dist.init_process_group(backend, **kw)
    _DistributedContext.INITIALIZED = True
    return True


def reset_distributed():
    destroy_parallel_group()
    if dist.is_initialized():
        dist.destroy_process_group()
    _DistributedContext.INITIALIZED = False


def get_pg_ranks(slicing_dim: Sequence[Tuple[str, int]], rank_order: List[int]) -> List[Dict[str, List[List[int]]]]:
    """Per parallel instance: {name: [ranks of every group of that dim]}."""
    total = int(np.prod([s for _, s in slicing_dim]))
    instances = []
    for inst in range(len(rank_order) // total):
        order = rank_order[inst * total:(inst + 1) * total]
        shape = [s for _, s in slicing_dim][::-1]  # outermost first
        grid = np.array(order).reshape(shape)
        d: Dict[str, List[List[int]]] = {}
        nd = len(slicing_dim)
        for i, (name, _size) in enumerate(slicing_dim):
            axis = nd - 1 - i
            moved = np.moveaxis(grid, axis, -1).reshape(-1, grid.shape[axis])
            d[name] = [list(map(int, row)) for row in moved]
        instances.append(d)
    return instances


def create_parallel_group(parallel_config, timeout: Optional[timedelta] = None):
    """``parallel_config = ([(name, size), ...], rank_order or None[, multi_instance])``."""
    assert dist.is_initialized(), "call init_distributed first"
    slicing_dim = list(parallel_config[0])
    rank_order = parallel_config[1]
    multi = parallel_config[2] if len(parallel_config) > 2 else False
    total = int(np.prod([s for _, s in slicing_dim]))
    if not multi and total != world_size():
        raise ValueError(f"product of parallel sizes ({total}) != world size ({world_size()}): {parallel_config}")
    rank_order = list(range(world_size())) if rank_order is None else list(rank_order)
    pre = _DistributedContext.PG_NAME_PREFIX
    _DistributedContext.PARALLEL_CONFIGS[pre] = (slicing_dim, rank_order, multi)
    if not pre:
        _DistributedContext.PARALLEL_CONFIG = (slicing_dim, rank_order, multi)
    _DistributedContext.PARALLEL_INSTANCE_NUM = world_size() // total
    _DistributedContext.PARALLEL_INSTANCE_INDEX = rank() // total if rank() < world_size() // total * total else None
    all_pg = get_pg_ranks(slicing_dim, rank_order)
    for dim_name, size in slicing_dim:
        name = pre + dim_name
        if len(slicing_dim) == 1 and total == world_size():
            _DistributedContext.PARALLEL_GROUP[name] = dist.group.WORLD
            _DistributedContext.PARALLEL_RANK[name] = rank()
            _DistributedContext.PARALLEL_GROUP_SIZE[name] = size
            _DistributedContext.PARALLEL_GROUPS_AND_RANKS[name] = [(dist.group.WORLD, list(range(world_size())))]
            continue
        groups = []
        for inst in all_pg:
            for ranks in inst[dim_name]:
                g = dist.new_group(ranks, timeout=timeout) if timeout else dist.new_group(ranks)
                groups.append((g, ranks))
                if rank() in ranks:
                    _DistributedContext.PARALLEL_GROUP[name] = g
                    _DistributedContext.PARALLEL_RANK[name] = ranks.index(rank())
        _DistributedContext.PARALLEL_GROUPS_AND_RANKS[name] = groups
        _DistributedContext.PARALLEL_GROUP_SIZE[name] = size


def destroy_parallel_group():
    _DistributedContext.PARALLEL_CONFIG = None
    _DistributedContext.PARALLEL_CONFIGS = {}
    _DistributedContext.PARALLEL_GROUP = {}
    _DistributedContext.PARALLEL_GROUPS_AND_RANKS = {}
    _DistributedContext.PARALLEL_RANK = {}
    _DistributedContext.PARALLEL_GROUP_SIZE = {}
    destroy_sequence_parallel_group()


class ParallelGroupContextManager:
    """Named parallel groups per model (ATorch ``ParallelGroupContextManager``,
    reference distributed/distributed.py:48): inside ``with
    ParallelGroupContextManager("actor"):`` every group this module creates or
    looks up is namespaced ``actor`` + name, so e.g. an RLHF actor (TP x DP)
    and critic (pure DP) keep independent parallel layouts in one job."""

    def __init__(self, name: str = ""):
        self.name = name
        self.old = ""

    def __enter__(self):
        self.old = _DistributedContext.PG_NAME_PREFIX
        _DistributedContext.PG_NAME_PREFIX = self.name
        return self

    def __exit__(self, *exc):
        _DistributedContext.PG_NAME_PREFIX = self.old
        return False


def _pn(name: str) -> str:
    return _DistributedContext.PG_NAME_PREFIX + name


def parallel_config():
    return _DistributedContext.PARALLEL_CONFIGS.get(_DistributedContext.PG_NAME_PREFIX)


def parallel_groups_and_ranks_all(name: str):
    """[(group, ranks)] of every group of parallel dimension ``name``."""
    return _DistributedContext.PARALLEL_GROUPS_AND_RANKS.get(_pn(name), [])


def parallel_group(name: str):
    return _DistributedContext.PARALLEL_GROUP.get(_pn(name))


def parallel_group_and_ranks(name: str):
    if _pn(name) not in _DistributedContext.PARALLEL_GROUP:
        return None, None
    for g, ranks in _DistributedContext.PARALLEL_GROUPS_AND_RANKS.get(_pn(name), []):
        if rank() in ranks:
            return g, ranks
    return None, None


def parallel_rank(name: str) -> Optional[int]:
    return _DistributedContext.PARALLEL_RANK.get(_pn(name))


def parallel_group_size(name: str) -> Optional[int]:
    return _DistributedContext.PARALLEL_GROUP_SIZE.get(_pn(name))


def parallel_instance_num() -> int:
    return _DistributedContext.PARALLEL_INSTANCE_NUM


def parallel_instance_index():
    return _DistributedContext.PARALLEL_INSTANCE_INDEX


# ------------------------------------------------------ sequence parallel
def create_sequence_parallel_group(sp_size: int):
    """Consecutive ranks form Ulysses groups of ``sp_size`` (intra-node)."""
    ws = world_size()
    assert ws % sp_size == 0, f"world {ws} not divisible by sp {sp_size}"
    for start in range(0, ws, sp_size):
        ranks = list(range(start, start + sp_size))
        g = dist.new_group(ranks)
        if rank() in ranks:
            _DistributedContext.SEQUENCE_PARALLEL_GROUP = g
    _DistributedContext.SEQUENCE_PARALLEL_SIZE = sp_size


def destroy_sequence_parallel_group():
    _DistributedContext.SEQUENCE_PARALLEL_GROUP = None
    _DistributedContext.SEQUENCE_PARALLEL_SIZE = 1


def get_sequence_parallel_group():
    return _DistributedContext.SEQUENCE_PARALLEL_GROUP


def get_sequence_parallel_size() -> int:
    return _DistributedContext.SEQUENCE_PARALLEL_SIZE


def get_sequence_parallel_rank() -> int:
    g = _DistributedContext.SEQUENCE_PARALLEL_GROUP
    return dist.get_rank(g) if g is not None else 0


def _all_to_all(x: torch.Tensor, scatter_idx: int, gather_idx: int, group, n: int) -> torch.Tensor:
    """Split ``x`` along ``scatter_idx`` into n parts, exchange, concatenate
    the received parts along ``gather_idx`` (one all_to_all_single)."""
    if n == 1:
        return x
    parts = [t.contiguous() for t in torch.tensor_split(x, n, dim=scatter_idx)]
    inp = torch.stack(parts, 0).contiguous()
    out = torch.empty_like(inp)
    dist.all_to_all_single(out, inp, group=group)
    return torch.cat(list(out.unbind(0)), dim=gather_idx).contiguous()


class _SeqAllToAll(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, scatter_idx, gather_idx, group, n):
        ctx.args = (scatter_idx, gather_idx, group, n)
        return _all_to_all(x, scatter_idx, gather_idx, group, n)

    @staticmethod
    def backward(ctx, g):
        scatter_idx, gather_idx, group, n = ctx.args
        return _all_to_all(g, gather_idx, scatter_idx, group, n), None, None, None, None


def seq_all_to_all(x: torch.Tensor, scatter_idx: int, gather_idx: int, group=None,
                   group_size: Optional[int] = None) -> torch.Tensor:
    group = group if group is not None else get_sequence_parallel_group()
    n = group_size or (dist.get_world_size(group) if group is not None else 1)
    return _SeqAllToAll.apply(x, scatter_idx, gather_idx, group, n)
