"""Data parallelism for models with expert-parallel MoE layers (reference:
atorch/modules/moe/ddp.py ``MoEMixtureDistributedDataParallel``).

Expert parameters (``p.expert_parallel``, set by ``parallel.moe.Experts``)
hold DIFFERENT experts on the ranks of an EP group, so they must never be
averaged across it -- plain DDP over the world would silently mix the
gradients of different experts.  Here:

  * dense parameters: torch DDP over the data-parallel group (bucketed RCCL
    all-reduce overlapped with the backward), expert parameters excluded
    from it;
  * expert parameters: one async all-reduce per parameter over the
    EXPERT-data-parallel group (the ranks holding the same experts: one per
    EP group), launched from a post-accumulate-grad hook as soon as the
    parameter's gradient is final -- overlapped with the rest of the
    backward -- and waited in ``finish_gradient_synchronization()`` (called
    by the optimizer-step hook this wrapper installs, or by hand).

Scaling: every rank's loss is a mean over its own batch and the objective is
their mean over the ``world`` data ranks; a rank's expert gradient already
sums the contributions of all tokens routed to it across its EP group (the
all-to-all backward), so the expert all-reduce SUM is divided by the number
of data-parallel ranks in the world (not by the expert-DP group size) --
dense and expert gradients then both equal d(mean loss)/d(param).

MI355X layout: EP inside a node's xGMI mesh, expert-DP across nodes; the
expert all-reduces are few and large (one per expert weight tensor).
"""

import contextlib
from typing import List, Optional

import torch
import torch.distributed as dist
import torch.nn as nn


def expert_data_parallel_group(ep_size: int, ranks: Optional[List[int]] = None):
    """The group of ranks holding the same experts, for EP groups made of
    consecutive ranks ``[i*ep, (i+1)*ep)``: ranks with equal ``r % ep``.
    Every rank must call this (it creates all ``ep_size`` groups)."""
    ranks = list(ranks if ranks is not None else range(dist.get_world_size()))
    me = dist.get_rank()
    mine = None
    for i in range(ep_size):
        members = [r for j, r in enumerate(ranks) if j % ep_size == i]
        g = dist.new_group(members)
        if me in members:
            mine = g
    return mine


class MoEDistributedDataParallel(nn.Module):
    def __init__(self, module: nn.Module, expert_dp_group=None, process_group=None, data_parallel_size: int = 0,
                 **ddp_kwargs):
        super().__init__()
        self.expert_params = [(n, p) for n, p in module.named_parameters()
                              if getattr(p, "expert_parallel", False) and p.requires_grad]
        names = [n for n, _ in self.expert_params]
        nn.parallel.DistributedDataParallel._set_params_and_buffers_to_ignore_for_model(module, names)
        dense = [p for n, p in module.named_parameters() if p.requires_grad and n not in set(names)]
        self.dense_ddp = bool(dense)
        if self.dense_ddp:
            self.module = nn.parallel.DistributedDataParallel(module, process_group=process_group, **ddp_kwargs)
        else:
            self.module = module
        self.expert_dp_group = expert_dp_group
        self.dp_size = data_parallel_size or dist.get_world_size(process_group)
        self._pending = []
        self._sync = True
        for _n, p in self.expert_params:
            p.register_post_accumulate_grad_hook(self._reduce_expert)

    @contextlib.contextmanager
    def no_sync(self):
        """Gradient accumulation: no dense or expert all-reduce inside (as
        DDP.no_sync); the backward after the block reduces the sums."""
        prev, self._sync = self._sync, False
        try:
            if self.dense_ddp:
                with self.module.no_sync():
                    yield
            else:
                yield
        finally:
            self._sync = prev

    def _reduce_expert(self, p: torch.Tensor):
        if not self._sync:
            return
        # SUM over the replicas of these experts, scaled by 1 / (data ranks)
        p.grad.div_(self.dp_size)
        work = dist.all_reduce(p.grad, group=self.expert_dp_group, async_op=True)
        self._pending.append(work)

    def finish_gradient_synchronization(self):
        for w in self._pending:
            w.wait()
        self._pending.clear()

    def attach_optimizer(self, optimizer):
        """Wait for the expert all-reduces before every ``optimizer.step()``."""
        optimizer.register_step_pre_hook(lambda *_a, **_k: self.finish_gradient_synchronization())
        return optimizer

    def forward(self, *args, **kwargs):
        return self.module(*args, **kwargs)


MoEMixtureDistributedDataParallel = MoEDistributedDataParallel  # reference name

__all__ = ["MoEDistributedDataParallel", "MoEMixtureDistributedDataParallel", "expert_data_parallel_group"]
