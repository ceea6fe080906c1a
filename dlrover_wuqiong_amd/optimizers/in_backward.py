"""Optimizer step inside the FSDP2 backward.

Under FSDP2 every ``fully_shard`` unit reduce-scatters its gradients as soon
as its part of the backward is done (``FSDPParamGroup.post_backward``).  The
optimizer normally runs after the WHOLE backward: on a Llama-3-8B step the
multi-tensor AdamW (HBM-bound, ~30 B per parameter) is ~38 ms of serial time
after ~210 ms of backward (``profiles/r5/llama3_8b_fsdp_half_noac_kernels.md``).

Here each unit's update is launched from its post-backward, on a side HIP
stream that waits for the unit's reduce-scatter (``_post_reduce_event``), so
the update of layer L overlaps the backward GEMMs of layers L-1 ... 0.  It is
the same multi-tensor kernel (``csrc/kernels/optim_multi.hip``) over the
unit's sharded parameters, same math and state layout as the plain step:
results are bit-identical (``tests/test_optim_in_backward_gpu.py``).
``optimizer.step()`` (its hooks run as usual) then only orders the compute
stream after the side stream and updates parameters no unit covered (none
with a wrapped model).

Conditions (checked at install; otherwise the plain step runs):
* a :class:`~.multi_tensor._MultiTensorOptimizer` without global-norm
  clipping (``max_grad_norm == 0``): a clipped update needs every gradient
  before the first parameter moves.  Clipping outside the optimizer
  (``clip_grad_norm_`` between backward and step) is not possible either;
* gradient accumulation is honoured: micro-steps that do not reduce
  (``set_requires_gradient_sync(False)``) launch nothing.

Parity: ATorch ADP ``inject_optimizer`` (the per-module optimizer step
queued when the module's gradient reduce-scatter finishes,
``atorch/atorch/data_parallel/adp.py:26-36,108-159``) and
``register_overlap_optim`` (``atorch/atorch/optimizers/adam_offload.py:51``).
Enabled by ``auto_accelerate`` (``("fsdp"|"zero2", {"optim_in_backward": True})``).
"""

from typing import Dict, List, Optional, Tuple

import torch

from ..common.log import logger


def _fsdp_param_groups(model) -> List[Tuple[object, list]]:
    """(FSDPParamGroup, its sharded parameters) of every FSDP2 unit."""
    try:
        from torch.distributed.fsdp import FSDPModule
    except ImportError:  # pragma: no cover
        return []
    out = []
    for m in model.modules():
        if not isinstance(m, FSDPModule):
            continue
        pg = m._get_fsdp_state()._fsdp_param_group
        if pg is not None:
            out.append((pg, [fp.sharded_param for fp in pg.fsdp_params]))
    return out


class OptimizerInBackward:
    def __init__(self, model, optimizer, stream: Optional[torch.cuda.Stream] = None):
        from .multi_tensor import _MultiTensorOptimizer

        if not isinstance(optimizer, _MultiTensorOptimizer):
            raise TypeError(f"optimizer in backward needs a multi-tensor fused optimizer, got {type(optimizer)}")
        if optimizer.max_grad_norm > 0:
            raise ValueError("optimizer in backward: global-norm clipping needs every gradient first")
        self.opt = optimizer
        self.units = _fsdp_param_groups(model)
        if not self.units:
            raise ValueError("optimizer in backward: the model has no FSDP2 units")
        gi_of: Dict[int, int] = {id(p): gi for gi, g in enumerate(optimizer.param_groups) for p in g["params"]}
        self._unit_params = []
        for pg, params in self.units:
            self._unit_params.append([(gi_of[id(p)], p) for p in params if id(p) in gi_of])
        covered = {id(p) for ps in self._unit_params for _gi, p in ps}
        self._rest = [(gi, p) for gi, g in enumerate(optimizer.param_groups) for p in g["params"]
                      if id(p) not in covered]
        self.stream = stream
        # workgroups of each per-unit update (0: the plain step's grid).
        # Capping it measured slower (256: 312 ms, 64: 331 ms per Llama-3-8B
        # step, high-priority stream): kept for A/B
        import os

        self.max_blocks = int(os.environ.get("DWAMD_IN_BACKWARD_BLOCKS", "0"))
        self._started = False  # this backward launched updates (the step counter was advanced)
        self._done: set = set()
        self.enabled = True
        self.units_launched = 0
        for idx, (pg, _params) in enumerate(self.units):
            self._patch(pg, idx)
        # optimizer.step() (with every torch.optim hook) asks us first
        optimizer._in_backward = self

    def _patch(self, pg, idx: int):
        orig = pg.post_backward

        def post_backward(*a, **k):
            out = orig(*a, **k)
            try:
                self._after_unit(pg, idx)
            except Exception as e:  # never break the backward: the plain step will run
                logger.warning(f"optimizer in backward disabled: {e}")
                self.enabled = False
            return out

        pg.post_backward = post_backward

    def _side(self, device) -> torch.cuda.Stream:
        if self.stream is None:
            # normal priority: a high-priority stream let each unit's update
            # pre-empt the backward GEMMs (Llama-3-8B step 242 -> 283 ms;
            # profiles/r6/llama3_8b_fsdp_in_backward_ab.jsonl)
            self.stream = torch.cuda.Stream(device=device)
        return self.stream

    def _after_unit(self, pg, idx: int):
        if not self.enabled or not getattr(pg, "reduce_grads", True) or idx in self._done:
            return
        live = [(gi, p) for gi, p in self._unit_params[idx] if p.grad is not None]
        if not live:
            return
        from .multi_tensor import _local

        g0 = _local(live[0][1].grad)
        if not g0.is_cuda:
            return  # CPU (gloo) rehearsal: the plain step runs
        cur = torch.cuda.current_stream(g0.device)
        if not self._started:
            if self._done:
                self._done.clear()
            # the first write of this step's update: what a plain step's
            # pre-hooks order it after -- a pending overlapped / ring flash
            # checkpoint snapshot still reading parameters and state, and a
            # restart's deferred state restore still landing
            from ..flash_checkpoint import deferred_restore
            from ..flash_checkpoint.copier import fence_all

            fence_all()
            deferred_restore.wait_all(cur, g0.device)
            self.opt._step_t += 1  # once per optimizer step; every unit's update uses this count
            self._started = True
        side = self._side(g0.device)
        ev = getattr(pg, "_post_reduce_event", None)
        if ev is not None:
            side.wait_event(ev)  # this unit's reduce-scattered gradients
        side.wait_stream(cur)  # (and everything the backward queued so far for it)
        with torch.cuda.stream(side):
            self.opt._cuda_step(live, slot=("unit", idx), max_blocks=self.max_blocks)
        for _gi, p in live:
            _local(p.grad).record_stream(side)  # freed by zero_grad on the compute stream
        self._done.add(idx)
        self.units_launched += 1

    def owns_step(self) -> bool:
        """This backward already launched the update (``step()`` finishes it)."""
        return self._started

    def finish(self):
        """Called by ``optimizer.step()`` (after its pre-hooks): order the
        compute stream after the side stream and update what no unit
        covered, with the step count already advanced."""
        self._started = False
        missed = []
        for idx, ps in enumerate(self._unit_params):
            if idx not in self._done:
                missed.extend((gi, p) for gi, p in ps if p.grad is not None)
        self._done.clear()
        missed.extend((gi, p) for gi, p in self._rest if p.grad is not None)
        if self.stream is not None:
            torch.cuda.current_stream(self.stream.device).wait_stream(self.stream)
        if missed:
            self.opt._cuda_step(missed, slot="rest")

    def remove(self):
        for pg, _params in self.units:
            pg.__dict__.pop("post_backward", None)
        self.opt._in_backward = None


def install(model, optimizer) -> Optional[OptimizerInBackward]:
    """Attach the per-unit update to ``model``'s FSDP2 units (None, with a
    log line, when the conditions above do not hold)."""
    try:
        return OptimizerInBackward(model, optimizer)
    except (TypeError, ValueError) as e:
        logger.warning(f"optimizer in backward not installed: {e}")
        return None
