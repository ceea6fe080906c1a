"""Slice all-gather for the replicated-checkpoint restore, for every backend.

A replicated (DDP) checkpoint is split 1/L across the node's local ranks:
each rank copies only its slice host->device (or device->device from its HBM
tier) and the slices meet with one all-gather.  On MI355X the group is RCCL
over xGMI and the gather is ``all_gather_into_tensor`` on device memory.

A gloo world has no device collectives: the CPU rehearsal of the N>1 fault
path and ranks that share one GPU (``bench.py --rehearse-shared-device``)
run gloo.  For those the device slice is staged through pinned host memory
in bounded chunks (``all_gather_into_tensor`` on CPU, then H2D into every
rank's region), so such worlds execute the SAME restore branches as an RCCL
world -- sliced H2D / HBM-tier D2D, the all-gather, the scatter kernel --
and only the transport of the gather differs.

Reference: the reference restores a replicated checkpoint with every rank
reading the whole shm segment (``flash_checkpoint/engine.py:332-347``); the
sliced restore is this framework's xGMI design.
"""

import torch
import torch.distributed as dist

_CHUNK = 256 << 20  # bytes per rank per staged gather round (pinned: world x chunk)


def _is_device_backend(group) -> bool:
    try:
        return dist.get_backend(group) != "gloo"
    except Exception:
        return False


def all_gather_slices(full: torch.Tensor, mine: torch.Tensor, group, chunk_bytes: int = _CHUNK) -> str:
    """``full`` (uint8, world * per) receives rank r's ``mine`` (per bytes,
    a view of ``full`` is fine) at ``[r * per, (r + 1) * per)``.  Returns the
    transport used: ``"device"`` (RCCL) or ``"host-staged"`` (gloo)."""
    if not full.is_cuda or _is_device_backend(group):
        dist.all_gather_into_tensor(full, mine, group=group)
        return "device" if full.is_cuda else "host"
    world = dist.get_world_size(group)
    per = mine.numel()
    assert full.numel() == per * world, (full.numel(), per, world)
    c = max(1, min(per, chunk_bytes))
    host_mine = torch.empty(c, dtype=torch.uint8, pin_memory=True)
    host_all = torch.empty(c * world, dtype=torch.uint8, pin_memory=True)
    stream = torch.cuda.current_stream(full.device)
    for o in range(0, per, c):
        n = min(c, per - o)
        hm = host_mine[:n]
        hm.copy_(mine[o:o + n], non_blocking=True)
        stream.synchronize()
        ha = host_all[: n * world]
        dist.all_gather_into_tensor(ha, hm, group=group)
        hv = ha.view(world, n)
        for r in range(world):
            full[r * per + o: r * per + o + n].copy_(hv[r], non_blocking=True)
        stream.synchronize()  # the pinned buffers are reused by the next round
    return "host-staged"
