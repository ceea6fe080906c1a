"""Data loading through node-local shared memory.

Two deployments (same as ATorch's ``ShmDataContext`` O1/O2 cases):

* **Model-parallel group** (``ShmDataLoader``): ranks of one tensor/sequence
  parallel group need the SAME batch.  The group's rank 0 runs the real
  ``DataLoader`` (workers, collation) and publishes every batch into a
  BROADCAST ring; the other ranks read it from shared memory instead of
  running their own (duplicate) input pipelines.
* **Coworkers** (``coworker_produce`` + ``ShmDataLoader(coworker=True)``):
  dedicated producer processes preprocess data into a SHARED ring and the
  training processes each take distinct batches from it.

With ``device="cuda"`` a reader's batches arrive as device tensors copied by
DMA straight from the registered shm slot (see ``shm_ring``).

Parity: ATorch ``atorch/data/shm_dataloader.py`` (``ShmDataloader``,
``create_shm_dataloader``) and ``shm_context.py``.
"""

import os
from typing import Optional

import torch
from torch.utils.data import DataLoader, Dataset, Subset

from ...common.log import logger
from .shm_ring import BROADCAST, SHARED, ShmBatchRing, batch_nbytes


def _ring_name(prefix: str) -> str:
    job = os.getenv("TORCHELASTIC_RUN_ID", os.getenv("DWAMD_JOB_NAME", "local"))
    return f"dwamd_data_{job}_{prefix}".replace("/", "_")


def _to_device(batch, device):
    if device is None:
        return batch
    return torch.utils._pytree.tree_map(
        lambda x: x.to(device, non_blocking=True) if isinstance(x, torch.Tensor) else x, batch)


def get_loader_size(dataset, **dataloader_args) -> int:
    return len(DataLoader(dataset, **{k: v for k, v in dataloader_args.items() if k != "num_workers"}))


class ShmDataLoader:
    """Iterable over batches; ``len()`` is known when the dataset is sized.

    Args:
        dataset, dataloader_args: the loader rank 0 (or each coworker) runs.
        rank, group_size: rank within the model-parallel group sharing batches.
        shm_data_size: ring slots (batches in flight).
        slot_bytes: slot size; default 2x the first batch (min 1 MiB).
        device: move/copy batches to this device.
        coworker: read from a coworker SHARED ring instead of a group rank 0.
    """

    def __init__(self, dataset: Optional[Dataset], dataloader_args: dict, rank: int = 0, group_size: int = 1,
                 shm_name_prefix: str = "batch", shm_data_size: int = 8, slot_bytes: Optional[int] = None,
                 io_timeout: float = 60.0, initialize_timeout: float = 300.0, device=None, coworker: bool = False):
        self.dataset = dataset
        self.args = dict(dataloader_args)
        self.rank, self.group_size = rank, group_size
        self.name = _ring_name(shm_name_prefix)
        self.io_timeout = io_timeout
        self.device = device
        self.coworker = coworker
        self.epoch = 0
        self.ring: Optional[ShmBatchRing] = None
        self.loader: Optional[DataLoader] = None
        self.is_producer = (not coworker) and rank == 0
        if self.is_producer:
            self.loader = DataLoader(dataset, **self.args)
            if group_size > 1:
                if slot_bytes is None:
                    first = next(iter(DataLoader(dataset, **{**self.args, "num_workers": 0})))
                    slot_bytes = max(1 << 20, 2 * batch_nbytes(first))
                self.ring = ShmBatchRing(self.name, True, nslots=shm_data_size, slot_bytes=slot_bytes,
                                         nreaders=group_size - 1, mode=BROADCAST)
        else:
            self.ring = ShmBatchRing(self.name, False, timeout=initialize_timeout)

    def __len__(self):
        if self.loader is not None:
            return len(self.loader)
        if self.dataset is not None and hasattr(self.dataset, "__len__"):
            return get_loader_size(self.dataset, **self.args)
        raise TypeError("length unknown on a coworker-fed reader")

    def __iter__(self):
        epoch = self.epoch
        self.epoch += 1
        if self.is_producer:
            if self.ring is not None and epoch > 0:
                self.ring.next_epoch(self.io_timeout * 10)
            try:
                for batch in self.loader:
                    if self.ring is not None:
                        self.ring.put(batch, self.io_timeout)
                    yield _to_device(batch, self.device)
            finally:
                if self.ring is not None:
                    self.ring.stop()
            return
        if not self.coworker:
            self.ring.wait_epoch(epoch, self.io_timeout * 10)
        reader = 0 if self.coworker else self.rank - 1
        gpu = self.device is not None and torch.device(self.device).type == "cuda"
        while True:
            b = self.ring.get(reader, self.io_timeout, device=self.device if gpu else None)
            if b is None:
                return
            yield b if gpu else _to_device(b, self.device)

    def stop(self):
        if self.ring is not None:
            self.ring.abort()

    def close(self):
        if self.ring is not None:
            self.ring.close()
            self.ring = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def create_shm_dataloader(dataset, dataloader_args, rank: int = 0, group_size: int = 1, **kw) -> ShmDataLoader:
    return ShmDataLoader(dataset, dataloader_args, rank=rank, group_size=group_size, **kw)


def coworker_produce(dataset: Dataset, dataloader_args: dict, coworker_rank: int, num_coworkers: int,
                     shm_name_prefix: str = "coworker", shm_data_size: int = 16, slot_bytes: Optional[int] = None,
                     io_timeout: float = 300.0, initialize_timeout: float = 300.0, process_fn=None) -> int:
    """Run in a coworker process: load this coworker's share of ``dataset``
    (strided by coworker rank), optionally post-process each batch, and
    publish the batches into the SHARED ring the workers read.  Coworker 0
    creates the ring.  Returns the number of batches produced."""
    name = _ring_name(shm_name_prefix)
    shard = Subset(dataset, range(coworker_rank, len(dataset), num_coworkers))
    loader = DataLoader(shard, **dataloader_args)
    if coworker_rank == 0:
        if slot_bytes is None:
            first = next(iter(DataLoader(shard, **{**dataloader_args, "num_workers": 0})))
            if process_fn is not None:
                first = process_fn(first)
            slot_bytes = max(1 << 20, 2 * batch_nbytes(first))
        ring = ShmBatchRing(name, True, nslots=shm_data_size, slot_bytes=slot_bytes, mode=SHARED,
                            nproducers=num_coworkers)
    else:
        ring = ShmBatchRing(name, False, timeout=initialize_timeout)
    n = 0
    try:
        for batch in loader:
            if process_fn is not None:
                batch = process_fn(batch)
            if not ring.put(batch, io_timeout):
                break
            n += 1
    finally:
        ring.stop()
    logger.info(f"coworker {coworker_rank}: produced {n} batches")
    ring.close(unlink=False)
    return n
