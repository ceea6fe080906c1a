"""Dynamic data sharding client (workers pull shards from the master).

Parity: reference ``dlrover/python/elastic_agent/sharding/client.py``
(``ShardingClient`` :29-228, ``IndexShardingClient`` :231-330).  A worker
that dies loses nothing: its un-acknowledged shards time out on the master
and are handed to another worker; ``get_shard_checkpoint`` /
``restore_shard_from_checkpoint`` save and restore the dataset position.
"""

import queue
import sys
import threading
from collections import OrderedDict
from typing import List, Optional

from ..common import comm
from ..common.log import logger
from .master_client import MasterClient

_DEFAULT_MINI_BATCH_NUM_PER_SHARD = 10


class TaskType:
    NONE = 0
    TRAINING = 1
    EVALUATION = 2
    PREDICTION = 3
    WAIT = 4


class ShardingClient:
    """Fetch shards ``[start, end)`` of a dataset of ``dataset_size`` records
    and acknowledge them batch by batch.

    >>> client = ShardingClient("train", batch_size=64, num_epochs=1, dataset_size=10000)
    >>> while (shard := client.fetch_shard()):
    ...     for i in range(shard.start, shard.end): ...
    ...     client.report_batch_done()
    """

    def __init__(self, dataset_name, batch_size, num_epochs, dataset_size, shuffle=False,
                 task_type=TaskType.TRAINING, num_minibatches_per_shard=_DEFAULT_MINI_BATCH_NUM_PER_SHARD,
                 storage_type="", master_client: Optional[MasterClient] = None):
        self._mc = master_client or MasterClient.singleton_instance()
        self._batch_size = batch_size
        self._num_epochs = num_epochs
        self._dataset_size = dataset_size
        self._shuffle = shuffle
        self._task_type = task_type
        self._storage_type = storage_type
        self._num_minibatches_per_shard = num_minibatches_per_shard
        self._lock = threading.Lock()
        self._reported_record_count = {}
        self._current_task = None
        self._pending_tasks: "OrderedDict[int, comm.Task]" = OrderedDict()
        self._dataset_name = dataset_name
        self._batch_count = 0
        self._max_shard_count = sys.maxsize
        self._shard_count = 0
        self._report_sharding_params()

    def _report_sharding_params(self):
        if self._num_epochs and self._dataset_size:
            self._mc.report_dataset_shard_params(
                batch_size=self._batch_size, num_epochs=self._num_epochs, dataset_size=self._dataset_size,
                shuffle=self._shuffle, num_minibatches_per_shard=self._num_minibatches_per_shard,
                dataset_name=self._dataset_name, task_type=self._task_type, storage_type=self._storage_type)

    def get_minibatch_count_per_epoch(self):
        return self._dataset_size // self._batch_size

    def get_current_task(self):
        return self._current_task

    def get_task(self) -> Optional[comm.Task]:
        if self._shard_count >= self._max_shard_count:
            return None
        task = self._mc.get_task(self._dataset_name)
        if task is None or task.task_id < 0 or task.shard is None:
            return None
        with self._lock:
            self._pending_tasks[task.task_id] = task
            if len(self._pending_tasks) == 1:
                self._current_task = task
        self._shard_count += 1
        return task

    def _report_task(self, task: comm.Task, err_msg: str = ""):
        self._mc.report_task_result(self._dataset_name, task.task_id, err_msg)

    def report_all_task_error(self, err_msg):
        while self._pending_tasks:
            _, task = self._pending_tasks.popitem(last=False)
            self._report_task(task, err_msg)

    def report_batch_done(self, batch_size: Optional[int] = None, err_msg: str = "",
                          task_ids: Optional[List[int]] = None) -> bool:
        """Acknowledge ``batch_size`` records; a shard is reported done once
        all of its records are acknowledged."""
        record_count = batch_size or self._batch_size
        self._batch_count += 1
        with self._lock:
            if not task_ids:
                task_ids = list(self._pending_tasks.keys())
            for tid in task_ids:
                task = self._pending_tasks.get(tid)
                if task is None:
                    continue
                shard = task.shard
                size = (len(shard.indices) if shard.indices else shard.end - shard.start)
                done = self._reported_record_count.get(tid, 0) + record_count
                if done >= size:
                    self._report_task(task, err_msg)
                    self._pending_tasks.pop(tid)
                    self._reported_record_count.pop(tid, None)
                    record_count = done - size
                    self._current_task = next(iter(self._pending_tasks.values()), None)
                    if record_count <= 0:
                        break
                else:
                    self._reported_record_count[tid] = done
                    break
        return True

    def fetch_shard(self) -> Optional[comm.Shard]:
        task = self.get_task()
        return task.shard if task else None

    def get_shard_checkpoint(self) -> str:
        return self._mc.get_shard_checkpoint(self._dataset_name)

    def restore_shard_from_checkpoint(self, shard_checkpoint: str) -> bool:
        return self._mc.report_shard_checkpoint(shard_checkpoint)

    def get_total_sample_num(self):
        return self._dataset_size * self._num_epochs


class IndexShardingClient(ShardingClient):
    """Yields sample indices one by one (prefetching shards in a thread),
    e.g. for a ``torch.utils.data.Sampler``."""

    def __init__(self, dataset_name, batch_size, num_epochs, dataset_size, shuffle=False,
                 task_type=TaskType.TRAINING, num_minibatches_per_shard=_DEFAULT_MINI_BATCH_NUM_PER_SHARD,
                 storage_type="", num_workers: int = 1, master_client: Optional[MasterClient] = None):
        super().__init__(dataset_name, batch_size, num_epochs, dataset_size, shuffle, task_type,
                         num_minibatches_per_shard, storage_type, master_client)
        self._num_workers = num_workers
        self._sample_queue: "queue.Queue[int]" = queue.Queue(maxsize=batch_size * num_minibatches_per_shard * 4)
        self._exhausted = threading.Event()
        self._thread = threading.Thread(target=self._prefetch_sample_indices, daemon=True,
                                        name="dwamd-index-prefetch")
        self._thread.start()

    def _prefetch_sample_indices(self):
        while True:
            task = self.get_task()
            if task is None:
                self._exhausted.set()
                self._sample_queue.put(-1)
                return
            s = task.shard
            for i in (s.indices if s.indices else range(s.start, s.end)):
                self._sample_queue.put(int(i))

    def fetch_sample_index(self) -> Optional[int]:
        """Next sample index, or None when the dataset is exhausted."""
        i = self._sample_queue.get()
        if i < 0:
            self._sample_queue.put(-1)
            return None
        return i

    def clear_shard_queue(self):
        while not self._sample_queue.empty():
            try:
                self._sample_queue.get_nowait()
            except queue.Empty:
                break

    def restore_shard_from_checkpoint(self, shard_checkpoint: str) -> bool:
        self.clear_shard_queue()
        ok = super().restore_shard_from_checkpoint(shard_checkpoint)
        logger.info(f"restored dataset shards from checkpoint: {ok}")
        return ok
