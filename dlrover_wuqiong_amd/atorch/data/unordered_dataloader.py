"""DataLoader that yields batches in COMPLETION order from a shared work queue.

A stock ``DataLoader`` assigns batch k to worker k mod W up front and hands
batches out in index order, so one slow sample (a huge image, a remote read,
a decode retry) stalls every batch behind it, and the batches queued on the
slow worker wait even when the other workers are idle.  Here:

  * the main process keeps ``prefetch_factor * num_workers`` batches of
    indices in ONE shared index queue; whichever worker is free takes the
    next one (work stealing -- a slow worker holds at most the batch it is
    on, nothing queued behind it);
  * results come back through one result queue and are yielded as they
    arrive, every batch exactly once; each received batch refills one index
    batch;
  * worker exceptions are re-raised in the main process with the worker's
    traceback; a worker that dies (OOM kill, segfault) is detected from its
    exit code while the main process waits, instead of hanging;
  * ``stats()`` reports how many batches each worker produced (load balance).

Map-style datasets only (an iterable dataset has no index to hand out); for
iterable datasets and ``num_workers == 0`` it behaves like ``DataLoader``.

Parity: ATorch ``atorch/data/unordered_dataloader.py``
(``_MultiProcessingUnorderedDataLoaderIter``: completion-order ``_next_data``,
``_try_put_index`` refilling the worker that just finished).  The shared
queue is a different mechanism with the same goal: no batch waits behind
a slow one.
"""

import multiprocessing as mp
import queue
import traceback
from typing import Any, Callable, Iterator, List, Optional

import torch
from torch.utils.data import BatchSampler, DataLoader, IterableDataset, RandomSampler, SequentialSampler

_POLL_S = 1.0


class _WorkerError:
    def __init__(self, worker_id: int, exc: BaseException):
        self.worker_id = worker_id
        self.exc_type = type(exc).__name__
        self.text = "".join(traceback.format_exception(type(exc), exc, exc.__traceback__))

    def reraise(self):
        raise RuntimeError(f"worker {self.worker_id} raised {self.exc_type}:\n{self.text}")


def _worker_loop(worker_id: int, dataset, collate_fn: Callable, index_q, result_q, seed: int,
                 worker_init_fn: Optional[Callable]):
    torch.manual_seed(seed + worker_id)
    torch.set_num_threads(1)
    try:
        if worker_init_fn is not None:
            worker_init_fn(worker_id)
    except Exception as e:  # reported with the first batch request
        err = _WorkerError(worker_id, e)
        while True:
            task = index_q.get()
            if task is None:
                return
            result_q.put((task[0], worker_id, err))
    while True:
        task = index_q.get()
        if task is None:
            return
        bidx, indices = task
        try:
            out = collate_fn([dataset[i] for i in indices])
        except Exception as e:
            out = _WorkerError(worker_id, e)
        result_q.put((bidx, worker_id, out))


class _UnorderedIter:
    def __init__(self, loader: "UnorderedDataLoader"):
        self._loader = loader
        ctx = loader.multiprocessing_context or mp.get_context()
        self._index_q = ctx.Queue()
        self._result_q = ctx.Queue()
        self._batches = iter(loader.batch_sampler)
        seed = int(torch.empty((), dtype=torch.int64).random_().item())
        self._workers = [ctx.Process(target=_worker_loop, daemon=True,
                                     args=(w, loader.dataset, loader.collate_fn, self._index_q, self._result_q,
                                           seed, loader.worker_init_fn))
                         for w in range(loader.num_workers)]
        for p in self._workers:
            p.start()
        self._sent = 0
        self._received = 0
        self._exhausted = False
        self._per_worker = [0] * loader.num_workers
        self._closed = False
        for _ in range(loader.prefetch_factor * loader.num_workers):
            if not self._put_one():
                break

    def _put_one(self) -> bool:
        if self._exhausted:
            return False
        try:
            indices = next(self._batches)
        except StopIteration:
            self._exhausted = True
            return False
        self._index_q.put((self._sent, list(indices)))
        self._sent += 1
        return True

    def __iter__(self):
        return self

    def __next__(self):
        if self._received >= self._sent:
            self.close()
            raise StopIteration
        timeout = self._loader.timeout or 0
        waited = 0.0
        while True:
            try:
                _bidx, wid, data = self._result_q.get(timeout=_POLL_S)
                break
            except queue.Empty:
                waited += _POLL_S
                dead = [(i, p.exitcode) for i, p in enumerate(self._workers)
                        if p.exitcode is not None and p.exitcode != 0]
                if dead:
                    self.close()
                    raise RuntimeError(f"unordered dataloader worker(s) exited unexpectedly: {dead}")
                if timeout and waited >= timeout:
                    self.close()
                    raise RuntimeError(f"unordered dataloader timed out after {timeout}s")
        self._received += 1
        self._per_worker[wid] += 1
        if isinstance(data, _WorkerError):
            self.close()
            data.reraise()
        self._put_one()
        if self._loader.pin_memory and torch.cuda.is_available():
            data = _pin(data)
        return data

    def stats(self) -> List[int]:
        return list(self._per_worker)

    def close(self):
        if self._closed:
            return
        self._closed = True
        for _ in self._workers:
            self._index_q.put(None)
        for p in self._workers:
            p.join(timeout=5)
            if p.is_alive():
                p.terminate()
        for q in (self._index_q, self._result_q):
            q.cancel_join_thread()
            q.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _pin(x):
    if torch.is_tensor(x):
        return x.pin_memory()
    if isinstance(x, dict):
        return {k: _pin(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(_pin(v) for v in x)
    return x


class UnorderedDataLoader(DataLoader):
    """``DataLoader`` whose multi-worker iteration yields batches in
    completion order from a shared work queue (see module docstring)."""

    def __init__(self, dataset, batch_size: Optional[int] = 1, shuffle: bool = False, sampler=None,
                 batch_sampler=None, num_workers: int = 0, collate_fn: Optional[Callable] = None,
                 pin_memory: bool = False, drop_last: bool = False, timeout: float = 0,
                 worker_init_fn: Optional[Callable] = None, multiprocessing_context=None,
                 prefetch_factor: Optional[int] = None, **kwargs: Any):
        iterable = isinstance(dataset, IterableDataset)
        if not iterable and batch_sampler is None and batch_size is not None:
            sampler = sampler or (RandomSampler(dataset) if shuffle else SequentialSampler(dataset))
            batch_sampler = BatchSampler(sampler, batch_size, drop_last)
            batch_size, shuffle, sampler, drop_last = 1, False, None, False
        if num_workers > 0 and prefetch_factor is None:
            prefetch_factor = 2
        if iterable and num_workers > 0:
            kwargs["in_order"] = False  # iterable datasets: torch's own completion-order mode
        super().__init__(dataset, batch_size=batch_size, shuffle=shuffle, sampler=sampler,
                         batch_sampler=batch_sampler, num_workers=num_workers,
                         collate_fn=collate_fn, pin_memory=pin_memory, drop_last=drop_last, timeout=timeout,
                         worker_init_fn=worker_init_fn, multiprocessing_context=multiprocessing_context,
                         prefetch_factor=prefetch_factor, **kwargs)
        self._last_iter: Optional[_UnorderedIter] = None

    def __iter__(self) -> Iterator:
        if self.num_workers == 0 or isinstance(self.dataset, IterableDataset) or self.batch_sampler is None:
            return super().__iter__()
        self._last_iter = _UnorderedIter(self)
        return self._last_iter

    def stats(self) -> List[int]:
        """Batches produced per worker by the latest iteration."""
        return self._last_iter.stats() if self._last_iter is not None else []
