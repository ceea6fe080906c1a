"""GPU prefetching wrapper: batch i+1 is copied host->device on a side HIP
stream while step i computes.

Parity: ATorch ``atorch/data/preloader.py`` (``GpuPreLoader``: ``preload``,
``post_processing``, mask-aware ``to_gpu``).
"""

from typing import Callable, Optional

import torch
import torch.utils._pytree as pytree


class GpuPreLoader:
    def __init__(self, loader, device=None, post_processing: Optional[Callable] = None, pin_memory: bool = True):
        self.loader = loader
        self.device = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
        self.post_processing = post_processing
        self.pin = pin_memory and self.device.type == "cuda"
        self.stream = torch.cuda.Stream(self.device) if self.device.type == "cuda" else None
        self._it = None
        self._next = None
        self._event = None

    def __len__(self):
        return len(self.loader)

    def __getattr__(self, name):  # sampler, batch_size, drop_last, ... of the wrapped loader
        if name in ("loader",):
            raise AttributeError(name)
        return getattr(self.loader, name)

    def _move(self, batch):
        def mv(x):
            if not isinstance(x, torch.Tensor):
                return x
            if self.pin and not x.is_pinned():
                x = x.pin_memory()
            return x.to(self.device, non_blocking=True)

        return pytree.tree_map(mv, batch)

    def preload(self):
        try:
            batch = next(self._it)
        except StopIteration:
            self._next = None
            return
        if self.stream is None:
            self._next = self.post_processing(batch) if self.post_processing else batch
            return
        with torch.cuda.stream(self.stream):
            b = self._move(batch)
            if self.post_processing is not None:
                b = self.post_processing(b)
            self._event = torch.cuda.Event()
            self._event.record(self.stream)
        self._next = b

    def __iter__(self):
        self._it = iter(self.loader)
        self.preload()
        return self

    def __next__(self):
        if self._next is None:
            raise StopIteration
        batch = self._next
        if self.stream is not None:
            cur = torch.cuda.current_stream(self.device)
            cur.wait_event(self._event)
            pytree.tree_map(lambda x: x.record_stream(cur) if isinstance(x, torch.Tensor) and x.is_cuda else x,
                            batch)
        self.preload()
        return batch
