"""Keyed replay buffer for RL samples (dict of per-key lists) with a
process-group sync.

``sync`` gathers every rank's samples so each data-parallel rank trains on
the union: tensors travel as one padded ``all_gather`` per key over the
group's backend (RCCL for cuda tensors, gloo for cpu) -- no pickling of
tensor payloads; only the per-rank sample counts and shapes go through
``all_gather_object``.

Parity: ATorch ``atorch/rl/replay_buffer/replay_buffer.py`` (reset,
add_samples, add_sample with in-place index update, sync, create_dataset;
the reference's sync is a stub).
"""

from typing import Dict, List, Optional

import torch
import torch.distributed as dist


class SampleReplayBuffer:
    def __init__(self, config=None, element_keys: Optional[List[str]] = None):
        self.config = config
        self.element_keys = element_keys
        self.data: Dict[str, list] = {}
        self.num = 0

    def reset(self):
        for k in self.data:
            self.data[k] = []
        self.num = 0

    def add_samples(self, samples: list):
        assert isinstance(samples, list)
        for s in samples:
            self.add_sample(s)

    def add_sample(self, sample: dict, index: Optional[int] = None) -> bool:
        """Append ``sample`` or, with ``index``, overwrite that sample's keys
        in place (False if the index does not exist)."""
        if self.element_keys is not None and not set(sample).issubset(self.element_keys):
            raise KeyError(f"sample keys {sorted(sample)} not in the buffer's {sorted(self.element_keys)}")
        if index is not None:
            if any(len(self.data.get(k, [])) <= index for k in sample):
                return False
            for k, v in sample.items():
                self.data[k][index] = v
            return True
        for k, v in sample.items():
            self.data.setdefault(k, []).append(v)
        self.num += 1
        return True

    def __len__(self):
        return self.num

    def __getitem__(self, i: int) -> dict:
        return {k: v[i] for k, v in self.data.items()}

    def sync(self, process_group=None):
        """All-gather every rank's samples (rank order) into every rank."""
        if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(process_group) == 1:
            return
        ws = dist.get_world_size(process_group)
        keys = sorted(self.data)
        meta = {k: [(tuple(t.shape), t.dtype) if torch.is_tensor(t) else None for t in self.data[k]] for k in keys}
        metas = [None] * ws
        dist.all_gather_object(metas, (self.num, keys, meta), group=process_group)
        if any(m[1] != keys for m in metas):
            raise RuntimeError(f"replay buffer keys differ across ranks: {[m[1] for m in metas]}")
        dev = torch.device("cpu")
        if dist.get_backend(process_group) == "nccl":
            dev = torch.device("cuda", torch.cuda.current_device())
        new: Dict[str, list] = {k: [] for k in keys}
        for k in keys:
            tensors = [t for t in self.data[k] if torch.is_tensor(t)]
            if len(tensors) != len(self.data[k]):
                # non-tensor values (strings, scores as floats): small, gathered as objects
                objs = [None] * ws
                dist.all_gather_object(objs, self.data[k], group=process_group)
                for o in objs:
                    new[k].extend(o)
                continue
            dtype = tensors[0].dtype if tensors else next(
                (m[2][k][0][1] for m in metas if m[2][k]), torch.float32)
            flat = torch.cat([t.reshape(-1) for t in tensors]).to(dev, dtype) if tensors else \
                torch.empty(0, dtype=dtype, device=dev)
            sizes = [sum(int(torch.Size(s).numel()) for s, _ in m[2][k]) for m in metas]
            buf = [torch.empty(max(sizes), dtype=dtype, device=dev) for _ in range(ws)]
            pad = torch.empty(max(sizes), dtype=dtype, device=dev)
            pad[:flat.numel()] = flat
            dist.all_gather(buf, pad, group=process_group)
            for r, m in enumerate(metas):
                off = 0
                for shape, _ in m[2][k]:
                    n = int(torch.Size(shape).numel())
                    new[k].append(buf[r][off:off + n].view(shape).to(tensors[0].device if tensors else "cpu"))
                    off += n
        self.data = new
        self.num = sum(m[0] for m in metas)

    def create_dataset(self):
        return _BufferDataset(self)


class _BufferDataset(torch.utils.data.Dataset):
    def __init__(self, buf: SampleReplayBuffer):
        self.buf = buf

    def __len__(self):
        return len(self.buf)

    def __getitem__(self, i):
        return self.buf[i]
