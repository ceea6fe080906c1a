"""Random streams that are equal exactly across the chosen parallel
dimensions (reference: atorch/modules/distributed_modules/randomizer.py
``MultiDimParallelRandomizer`` / ``get_randomizer``).

With parallel dimensions d_0..d_{n-1} (sizes s_i, this rank's index r_i) a
request for "the same stream across dimensions G" gets the seed

    base + code(G) * prod(s) + sum_{i not in G} r_i * prod(s_0..s_{i-1})

so ranks that differ only along dimensions in G share it and every other
pair differs (``code`` keeps the streams of different G apart).  Typical
uses: weight init equal across tensor ranks and data replicas
(``get_randomizer("tensor", "data")``), dropout on replicated TP
activations equal across the tensor group (``get_randomizer("tensor")``),
dropout on sharded activations different everywhere (``get_randomizer()``).

Two ways to draw from a stream:
  * ``with r.fork(): ...`` swaps torch's CPU and GPU generator states in and
    out (the reference's mechanism; any torch random op inside);
  * ``seed, offset = r.philox(n)`` hands a (seed, counter offset) pair to
    the framework's counter-hash kernels (attention dropout:
    ``ops/attention.py``, AttnExt seed / offset) and advances the counter by
    ``n`` -- no generator state touched, nothing synchronised, and the
    backward regenerates the identical mask from the same pair.
Both are checkpointable (``get_states`` / ``set_states``).
"""

from contextlib import contextmanager
from typing import Dict, Optional, Tuple

import torch


class _Stream:
    def __init__(self, seed: int):
        self.seed = int(seed)
        self.offset = 0
        cpu = torch.get_rng_state()
        torch.manual_seed(self.seed)
        self.cpu_rng = torch.get_rng_state()
        torch.set_rng_state(cpu)
        self.cuda_rng = None
        if torch.cuda.is_available():
            cur = torch.cuda.get_rng_state()
            torch.cuda.manual_seed(self.seed)
            self.cuda_rng = torch.cuda.get_rng_state()
            torch.cuda.set_rng_state(cur)

    @contextmanager
    def fork(self):
        cpu = torch.get_rng_state()
        torch.set_rng_state(self.cpu_rng)
        gpu = None
        if self.cuda_rng is not None:
            gpu = torch.cuda.get_rng_state()
            torch.cuda.set_rng_state(self.cuda_rng)
        try:
            yield self
        finally:
            self.cpu_rng = torch.get_rng_state()
            torch.set_rng_state(cpu)
            if gpu is not None:
                self.cuda_rng = torch.cuda.get_rng_state()
                torch.cuda.set_rng_state(gpu)

    def philox(self, n: int = 1) -> Tuple[int, int]:
        """(seed, offset) for ``n`` counter-hash draws; advances the counter."""
        out = (self.seed, self.offset)
        self.offset += int(n)
        return out


class MultiDimParallelRandomizer:
    def __init__(self, base_seed: int = 1234, dims: Optional[Dict[str, Tuple[int, int]]] = None):
        """``dims``: {name: (size, rank)} in a fixed order; default: the
        named parallel groups of ``atorch.distributed`` (create_parallel_group)."""
        if dims is None:
            from ..atorch import distributed as adist

            cfg = adist.parallel_config()
            names = [n for n, _s in cfg[0]] if cfg else []
            dims = {n: (int(adist.parallel_group_size(n) or 1), int(adist.parallel_rank(n) or 0)) for n in names}
        self.base_seed = int(base_seed)
        self.names = list(dims)
        self.sizes = [dims[n][0] for n in self.names]
        self.ranks = [dims[n][1] for n in self.names]
        self.stride = [1]
        for s in self.sizes:
            self.stride.append(self.stride[-1] * s)
        self._streams: Dict[Tuple[bool, ...], _Stream] = {}

    def seed_for(self, *same_groups: str) -> int:
        bad = [g for g in same_groups if g not in self.names]
        if bad:
            raise ValueError(f"unknown parallel dimensions {bad}; have {self.names}")
        same = tuple(n in same_groups for n in self.names)
        code = sum(1 << i for i, s in enumerate(same) if s)
        off = code * self.stride[-1] + sum(r * self.stride[i] for i, (r, s) in enumerate(zip(self.ranks, same))
                                           if not s)
        return self.base_seed + off

    def get_randomizer(self, *same_groups: str) -> _Stream:
        key = tuple(n in same_groups for n in self.names)
        if key not in self._streams:
            self._streams[key] = _Stream(self.seed_for(*same_groups))
        return self._streams[key]

    def get_states(self) -> dict:
        return {k: {"cpu_rng": s.cpu_rng, "cuda_rng": s.cuda_rng, "offset": s.offset} for k, s in self._streams.items()}

    def set_states(self, states: dict):
        for k, st in states.items():
            k = tuple(k)
            if k not in self._streams:
                self._streams[k] = _Stream(self.seed_for(*[n for n, s in zip(self.names, k) if s]))
            s = self._streams[k]
            s.cpu_rng, s.offset = st["cpu_rng"], int(st.get("offset", 0))
            if st.get("cuda_rng") is not None and s.cuda_rng is not None:
                s.cuda_rng = st["cuda_rng"]


_INSTANCE: Optional[MultiDimParallelRandomizer] = None


def init_randomizer(base_seed: int = 1234, dims=None) -> MultiDimParallelRandomizer:
    global _INSTANCE
    if _INSTANCE is not None:
        raise RuntimeError("multi-dimension parallel randomizer already initialised")
    _INSTANCE = MultiDimParallelRandomizer(base_seed, dims)
    return _INSTANCE


def get_MDPRInstance() -> MultiDimParallelRandomizer:  # noqa: N802  (reference name)
    if _INSTANCE is None:
        raise RuntimeError("multi-dimension parallel randomizer not initialised (init_randomizer)")
    return _INSTANCE


def get_randomizer(*same_groups: str) -> _Stream:
    return get_MDPRInstance().get_randomizer(*same_groups)


def reset_randomizer():
    global _INSTANCE
    _INSTANCE = None


__all__ = ["MultiDimParallelRandomizer", "init_randomizer", "get_MDPRInstance", "get_randomizer",
           "reset_randomizer"]
