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
        """Restore a ``get_states`` snapshot.  Streams first requested after
        the snapshot did not exist then: they go back to their initial
        state (a checkpoint recompute replays them from the start too)."""
        for k in [k for k in self._streams if k not in {tuple(x) for x in states}]:
            self._streams[k] = _Stream(self._streams[k].seed)
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


# ------------------------------------------------ Megatron-style named tracker
class CudaRNGStatesTracker:
    """Named GPU generator states (reference activation_checkpointing.py
    ``CudaRNGStatesTracker``): ``add(name, seed)``, ``fork(name)``,
    ``get_states`` / ``set_states``.  On a host without a GPU the CPU
    generator is tracked instead (the CPU / gloo execution path)."""

    def __init__(self):
        self.states_: Dict[str, torch.Tensor] = {}
        self.seeds_ = set()

    @staticmethod
    def _get():
        return torch.cuda.get_rng_state() if torch.cuda.is_available() else torch.get_rng_state()

    @staticmethod
    def _set(st):
        (torch.cuda.set_rng_state if torch.cuda.is_available() else torch.set_rng_state)(st)

    def reset(self):
        self.states_, self.seeds_ = {}, set()

    def get_states(self) -> Dict[str, torch.Tensor]:
        return dict(self.states_)

    def set_states(self, states: Dict[str, torch.Tensor]):
        self.states_ = dict(states)

    def add(self, name: str, seed: int):
        if seed in self.seeds_ or name in self.states_:
            raise RuntimeError(f"rng state {name} / seed {seed} already tracked")
        self.seeds_.add(seed)
        cur = self._get()
        (torch.cuda.manual_seed if torch.cuda.is_available() else torch.manual_seed)(seed)
        self.states_[name] = self._get()
        self._set(cur)

    @contextmanager
    def fork(self, name: str = "model-parallel-rng"):
        if name not in self.states_:
            raise RuntimeError(f"rng state {name} is not tracked")
        cur = self._get()
        self._set(self.states_[name])
        try:
            yield
        finally:
            self.states_[name] = self._get()
            self._set(cur)


_TRACKER = CudaRNGStatesTracker()


def get_cuda_rng_tracker() -> CudaRNGStatesTracker:
    return _TRACKER


def model_parallel_cuda_manual_seed(seed: int, group: str = "tensor"):
    """Default generator: ``seed`` (equal across the tensor group, as the
    replicated regions need); tracked "model-parallel-rng": seed + 2718 +
    tensor rank (different across the tensor group, equal across data
    replicas) for dropout inside the sharded regions."""
    from ..atorch import distributed as adist

    r = adist.parallel_rank(group) or 0
    (torch.cuda.manual_seed if torch.cuda.is_available() else torch.manual_seed)(seed)
    _TRACKER.reset()
    _TRACKER.add("model-parallel-rng", seed + 2718 + r)


# ------------------------------------------ RNG-consistent activation checkpoint
def _rng_context():
    """(forward, recompute) contexts for torch.utils.checkpoint: the
    recompute replays the randomizer streams and tracked states (incl. the
    counter offsets) exactly as the forward saw them, so dropout inside a
    forked stream regenerates the same mask."""
    from contextlib import nullcontext

    inst = _INSTANCE
    snap_streams = inst.get_states() if inst is not None else None
    snap_tracker = _TRACKER.get_states()

    @contextmanager
    def recompute():
        cur_streams = inst.get_states() if inst is not None else None
        cur_tracker = _TRACKER.get_states()
        if inst is not None:
            inst.set_states(snap_streams)
        _TRACKER.set_states(snap_tracker)
        try:
            yield
        finally:
            if inst is not None:
                inst.set_states(cur_streams)
            _TRACKER.set_states(cur_tracker)

    return nullcontext(), recompute()


def rng_checkpoint(function, *args, **kwargs):
    """Non-reentrant activation checkpoint that also restores the parallel
    randomizer / tracker states for the recompute (reference
    ``CheckpointFunction`` / ``checkpoint``; torch's own checkpoint restores
    only the default generators)."""
    return torch.utils.checkpoint.checkpoint(function, *args, use_reentrant=False, context_fn=_rng_context,
                                             **kwargs)


def tp_wrap_fn(module: torch.nn.Module) -> torch.nn.Module:
    """Wrap ``module`` so its forward runs under :func:`rng_checkpoint`
    (reference ``TPCheckpointWrapper`` / ``tp_wrap_fn``)."""
    from torch.distributed.algorithms._checkpoint.checkpoint_wrapper import checkpoint_wrapper

    return checkpoint_wrapper(module, checkpoint_fn=rng_checkpoint)


__all__ = ["MultiDimParallelRandomizer", "init_randomizer", "get_MDPRInstance", "get_randomizer",
           "reset_randomizer", "CudaRNGStatesTracker", "get_cuda_rng_tracker", "model_parallel_cuda_manual_seed",
           "rng_checkpoint", "tp_wrap_fn"]
