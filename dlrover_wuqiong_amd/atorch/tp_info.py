"""Manual tensor-parallel annotations and the 3D-parallel config object of
ATorch's DeepSpeed path (reference: atorch/atorch/utils/manual_tp_utils.py
``TPInfo``; auto/opt_lib/ds_3d_parallel_optimization.py
``DeepSpeed3DParallelConfig``).

Here the TP rebuild of a Llama is structural (models/llama.py Megatron layers,
atorch/tp_planner.py for other models), so a ``TPInfo`` is a declaration the
planner checks against, not a required input: user scripts that build one run
unchanged, and ``mixed_parallel`` reads ``ds_config`` / ``batch_fn`` from the
config object.
"""

from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Set


class TPInfo:
    """Which sub-modules are column / row / vocab sharded, and which
    attributes shrink with the shard (e.g. ``num_heads``)."""

    def __init__(self):
        self.col: List[str] = []
        self.row: List[str] = []
        self.vocab: List[str] = []
        self.shrink_attrs: Dict[str, Set[str]] = {}
        self.replicate: List[str] = []

    def shard_col(self, *names):
        self.col.extend(names)
        return self

    def shard_row(self, *names):
        self.row.extend(names)
        return self

    def shard_vocab(self, *names):
        self.vocab.extend(names)
        return self

    def shrink(self, spec: Dict[str, Set[str]]):
        for k, v in spec.items():
            self.shrink_attrs.setdefault(k, set()).update(v)
        return self

    def replic(self, *names):
        self.replicate.extend(names)
        return self

    def kind_of(self, qualified_name: str) -> Optional[str]:
        """"col" / "row" / "vocab" for a module name ending in a declared suffix."""
        for kind, names in (("col", self.col), ("row", self.row), ("vocab", self.vocab)):
            if any(qualified_name == n or qualified_name.endswith("." + n) for n in names):
                return kind
        return None


@dataclass
class DeepSpeed3DParallelConfig:
    """TP x PP x DP config for ``auto_accelerate``'s ``deepspeed_3d_parallel``
    (= ``mixed_parallel``).  Sizes default to the ``parallel_mode`` groups;
    ``ds_config`` (dict or JSON path) gives ``gradient_accumulation_steps`` =
    micro-batches per pipeline step; ``batch_fn`` maps a loader batch to
    ``(inputs, labels)`` for ``model.train_batch(data_iter)``."""

    tpinfo: Optional[TPInfo] = None
    ds_config: Any = None
    batch_fn: Optional[Callable] = None
    tensor: int = 0
    pipeline: int = 0
    data: int = 0
    schedule: str = "1f1b"
    virtual_stages: int = 1
    extra: Dict[str, Any] = field(default_factory=dict)
