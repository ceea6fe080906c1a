"""Cross-process class construction + JSON helpers.

Parity: reference ``dlrover/python/common/serialize.py:28,39``
(``JsonSerializable`` and ``ClassMeta``).  ``ClassMeta`` lets a worker tell
the agent *which* saver/storage class to instantiate without shipping code.
"""

import importlib
import json
from dataclasses import dataclass, field
from typing import Any, Dict


class JsonSerializable:
    def to_json(self, indent=None) -> str:
        return json.dumps(self, default=lambda o: o.__dict__, sort_keys=True, indent=indent)


@dataclass
class ClassMeta:
    module_path: str = ""
    class_name: str = ""
    kwargs: Dict[str, Any] = field(default_factory=dict)

    def build(self):
        module = importlib.import_module(self.module_path)
        cls = getattr(module, self.class_name)
        return cls(**self.kwargs)

    @classmethod
    def of(cls, clazz, **kwargs) -> "ClassMeta":
        return cls(module_path=clazz.__module__, class_name=clazz.__name__, kwargs=kwargs)


# ---------------------------------------------------------------------------
# Restricted unpickling for checkpoint payloads that ``weights_only=True``
# cannot express (Megatron ``args`` namespaces, DCP metadata, numpy RNG
# state, small framework objects).  Only classes from an allow-list of
# modules and a fixed set of reconstruction functions resolve; anything else
# (os.system, subprocess, eval, ...) raises UnpicklingError before its module
# is even imported.
import io  # noqa: E402
import pickle  # noqa: E402

_SAFE_BUILTINS = {"set", "frozenset", "dict", "list", "tuple", "int", "float", "complex", "bytes", "bytearray",
                  "str", "bool", "slice", "range", "NoneType", "Ellipsis"}
# exact (module, name) pairs: plain data classes and the reconstruction
# helpers torch / numpy pickles reference.  Everything not listed here or
# under _CLASS_PREFIXES is refused -- in particular nothing from ``types``
# (bar the plain-data SimpleNamespace), ``typing``, ``functools``, ``operator``, ``pathlib``, ``os`` or ``sys``, so a
# payload cannot build a CodeType / FunctionType and REDUCE on it.
_SAFE_PAIRS = {
    ("collections", "OrderedDict"), ("collections", "defaultdict"), ("collections", "deque"),
    ("collections", "Counter"), ("argparse", "Namespace"), ("copyreg", "_reconstructor"), ("_codecs", "encode"),
    ("datetime", "datetime"), ("datetime", "date"), ("datetime", "time"), ("datetime", "timedelta"),
    ("datetime", "timezone"), ("decimal", "Decimal"), ("fractions", "Fraction"), ("uuid", "UUID"),
    ("enum", "Enum"), ("enum", "IntEnum"), ("types", "SimpleNamespace"),
    ("torch", "device"), ("torch", "Size"), ("torch", "dtype"), ("torch", "layout"), ("torch", "memory_format"),
    ("torch", "Tensor"), ("torch._tensor", "_rebuild_from_type_v2"), ("torch.nn.parameter", "Parameter"),
    ("torch.serialization", "_get_layout"), ("torch.storage", "UntypedStorage"), ("torch.storage", "TypedStorage"),
    ("torch", "UntypedStorage"), ("torch.distributed.checkpoint.filesystem", "_StorageInfo"),
    ("numpy", "ndarray"), ("numpy", "dtype"), ("numpy.core.multiarray", "_reconstruct"),
    ("numpy._core.multiarray", "_reconstruct"), ("numpy.core.multiarray", "scalar"),
    ("numpy._core.multiarray", "scalar"), ("numpy.random._pickle", "__randomstate_ctor"),
    ("numpy.random._pickle", "__bit_generator_ctor"), ("numpy.random._pickle", "__generator_ctor"),
    ("numpy.random.mtrand", "RandomState"), ("numpy.random._generator", "Generator"),
    ("numpy.random._mt19937", "MT19937"), ("numpy.random._pcg64", "PCG64"),
}
# modules whose *classes* (never functions) may resolve: checkpoint metadata
# and framework config objects.  Metaclasses and callable-wrapping types are
# still refused (see _class_ok).
_CLASS_PREFIXES = ("torch.distributed.checkpoint.metadata", "torch.distributed.checkpoint.planner",
                   "torch.distributed._shard.metadata", "torch.distributed._shard.sharded_tensor.metadata",
                   "torch.distributed._shard.sharding_spec", "numpy.dtypes", "megatron", "deepspeed",
                   "transformers.training_args", "transformers.trainer_utils", "transformers.trainer_callback",
                   "dlrover_wuqiong_amd", "dlrover", "atorch")


def _under(module: str, prefixes) -> bool:
    return any(module == m or module.startswith(m + ".") for m in prefixes)


def _class_ok(obj) -> bool:
    import types as _t

    if not isinstance(obj, type) or issubclass(obj, type):
        return False  # metaclasses build arbitrary classes
    bad = (_t.FunctionType, _t.CodeType, _t.ModuleType, _t.MethodType, _t.BuiltinFunctionType)
    return not issubclass(obj, bad)


class RestrictedUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        if module == "builtins":
            if name not in _SAFE_BUILTINS:
                raise pickle.UnpicklingError(f"refusing to unpickle builtins.{name}")
            return super().find_class(module, name)
        import torch

        if (module, name) in _SAFE_PAIRS:
            return super().find_class(module, name)
        if module == "torch._utils" and name.startswith("_rebuild"):
            return super().find_class(module, name)
        if module == "torch" and (name.endswith("Storage") or isinstance(getattr(torch, name, None),
                                                                          (torch.dtype, torch.layout,
                                                                           torch.memory_format))):
            return super().find_class(module, name)
        if _under(module, _CLASS_PREFIXES):
            obj = super().find_class(module, name)
            if _class_ok(obj):
                return obj
            raise pickle.UnpicklingError(f"refusing to unpickle non-class {module}.{name}")
        raise pickle.UnpicklingError(f"refusing to unpickle {module}.{name}")


def restricted_loads(data: bytes):
    return RestrictedUnpickler(io.BytesIO(data)).load()


class restricted_pickle:  # noqa: N801 - a module-like object for torch.load(pickle_module=...)
    Unpickler = RestrictedUnpickler
    UnpicklingError = pickle.UnpicklingError
    __name__ = "restricted_pickle"

    @staticmethod
    def load(f, **kw):
        return RestrictedUnpickler(f, **kw).load()

    @staticmethod
    def loads(b, **kw):
        return RestrictedUnpickler(io.BytesIO(b), **kw).load()


def safe_torch_load(f, map_location="cpu"):
    """``torch.load`` that tries ``weights_only=True`` first and falls back to
    the allow-listed unpickler (never arbitrary code)."""
    import torch

    pos = f.tell() if hasattr(f, "tell") else None
    try:
        return torch.load(f, map_location=map_location, weights_only=True)
    except Exception:
        if pos is not None:
            f.seek(pos)
        return torch.load(f, map_location=map_location, weights_only=False, pickle_module=restricted_pickle)
