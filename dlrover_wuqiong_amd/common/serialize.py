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
                  "str", "bool", "slice", "range", "object", "NoneType", "Ellipsis"}
_CLASS_MODULES = ("collections", "torch", "numpy", "argparse", "enum", "datetime", "decimal", "fractions",
                  "megatron", "deepspeed", "transformers", "dlrover_wuqiong_amd", "dlrover", "atorch", "pathlib",
                  "types", "typing", "uuid")
_SAFE_FUNCS = {("copyreg", "_reconstructor"), ("_codecs", "encode"), ("torch._tensor", "_rebuild_from_type_v2"),
               ("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
               ("numpy.core.multiarray", "scalar"), ("numpy._core.multiarray", "scalar"),
               ("numpy.random._pickle", "__randomstate_ctor"), ("numpy.random._pickle", "__bit_generator_ctor"),
               ("numpy.random._pickle", "__generator_ctor"), ("torch", "device"), ("torch", "Size"),
               ("collections", "OrderedDict"), ("torch.serialization", "_get_layout")}


def _module_ok(module: str) -> bool:
    return module in ("builtins", "copyreg", "_codecs") or any(
        module == m or module.startswith(m + ".") for m in _CLASS_MODULES)


class RestrictedUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        if not _module_ok(module):
            raise pickle.UnpicklingError(f"refusing to unpickle {module}.{name}")
        if module == "builtins" and name not in _SAFE_BUILTINS:
            raise pickle.UnpicklingError(f"refusing to unpickle builtins.{name}")
        obj = super().find_class(module, name)
        if isinstance(obj, type):
            return obj
        if (module, name) in _SAFE_FUNCS or (module == "torch._utils" and name.startswith("_rebuild")):
            return obj
        import torch

        if isinstance(obj, (torch.dtype, torch.layout, torch.memory_format)):
            return obj
        raise pickle.UnpicklingError(f"refusing to unpickle callable {module}.{name}")


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
