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
