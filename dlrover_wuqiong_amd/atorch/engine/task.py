"""Tasks the acceleration engine hands to training processes, and the wire
format of strategies.

A strategy on the wire is a list of ``[name, config, tunable]``; configs are
JSON with two tagged forms (``{"__dtype__": "bfloat16"}`` for torch dtypes,
``{"__tuple__": [...]}`` for tuples), so the service needs no pickling in
either direction (the reference ships pickled configs through protobuf bytes
fields).

Parity: reference ``atorch/atorch/auto/engine/task.py`` (``TaskType``,
``TaskProcessMode``, ``TaskStatus``, ``Task``).
"""

import json
from dataclasses import dataclass, field
from typing import Any, List, Optional

import torch


class TaskType:
    ANALYSE = "ANALYSE"
    SETUP_PARALLEL_GROUP = "SETUP_PARALLEL_GROUP"
    TUNE = "TUNE"
    DRYRUN = "DRYRUN"
    FINISH = "FINISH"
    FAIL = "FAIL"
    WAIT = "WAIT"


class ProcessMode:
    """ONE_PROCESS: any single idle process runs it.  ALL_PROCESS: every
    process runs it together (collectives inside), handed out only once all
    processes are idle."""

    ONE = "ONE_PROCESS"
    ALL = "ALL_PROCESS"


class TaskStatus:
    PENDING = "PENDING"
    ASSIGNING = "ASSIGNING"
    RUNNING = "RUNNING"
    SUCCEEDED = "SUCCEEDED"
    FAILED = "FAILED"


@dataclass
class Task:
    task_type: str
    info: Any = None                 # strategy / analyse method names / parallel mode
    task_id: int = -1
    strategy_id: int = -1
    process_mode: str = ProcessMode.ONE
    time_limit: Optional[float] = None
    status: str = TaskStatus.PENDING
    result: Any = None
    assigned: List[int] = field(default_factory=list)

    def wire(self) -> dict:
        return {"task_id": self.task_id, "task_type": self.task_type, "process_mode": self.process_mode,
                "time_limit": self.time_limit, "info": encode(self.info)}


def encode(obj):
    """JSON-safe form of strategy configs (dtypes and tuples tagged)."""
    if isinstance(obj, torch.dtype):
        return {"__dtype__": str(obj).split(".", 1)[1]}
    if isinstance(obj, tuple):
        return {"__tuple__": [encode(x) for x in obj]}
    if isinstance(obj, list):
        return [encode(x) for x in obj]
    if isinstance(obj, dict):
        return {str(k): encode(v) for k, v in obj.items()}
    if obj is None or isinstance(obj, (bool, int, float, str)):
        return obj
    raise TypeError(f"engine strategies carry JSON, dtypes and tuples only (got {type(obj).__name__})")


def decode(obj):
    if isinstance(obj, dict):
        if "__dtype__" in obj:
            dt = getattr(torch, obj["__dtype__"])
            if not isinstance(dt, torch.dtype):
                raise ValueError(f"not a dtype: {obj}")
            return dt
        if "__tuple__" in obj:
            return tuple(decode(x) for x in obj["__tuple__"])
        return {k: decode(v) for k, v in obj.items()}
    if isinstance(obj, list):
        return [decode(x) for x in obj]
    return obj


def dumps(obj) -> bytes:
    return json.dumps(obj).encode()


def loads(b: bytes):
    return json.loads(b.decode()) if b else None
