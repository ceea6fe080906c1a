"""Control-plane messages between agents/workers and the job master.

Parity: reference ``dlrover/python/common/grpc.py:135-468`` (the ~40 message
dataclasses carried by the generic ``Master.report`` / ``Master.get`` RPCs).

Difference: messages travel as tagged JSON, not pickle - the master never
unpickles bytes from the network.  Nested messages, ``bytes`` and dicts with
non-string keys round-trip exactly.
"""

import base64
import json
from dataclasses import dataclass, field, fields, is_dataclass
from typing import Any, Dict, List, Type

_REGISTRY: Dict[str, Type["Message"]] = {}


def message(cls):
    """Class decorator: dataclass + registration under its class name."""
    cls = dataclass(cls)
    _REGISTRY[cls.__name__] = cls
    return cls


def _enc(v: Any) -> Any:
    if isinstance(v, Message):
        return {"__t": type(v).__name__, **{f.name: _enc(getattr(v, f.name)) for f in fields(v)}}
    if isinstance(v, (bytes, bytearray, memoryview)):
        return {"__b": base64.b64encode(bytes(v)).decode()}
    if isinstance(v, dict):
        return {"__d": [[_enc(k), _enc(x)] for k, x in v.items()]}
    if isinstance(v, (list, tuple)):
        return [_enc(x) for x in v]
    return v


def _dec(v: Any) -> Any:
    if isinstance(v, dict):
        if "__t" in v:
            cls = _REGISTRY[v["__t"]]
            kw = {k: _dec(x) for k, x in v.items() if k != "__t"}
            return cls(**kw)
        if "__b" in v:
            return base64.b64decode(v["__b"])
        if "__d" in v:
            return {_dec(k): _dec(x) for k, x in v["__d"]}
        return {k: _dec(x) for k, x in v.items()}
    if isinstance(v, list):
        return [_dec(x) for x in v]
    return v


class Message:
    def serialize(self) -> bytes:
        return json.dumps(_enc(self), separators=(",", ":")).encode()


def deserialize_message(data: bytes):
    if not data:
        return None
    return _dec(json.loads(data.decode()))


# ----------------------------------------------------------------- messages
@message
class Empty(Message):
    pass


@message
class Response(Message):
    success: bool = False
    reason: str = ""


@message
class BaseRequest(Message):
    node_id: int = 0
    node_type: str = "worker"
    data: Any = None


@message
class TaskRequest(Message):
    dataset_name: str = ""


@message
class Shard(Message):
    name: str = ""
    start: int = 0
    end: int = 0
    indices: List[int] = field(default_factory=list)


@message
class Task(Message):
    task_id: int = -1
    shard: Any = None
    type: int = 0
    extended_config: Dict[str, str] = field(default_factory=dict)


@message
class TaskResult(Message):
    dataset_name: str = ""
    task_id: int = 0
    err_message: str = ""
    exec_counters: Dict[str, int] = field(default_factory=dict)


@message
class DatasetShardParams(Message):
    batch_size: int = 0
    num_epochs: int = 0
    dataset_size: int = 0
    shuffle: bool = False
    num_minibatches_per_shard: int = 0
    dataset_name: str = ""
    task_type: int = 0
    storage_type: str = ""


@message
class ShardCheckpointRequest(Message):
    dataset_name: str = ""


@message
class ShardCheckpoint(Message):
    content: str = ""


@message
class GPUStats(Message):
    index: int = 0
    total_memory_mb: int = 0
    used_memory_mb: int = 0
    gpu_utilization: float = 0.0


@message
class ResourceStats(Message):
    memory: int = 0
    cpu: float = 0.0
    gpu_stats: List[Any] = field(default_factory=list)


@message
class ModelInfo(Message):
    num_params: int = 0
    flops_per_step: float = 0.0
    activation_memory: int = 0


@message
class GlobalStep(Message):
    timestamp: int = 0
    step: int = 0
    elapsed_time_per_step: float = 0.0


@message
class HeartBeat(Message):
    timestamp: int = 0


@message
class SyncJoin(Message):
    sync_name: str = ""


@message
class SyncFinish(Message):
    sync_name: str = ""


@message
class SyncBarrier(Message):
    barrier_name: str = ""
    notify: bool = False


@message
class NodeMeta(Message):
    type: str = ""
    addr: str = ""
    memory: int = 0
    cpu: float = 0.0
    gpu: int = 0
    gpu_type: str = ""
    id: int = 0
    rank: int = 0
    status: str = ""


@message
class NodeAddress(NodeMeta):
    pass


@message
class NetworkStatus(NodeMeta):
    elapsed_time: float = 0.0


@message
class NodeEvent(Message):
    event_type: str = ""
    message: str = ""
    node: Any = None


@message
class NodeFailure(Message):
    error_data: str = ""
    restart_count: int = 0
    level: str = ""


@message
class RendezvousParams(Message):
    min_nodes: int = 0
    max_nodes: int = 0
    waiting_timeout: int = 0
    node_unit: int = 1
    join_timeout: int = 600


@message
class RendezvousRequest(Message):
    node_id: int = 0
    local_world_size: int = 0
    rdzv_name: str = ""


@message
class CommWorldRequest(RendezvousRequest):
    pass


@message
class JoinRendezvousRequest(RendezvousRequest):
    node_ip: str = ""
    node_rank: int = -1


@message
class WaitingNodeNumRequest(RendezvousRequest):
    pass


@message
class NetworkReadyRequest(Message):
    pass


@message
class StragglerExistRequest(Message):
    pass


@message
class NetworkCheckResult(Message):
    nodes: List[int] = field(default_factory=list)
    reason: str = ""


@message
class RendezvousState(Message):
    world: Dict[int, int] = field(default_factory=dict)
    waiting_num: int = 0
    round: int = 0
    group: int = 0


@message
class RunningNodesRequest(Message):
    pass


@message
class RunningNodes(Message):
    nodes: List[Any] = field(default_factory=list)


@message
class TrainingStatusRequest(Message):
    pass


@message
class TrainingStatus(Message):
    status: int = 0


@message
class KeyValuePair(Message):
    key: str = ""
    value: bytes = b""


@message
class KeyValueAdd(Message):
    key: str = ""
    amount: int = 0


@message
class DataLoaderConfig(Message):
    version: int = 0
    dataloader_name: str = ""
    last_batch_size: int = 0
    batch_size: int = 0
    num_workers: int = 0
    pin_memory: int = 0


@message
class OptimizerConfig(Message):
    version: int = 0
    optimizer_name: str = ""
    learning_rate: float = 0.0
    weight_decay: float = 0.0


@message
class ParallelConfigRequest(Message):
    pass


@message
class ParallelConfig(Message):
    dataloader: Any = None
    optimizer: Any = None
    restart: bool = False


@message
class CheckHardwareResetRequest(Message):
    pass


@message
class NodeCheckpointState(Message):
    step: int = 0


@message
class DiagnosisReport(Message):
    data_cls: str = ""
    data_content: str = ""
    node_id: int = 0
    timestamp: float = 0.0


@message
class ElasticRunConfigRequest(Message):
    pass


@message
class ElasticRunConfig(Message):
    configs: Dict[str, str] = field(default_factory=dict)


@message
class ClusterVersionRequest(Message):
    task_type: str = ""
    task_id: int = 0
    version_type: str = ""


@message
class ClusterVersion(Message):
    task_type: str = ""
    task_id: int = 0
    version_type: str = ""
    version: int = 0


@message
class PsNodesRequest(Message):
    pass


@message
class PsNodes(Message):
    nodes: List[Any] = field(default_factory=list)
    new_ps_ready: bool = False
    ps_failure: bool = False


def is_message(x) -> bool:
    return isinstance(x, Message) and is_dataclass(x)
