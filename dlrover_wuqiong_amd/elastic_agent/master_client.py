"""Client of the job master (used by agents and training processes).

Parity: reference ``dlrover/python/elastic_agent/master_client.py``
(singleton ``MasterClient`` :50, ``retry_grpc_request`` 10x/5 s :28-47,
rendezvous APIs :302-366, ``report_failures`` :372, ``sync_checkpoint`` :405,
``kv_store_set/get`` :123-131, ``report_heart_beat`` :230).
"""

import functools
import os
import socket
import threading
import time
from typing import Dict, List, Optional, Tuple

from ..common import comm, env_utils
from ..common.constants import JobConstant, NodeEnv, NodeType, RendezvousName
from ..common.log import logger
from ..common.rpc import RpcClient, addr_connected


def retry_rpc(func):
    @functools.wraps(func)
    def wrapper(self, *a, **kw):
        last = None
        for i in range(self.retries):
            try:
                return func(self, *a, **kw)
            except Exception as e:  # grpc.RpcError and friends
                last = e
                if i + 1 < self.retries:
                    time.sleep(self.retry_interval)
        logger.error(f"master RPC {func.__name__} failed after {self.retries} tries: {last}")
        raise last

    return wrapper


class MasterClient:
    _instance: Optional["MasterClient"] = None
    _lock = threading.Lock()

    def __init__(self, master_addr: str, node_id: int, node_type: str = NodeType.WORKER,
                 timeout: float = 10.0, retries: int = JobConstant.MASTER_CLIENT_RETRY, retry_interval: float = 5.0):
        self.master_addr = master_addr
        self.node_id = node_id
        self.node_type = node_type
        self.retries = retries
        self.retry_interval = retry_interval
        self._rpc = RpcClient(master_addr, timeout)
        try:
            self._host = socket.gethostbyname(socket.gethostname())
        except OSError:
            self._host = "127.0.0.1"

    @classmethod
    def singleton_instance(cls, master_addr: str = "", node_id: Optional[int] = None) -> Optional["MasterClient"]:
        with cls._lock:
            if cls._instance is None:
                addr = master_addr or os.getenv(NodeEnv.DLROVER_MASTER_ADDR, "")
                if not addr:
                    return None
                nid = node_id if node_id is not None else env_utils.get_node_id()
                cls._instance = MasterClient(addr, nid)
            return cls._instance

    @classmethod
    def reset(cls):
        with cls._lock:
            if cls._instance is not None:
                cls._instance.close()
            cls._instance = None

    def close(self):
        self._rpc.close()

    # ------------------------------------------------------------ envelope
    def _env(self, data) -> bytes:
        return comm.BaseRequest(node_id=self.node_id, node_type=self.node_type, data=data).serialize()

    @retry_rpc
    def _get(self, data):
        return comm.deserialize_message(self._rpc.get(self._env(data)))

    @retry_rpc
    def _report(self, data) -> comm.Response:
        return comm.deserialize_message(self._rpc.report(self._env(data)))

    # ---------------------------------------------------------- liveness
    def report_heart_beat(self, timestamp: Optional[float] = None):
        return self._report(comm.HeartBeat(timestamp=int(timestamp or time.time())))

    def report_used_resource(self, memory: int, cpu: float, gpu_stats=None):
        return self._report(comm.ResourceStats(memory=memory, cpu=cpu, gpu_stats=list(gpu_stats or [])))

    def report_global_step(self, step: int, timestamp: float, elapsed_per_step: float = 0.0):
        return self._report(comm.GlobalStep(step=step, timestamp=int(timestamp),
                                            elapsed_time_per_step=elapsed_per_step))

    def report_model_info(self, num_params: int, flops: float = 0.0):
        return self._report(comm.ModelInfo(num_params=num_params, flops_per_step=flops))

    def report_failures(self, error_data: str, restart_count: int = -1, level: str = ""):
        return self._report(comm.NodeFailure(error_data=error_data, restart_count=restart_count, level=level))

    def report_node_event(self, event_type: str, message: str = ""):
        return self._report(comm.NodeEvent(event_type=event_type, message=message,
                                           node=comm.NodeMeta(type=self.node_type, id=self.node_id)))

    def report_node_address(self, addr: str = ""):
        return self._report(comm.NodeAddress(type=self.node_type, id=self.node_id, addr=addr or self._host))

    def report_diagnosis(self, data_cls: str, content: str):
        return self._report(comm.DiagnosisReport(data_cls=data_cls, data_content=content, node_id=self.node_id,
                                                 timestamp=time.time()))

    # -------------------------------------------------------- rendezvous
    def report_rdzv_params(self, min_nodes: int, max_nodes: int, waiting_timeout: float, node_unit: int = 1,
                           join_timeout: int = 600):
        return self._report(comm.RendezvousParams(min_nodes=min_nodes, max_nodes=max_nodes,
                                                  waiting_timeout=int(waiting_timeout), node_unit=node_unit,
                                                  join_timeout=join_timeout))

    def join_rendezvous(self, node_rank: int, local_world_size: int,
                        rdzv_name: str = RendezvousName.ELASTIC_TRAINING, node_ip: str = "") -> int:
        r = self._get(comm.JoinRendezvousRequest(node_id=self.node_id, node_rank=node_rank,
                                                 local_world_size=local_world_size, rdzv_name=rdzv_name,
                                                 node_ip=node_ip or self._host))
        return r.round

    def get_comm_world(self, rdzv_name: str, node_rank: int) -> Tuple[int, int, Dict[int, int]]:
        r = self._get(comm.CommWorldRequest(node_id=node_rank, rdzv_name=rdzv_name))
        return r.round, r.group, dict(r.world)

    def num_nodes_waiting(self, rdzv_name: str = RendezvousName.ELASTIC_TRAINING) -> int:
        try:
            return self._get(comm.WaitingNodeNumRequest(rdzv_name=rdzv_name)).waiting_num
        except Exception:
            return 0

    def network_check_success(self) -> Tuple[bool, List[int], str]:
        r = self._get(comm.NetworkReadyRequest())
        return (not r.nodes and not r.reason), list(r.nodes), r.reason

    def check_straggler(self) -> Tuple[List[int], str]:
        r = self._get(comm.StragglerExistRequest())
        return list(r.nodes), r.reason

    def report_network_check_status(self, node_rank: int, status: str, elapsed_time: float):
        return self._report(comm.NetworkStatus(rank=node_rank, status=status, elapsed_time=elapsed_time))

    def sync_checkpoint(self, step: int) -> bool:
        return self._report(comm.NodeCheckpointState(step=step)).success

    # ------------------------------------------------------------- kv
    def kv_store_set(self, key: str, value: bytes):
        return self._report(comm.KeyValuePair(key=key, value=value))

    def kv_store_get(self, key: str) -> bytes:
        return self._get(comm.KeyValuePair(key=key)).value

    def kv_store_add(self, key: str, amount: int) -> int:
        return int(self._report(comm.KeyValueAdd(key=key, amount=amount)).reason)

    # -------------------------------------------------------------- sync
    def join_sync(self, name: str) -> bool:
        return self._report(comm.SyncJoin(sync_name=name)).success

    def sync_finished(self, name: str) -> bool:
        return self._get(comm.SyncJoin(sync_name=name)).success

    def barrier(self, name: str, notify: bool = False) -> bool:
        if notify:
            return self._report(comm.SyncBarrier(barrier_name=name, notify=True)).success
        return self._get(comm.SyncBarrier(barrier_name=name)).success

    # ----------------------------------------------------------- shards
    def report_dataset_shard_params(self, batch_size: int, num_epochs: int, dataset_size: int, shuffle: bool,
                                    num_minibatches_per_shard: int, dataset_name: str, task_type: int = 1,
                                    storage_type: str = "table"):
        return self._report(comm.DatasetShardParams(batch_size=batch_size, num_epochs=num_epochs,
                                                    dataset_size=dataset_size, shuffle=shuffle,
                                                    num_minibatches_per_shard=num_minibatches_per_shard,
                                                    dataset_name=dataset_name, task_type=task_type,
                                                    storage_type=storage_type))

    def get_task(self, dataset_name: str) -> comm.Task:
        return self._get(comm.TaskRequest(dataset_name=dataset_name))

    def report_task_result(self, dataset_name: str, task_id: int, err_msg: str = ""):
        return self._report(comm.TaskResult(dataset_name=dataset_name, task_id=task_id, err_message=err_msg))

    def get_shard_checkpoint(self, dataset_name: str) -> str:
        return self._get(comm.ShardCheckpointRequest(dataset_name=dataset_name)).content

    def report_shard_checkpoint(self, content: str) -> bool:
        return self._report(comm.ShardCheckpoint(content=content)).success

    # ---------------------------------------------------------- configs
    def get_running_nodes(self):
        return self._get(comm.RunningNodesRequest()).nodes

    def report_paral_config(self, config: comm.ParallelConfig):
        return self._report(config)

    def get_paral_config(self) -> comm.ParallelConfig:
        return self._get(comm.ParallelConfigRequest())

    def need_to_restart_training(self) -> bool:
        return self._get(comm.CheckHardwareResetRequest()).success

    # ------------------------------------------------ elastic PS versions
    def get_cluster_version(self, version_type: str, task_type: str, task_id: int) -> int:
        return int(self._get(comm.ClusterVersionRequest(task_type=task_type, task_id=task_id,
                                                        version_type=version_type)).version)

    def update_cluster_version(self, version_type: str, version: int, task_type: str, task_id: int):
        return self._report(comm.ClusterVersion(task_type=task_type, task_id=task_id, version_type=version_type,
                                                version=version))

    def query_ps_nodes(self):
        """(ps NodeMeta list, all new PS running, some PS failed)."""
        r = self._get(comm.PsNodesRequest())
        return r.nodes, r.new_ps_ready, r.ps_failure

    def get_elastic_run_config(self) -> Dict[str, str]:
        return dict(self._get(comm.ElasticRunConfigRequest()).configs)


def build_master_client(master_addr: str = "", timeout: float = 10.0) -> Optional[MasterClient]:
    addr = master_addr or os.getenv(NodeEnv.DLROVER_MASTER_ADDR, "")
    if not addr:
        return None
    if not addr_connected(addr, timeout=2.0):
        logger.warning(f"master {addr} is not reachable")
    return MasterClient(addr, env_utils.get_node_id(), timeout=timeout)
