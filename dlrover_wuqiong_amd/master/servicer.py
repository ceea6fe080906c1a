"""The master's RPC servicer: dispatch ``get``/``report`` by message type.

Parity: reference ``dlrover/python/master/servicer.py`` (``MasterServicer``
:71-96, ``get`` :98-138 with 14 request kinds, ``report`` :296-356 with 24
kinds, rendezvous handlers :243-276, ``_report_failure`` :551,
``_sync_checkpoint`` :594, ``create_master_service`` :630-668).
"""

import time
from typing import Dict, Optional

from ..common import comm
from ..common.constants import NodeStatus, NodeType, RendezvousName
from ..common.log import logger
from .job_manager import JobManager
from .rendezvous import RendezvousManager
from .services import (DiagnosisManager, ElasticPsService, ErrorMonitor, KVStoreService, SimpleStrategyGenerator,
                       SpeedMonitor, SyncService)
from .shard import TaskManager


class MasterServicer:
    def __init__(self, job_manager: JobManager, task_manager: TaskManager, speed_monitor: SpeedMonitor,
                 rdzv_managers: Dict[str, RendezvousManager], kv_store: KVStoreService,
                 sync_service: SyncService, error_monitor: Optional[ErrorMonitor] = None,
                 diagnosis: Optional[DiagnosisManager] = None, run_configs: Optional[Dict[str, str]] = None,
                 elastic_ps: Optional[ElasticPsService] = None):
        self.job_manager = job_manager
        self.task_manager = task_manager
        self.speed_monitor = speed_monitor
        self.rdzv = rdzv_managers
        self.kv = kv_store
        self.sync = sync_service
        self.errors = error_monitor or ErrorMonitor()
        self.diagnosis = diagnosis or DiagnosisManager(speed_monitor)
        self.strategy = SimpleStrategyGenerator()
        self.run_configs = run_configs or {}
        self.elastic_ps = elastic_ps or ElasticPsService()
        self._paral_configs: Dict[int, comm.ParallelConfig] = {}
        self._start_training_time = 0.0

    # ------------------------------------------------------------ transport
    def get_bytes(self, data: bytes) -> bytes:
        req = comm.deserialize_message(data)
        try:
            resp = self.get(req)
        except Exception as e:  # never kill the server thread
            logger.error(f"get({type(req.data).__name__}) failed: {e}", exc_info=True)
            resp = comm.Response(success=False, reason=str(e))
        return (resp or comm.Empty()).serialize()

    def report_bytes(self, data: bytes) -> bytes:
        req = comm.deserialize_message(data)
        try:
            resp = self.report(req)
        except Exception as e:
            logger.error(f"report({type(req.data).__name__}) failed: {e}", exc_info=True)
            resp = comm.Response(success=False, reason=str(e))
        return resp.serialize()

    # ------------------------------------------------------------------ get
    def get(self, req: comm.BaseRequest):
        m = req.data
        nid, ntype = req.node_id, req.node_type
        if isinstance(m, comm.TaskRequest):
            t = self.task_manager.get_dataset_task(nid, m.dataset_name)
            if t is None:
                return comm.Task(task_id=-1, type=0)
            s = t.shard
            return comm.Task(task_id=t.task_id, type=t.task_type,
                             shard=comm.Shard(name=s.name, start=s.start, end=s.end, indices=list(s.record_indices)))
        if isinstance(m, comm.ShardCheckpointRequest):
            return comm.ShardCheckpoint(content=self.task_manager.get_dataset_checkpoint(m.dataset_name))
        if isinstance(m, comm.RunningNodesRequest):
            return comm.RunningNodes(nodes=[comm.NodeMeta(type=n.type, id=n.id, rank=n.rank_index,
                                                          addr=n.host_addr, status=n.status)
                                            for n in self.job_manager.get_running_nodes()])
        if isinstance(m, comm.JoinRendezvousRequest):
            return self._join_rendezvous(m, nid)
        if isinstance(m, comm.WaitingNodeNumRequest):
            mgr = self.rdzv[m.rdzv_name or RendezvousName.ELASTIC_TRAINING]
            return comm.RendezvousState(waiting_num=mgr.num_nodes_waiting())
        if isinstance(m, comm.CommWorldRequest):
            mgr = self.rdzv[m.rdzv_name or RendezvousName.ELASTIC_TRAINING]
            rnd, group, world = mgr.get_comm_world(m.node_id)
            return comm.RendezvousState(world={r: meta.process_num for r, meta in world.items()}, round=rnd,
                                        group=group)
        if isinstance(m, comm.NetworkReadyRequest):
            mgr = self.rdzv[RendezvousName.NETWORK_CHECK]
            nodes, reason = mgr.check_fault_node()
            return comm.NetworkCheckResult(nodes=nodes, reason=reason)
        if isinstance(m, comm.StragglerExistRequest):
            mgr = self.rdzv[RendezvousName.NETWORK_CHECK]
            nodes, reason = mgr.get_straggler()
            return comm.NetworkCheckResult(nodes=nodes, reason=reason)
        if isinstance(m, comm.KeyValuePair):
            return comm.KeyValuePair(key=m.key, value=self.kv.get(m.key))
        if isinstance(m, comm.ParallelConfigRequest):
            return self._paral_configs.get(nid, comm.ParallelConfig())
        if isinstance(m, comm.TrainingStatusRequest):
            return comm.TrainingStatus(status=1 if self.task_manager.training_started() else 3)
        if isinstance(m, comm.CheckHardwareResetRequest):
            n = self.job_manager.get_node(nid)
            return comm.Response(success=bool(n and n.restart_training))
        if isinstance(m, comm.SyncJoin):
            return comm.Response(success=self.sync.sync_finished(m.sync_name))
        if isinstance(m, comm.SyncBarrier):
            return comm.Response(success=self.sync.barrier(m.barrier_name))
        if isinstance(m, comm.ElasticRunConfigRequest):
            return comm.ElasticRunConfig(configs=dict(self.run_configs))
        if isinstance(m, comm.GlobalStep):
            return comm.GlobalStep(step=self.speed_monitor.completed_global_step,
                                   timestamp=int(self.speed_monitor.last_step_time()))
        if isinstance(m, comm.ClusterVersionRequest):
            return comm.ClusterVersion(task_type=m.task_type, task_id=m.task_id, version_type=m.version_type,
                                       version=self.elastic_ps.get_version(m.task_type, m.version_type, m.task_id))
        if isinstance(m, comm.PsNodesRequest):
            return self._ps_nodes()
        return comm.Response(success=False, reason=f"unknown get request {type(m).__name__}")

    def _ps_nodes(self) -> comm.PsNodes:
        """The PS cluster workers should connect to (reference
        ``servicer.py:_query_ps_nodes``): alive PS by rank, whether all of
        them are running, and whether one has failed."""
        ps_nodes = sorted(getattr(self.job_manager, "job_nodes", {}).get(NodeType.PS, {}).values(), key=lambda n: n.rank_index)
        alive = [n for n in ps_nodes if not n.is_released and n.status not in (NodeStatus.FAILED, NodeStatus.DELETED)]
        metas = [comm.NodeMeta(type=NodeType.PS, id=n.id, rank=n.rank_index, addr=n.host_addr, status=n.status)
                 for n in alive]
        ready = bool(alive) and all(n.status == NodeStatus.RUNNING for n in alive)
        failed = any(n.status == NodeStatus.FAILED for n in ps_nodes)
        return comm.PsNodes(nodes=metas, new_ps_ready=ready, ps_failure=failed)

    def _join_rendezvous(self, m: comm.JoinRendezvousRequest, nid: int):
        name = m.rdzv_name or RendezvousName.ELASTIC_TRAINING
        mgr = self.rdzv[name]
        node_rank = m.node_rank if m.node_rank >= 0 else m.node_id
        self.job_manager.add_node(m.node_id, NodeType.WORKER, m.node_ip)
        for r in self.rdzv.values():
            r.add_alive_node(node_rank)
        rnd = mgr.join_rendezvous(node_rank, m.local_world_size, m.node_ip)
        if name == RendezvousName.NETWORK_CHECK:
            # nodes re-checking the network leave the training waiting list
            self.rdzv[RendezvousName.ELASTIC_TRAINING].clear_waiting_nodes()
        return comm.RendezvousState(round=rnd)

    # --------------------------------------------------------------- report
    def report(self, req: comm.BaseRequest) -> comm.Response:
        m = req.data
        nid, ntype = req.node_id, req.node_type
        ok = True
        if isinstance(m, comm.DatasetShardParams):
            self.task_manager.new_dataset(m.batch_size, m.dataset_size, m.dataset_name, m.num_epochs, m.shuffle,
                                          m.num_minibatches_per_shard, m.task_type or 1, m.storage_type or "table")
        elif isinstance(m, comm.TaskResult):
            self.task_manager.report_dataset_task(m.dataset_name, m.task_id, not m.err_message)
        elif isinstance(m, comm.ShardCheckpoint):
            ok = self.task_manager.restore_dataset_from_checkpoint(m.content)
        elif isinstance(m, comm.ResourceStats):
            self.job_manager.update_node_resource_usage(ntype, nid, m.cpu, m.memory, m.gpu_stats)
        elif isinstance(m, comm.ModelInfo):
            pass
        elif isinstance(m, comm.GlobalStep):
            self.speed_monitor.collect_global_step(m.step, m.timestamp or time.time())
            self.speed_monitor.add_running_worker(nid)
        elif isinstance(m, comm.HeartBeat):
            self.job_manager.collect_node_heart_beat(ntype, nid, m.timestamp)
        elif isinstance(m, comm.NodeFailure):
            self.errors.process_error(nid, m.restart_count, m.error_data, m.level)
            self.job_manager.handle_training_failure(ntype, nid, m.restart_count, m.error_data, m.level)
            self.task_manager.recover_tasks(nid)
        elif isinstance(m, comm.NetworkStatus):
            self.rdzv[RendezvousName.NETWORK_CHECK].report_network_check_result(
                m.rank, m.status == NodeStatus.SUCCEEDED, m.elapsed_time)
        elif isinstance(m, comm.KeyValuePair):
            self.kv.set(m.key, m.value)
        elif isinstance(m, comm.KeyValueAdd):
            v = self.kv.add(m.key, m.amount)
            return comm.Response(success=True, reason=str(v))
        elif isinstance(m, comm.SyncJoin):
            ok = self.sync.join_sync(m.sync_name, nid)
        elif isinstance(m, comm.SyncFinish):
            ok = self.sync.sync_finished(m.sync_name)
        elif isinstance(m, comm.SyncBarrier):
            ok = self.sync.notify_barrier(m.barrier_name) if m.notify else self.sync.barrier(m.barrier_name)
        elif isinstance(m, comm.NodeAddress):
            self.job_manager.add_node(m.id, m.type or NodeType.WORKER, m.addr)
        elif isinstance(m, comm.NodeEvent):
            node = m.node
            if node is not None and m.event_type in (NodeStatus.SUCCEEDED, NodeStatus.FAILED, NodeStatus.DELETED):
                self.job_manager.update_node_status(node.id, m.event_type, m.message)
                if m.event_type != NodeStatus.SUCCEEDED:
                    self.task_manager.recover_tasks(node.id)
                    for r in self.rdzv.values():
                        r.remove_alive_node(node.id)
        elif isinstance(m, comm.ParallelConfig):
            self._paral_configs[nid] = m
            self.job_manager.update_node_paral_config(ntype, nid, m)
        elif isinstance(m, comm.NodeCheckpointState):
            ok = self.rdzv[RendezvousName.ELASTIC_TRAINING].sync_ckpt_nodes(nid, m.step)
        elif isinstance(m, comm.DiagnosisReport):
            self.diagnosis.collect(m.node_id or nid, m.data_cls, m.data_content, m.timestamp or None)
        elif isinstance(m, comm.ClusterVersion):
            ok = self.elastic_ps.update_version(m.task_type, m.version_type, m.task_id, m.version)
        elif isinstance(m, comm.RendezvousParams):
            for r in self.rdzv.values():
                r.update_rdzv_params(m.min_nodes, m.max_nodes, m.waiting_timeout, m.node_unit)
        else:
            return comm.Response(success=False, reason=f"unknown report {type(m).__name__}")
        return comm.Response(success=bool(ok))
