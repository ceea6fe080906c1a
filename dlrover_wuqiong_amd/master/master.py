"""The job master process.

Parity: reference ``dlrover/python/master/local_master.py:38-118``
(``LocalJobMaster``), ``dist_master.py:81-304`` (``DistributedJobMaster``,
main loop every 30 s checking exit / hang / completion) and ``main.py``.
"""

import threading
import time
from typing import Dict, Optional

from ..common.constants import JobExitReason, RendezvousName
from ..common.log import logger
from ..common.rpc import RpcServer, find_free_port
from .job_manager import JobManager, NodeLauncher
from .rendezvous import ElasticTrainingRendezvousManager, NetworkCheckRendezvousManager
from .servicer import MasterServicer
from .services import DiagnosisManager, ErrorMonitor, KVStoreService, SpeedMonitor, SyncService
from .shard import TaskManager


class JobMaster:
    def __init__(self, port: int = 0, node_num: int = 1, launcher: Optional[NodeLauncher] = None,
                 loop_interval: float = 30.0, hang_secs: float = 1800.0,
                 run_configs: Optional[Dict[str, str]] = None, max_relaunch_count: int = 3,
                 job_manager: Optional[JobManager] = None, speed_monitor: Optional[SpeedMonitor] = None):
        self.port = port or find_free_port()
        self.node_num = node_num
        self.job_manager = job_manager or JobManager(node_num, launcher, max_relaunch_count=max_relaunch_count)
        self.task_manager = TaskManager()
        self.speed_monitor = speed_monitor or SpeedMonitor()
        self.rdzv_managers = {
            RendezvousName.ELASTIC_TRAINING: ElasticTrainingRendezvousManager(),
            RendezvousName.NETWORK_CHECK: NetworkCheckRendezvousManager(),
        }
        self.kv_store = KVStoreService()
        self.sync_service = SyncService(self.job_manager)
        self.error_monitor = ErrorMonitor()
        self.diagnosis = DiagnosisManager(self.speed_monitor, hang_secs=hang_secs)
        self.servicer = MasterServicer(self.job_manager, self.task_manager, self.speed_monitor, self.rdzv_managers,
                                       self.kv_store, self.sync_service, self.error_monitor, self.diagnosis,
                                       run_configs)
        self.server = RpcServer(self.port, self.servicer.report_bytes, self.servicer.get_bytes)
        self.port = self.server.port
        self._loop_interval = loop_interval
        self._stop = threading.Event()
        self.exit_reason = ""
        self._thread: Optional[threading.Thread] = None

    @property
    def addr(self) -> str:
        return f"127.0.0.1:{self.port}"

    def prepare(self):
        self.server.start()
        logger.info(f"job master serving on port {self.port}")

    def run(self) -> int:
        """Main loop: heartbeats, shard timeouts, hang detection, completion."""
        while not self._stop.wait(self._loop_interval):
            self.job_manager.monitor_heartbeats()
            self.task_manager.reassign_timeout_tasks()
            if self.diagnosis.check_training_hang():
                logger.error("training hang detected (no global step progress)")
                self.exit_reason = JobExitReason.HANG_ERROR
            pending_check = getattr(self.job_manager, "is_job_pending_too_long", None)
            if pending_check is not None and pending_check():
                self.exit_reason = JobExitReason.PENDING_TIMEOUT
                self.metric_collector.collect_job_exit_reason(self.exit_reason)
                return 1
            if self.job_manager.all_workers_exited():
                if self.job_manager.all_workers_failed():
                    self.exit_reason = JobExitReason.WORKER_ERROR
                    logger.error("all workers failed")
                    return 1
                self.exit_reason = JobExitReason.SUCCEEDED
                logger.info("all workers exited: job done")
                return 0
            if self.task_manager.finished():
                logger.info("all data shards consumed")
        return 0

    def start_background(self):
        self.prepare()
        self._thread = threading.Thread(target=self.run, daemon=True, name="dwamd-master-loop")
        self._thread.start()
        return self

    def stop(self):
        self._stop.set()
        self.job_manager.stop()
        self.server.stop()


LocalJobMaster = JobMaster


class DistributedJobMaster(JobMaster):
    """Master that also owns the nodes: launches them through a ``Scaler``,
    watches them, relaunches failed ones (same rank) and stops the job on
    unrecoverable failures (reference ``dist_master.py:81-304``)."""

    def __init__(self, job_resource, scaler_factory, watcher_factory=None, port: int = 0,
                 loop_interval: float = 5.0, hang_secs: float = 1800.0, max_relaunch_count: int = 3,
                 heartbeat_timeout: float = 300.0, node_unit: int = 1, auto_worker: bool = False,
                 stats_path: str = "", optimize_mode: str = "single-job", brain_addr: str = "",
                 job_name: str = "local", max_workers: int = 0):
        from .dist_job_manager import DistributedJobManager
        from .event_callback import AllReduceNodeHandlingCallback, PsClusterVersionCallback, TaskRescheduleCallback
        from .stats import JobMetricCollector, LocalStatsReporter
        from .watcher import ProcessWatcher

        port = port or find_free_port()
        self.scaler = scaler_factory(f"127.0.0.1:{port}")
        watcher = watcher_factory(self.scaler) if watcher_factory else ProcessWatcher(self.scaler)
        speed = SpeedMonitor()
        from .resource_optimizer import ResourceLimits, new_resource_optimizer

        # single-job: the Brain algorithms over this master's metrics; cluster: the Brain service
        self.resource_optimizer = new_resource_optimizer(
            optimize_mode, f"{job_name}-{port}", job_name,
            ResourceLimits(max_workers=max_workers, node_unit=node_unit), brain_addr=brain_addr or None)
        jm = DistributedJobManager(job_resource, self.scaler, watcher, max_relaunch_count=max_relaunch_count,
                                   heartbeat_timeout=heartbeat_timeout, speed_monitor=speed, node_unit=node_unit,
                                   auto_worker=auto_worker, resource_optimizer=self.resource_optimizer,
                                   max_workers=max_workers)
        super().__init__(port=port, node_num=job_resource.worker_num, loop_interval=loop_interval,
                         hang_secs=hang_secs, max_relaunch_count=max_relaunch_count, job_manager=jm,
                         speed_monitor=speed)
        self.rdzv_managers[RendezvousName.ELASTIC_TRAINING].update_rdzv_params(
            job_resource.worker_num, job_resource.worker_num, 60, node_unit)
        jm.add_node_event_callback(TaskRescheduleCallback(self.task_manager))
        jm.add_node_event_callback(AllReduceNodeHandlingCallback(self))
        jm.add_node_event_callback(PsClusterVersionCallback(self.servicer.elastic_ps))
        self.metric_collector = JobMetricCollector(jm, speed, LocalStatsReporter(stats_path))
        self._stop_request = None

    def request_stop(self, success: bool, reason: str, msg: str = ""):
        logger.info(f"job stop requested: success={success} reason={reason} {msg}")
        self._stop_request = (success, reason, msg)
        self._stop.set()

    def prepare(self):
        super().prepare()
        self.job_manager.start()

    def run(self) -> int:
        while not self._stop.wait(self._loop_interval):
            self.task_manager.reassign_timeout_tasks()
            self.metric_collector.collect_runtime_stats()
            if self.diagnosis.check_training_hang():
                logger.error("training hang detected (no global step progress)")
                self.exit_reason = JobExitReason.HANG_ERROR
            pending_check = getattr(self.job_manager, "is_job_pending_too_long", None)
            if pending_check is not None and pending_check():
                self.exit_reason = JobExitReason.PENDING_TIMEOUT
                self.metric_collector.collect_job_exit_reason(self.exit_reason)
                return 1
            if self.job_manager.all_workers_exited():
                ok = self.job_manager.all_workers_succeeded()
                self.exit_reason = JobExitReason.SUCCEEDED if ok else JobExitReason.WORKER_ERROR
                logger.info(f"all workers exited (success={ok})")
                self.metric_collector.collect_job_exit_reason(self.exit_reason)
                return 0 if ok else 1
        if self._stop_request is not None:
            ok, reason, _ = self._stop_request
            self.exit_reason = reason
            self.metric_collector.collect_job_exit_reason(reason)
            return 0 if ok else 1
        return 0


def main(argv=None) -> int:
    import argparse

    p = argparse.ArgumentParser("dwamd job master")
    p.add_argument("--port", type=int, default=0)
    p.add_argument("--node_num", "--node-num", type=int, default=1)
    p.add_argument("--job_name", "--job-name", default="local")
    p.add_argument("--namespace", default="default")
    p.add_argument("--platform", default="local")
    p.add_argument("--loop_interval", type=float, default=30.0)
    p.add_argument("--port_file", default="")
    p.add_argument("--nproc_per_node", "--nproc-per-node", type=int, default=1)
    p.add_argument("--max_relaunch_count", "--max-relaunch-count", type=int, default=3)
    p.add_argument("--log_dir", "--log-dir", default="")
    p.add_argument("--agent_args", "--agent-args", default="", help="extra dwamd-run flags (one string)")
    p.add_argument("--optimize_mode", "--optimize-mode", default="single-job", choices=["single-job", "cluster"])
    p.add_argument("--brain_addr", "--brain-addr", default="")
    p.add_argument("--max_workers", "--max-workers", type=int, default=0)
    p.add_argument("entry", nargs=argparse.REMAINDER, help="training script + args (platform=process)")
    a = p.parse_args(argv)
    if a.platform == "process":
        import shlex

        from ..common.node import JobResource
        from .scaler import ProcessScaler

        jr = JobResource()
        jr.update_node_group_resource("worker", a.node_num)
        m = DistributedJobMaster(
            jr, lambda addr: ProcessScaler(a.job_name, addr, a.entry, a.nproc_per_node, str(a.node_num),
                                           a.log_dir, agent_args=shlex.split(a.agent_args)),
            port=a.port, loop_interval=min(a.loop_interval, 5.0), max_relaunch_count=a.max_relaunch_count,
            optimize_mode=a.optimize_mode, brain_addr=a.brain_addr, job_name=a.job_name, max_workers=a.max_workers)
    elif a.platform in ("k8s", "pyk8s"):
        # in-cluster: worker pods through the Kubernetes API (platform/k8s.py)
        import os
        import shlex

        from ..common.node import JobResource
        from ..platform.k8s import ElasticJobScaler, K8sClient, K8sScalePlanWatcher, PodScaler, PodWatcher

        jr = JobResource()
        jr.update_node_group_resource("worker", a.node_num)
        cli = K8sClient(a.namespace)
        svc = f"elasticjob-{a.job_name}-dlrover-master"
        image = os.environ.get("DWAMD_WORKER_IMAGE", "")
        cmd = shlex.split(os.environ.get("DWAMD_WORKER_COMMAND", "dwamd-run --nnodes auto train.py"))
        if a.platform == "k8s":
            # the ElasticJob operator creates / deletes pods from our ScalePlans
            scaler_factory = lambda addr: ElasticJobScaler(a.job_name, cli)  # noqa: E731
        else:
            # pyk8s: the master creates the pods itself
            scaler_factory = lambda addr: PodScaler(a.job_name, cli, image,  # noqa: E731
                                                    f"{svc}:{addr.rsplit(':', 1)[1]}", cmd,
                                                    gpus_per_node=a.nproc_per_node)
        m = DistributedJobMaster(
            jr, scaler_factory,
            watcher_factory=lambda scaler: PodWatcher(a.job_name, cli), port=a.port,
            loop_interval=a.loop_interval, max_relaunch_count=a.max_relaunch_count,
            optimize_mode=a.optimize_mode, brain_addr=a.brain_addr, job_name=a.job_name, max_workers=a.max_workers)
        # manual ScalePlans (spec.manualScaling) of this job -> the job manager
        sp_watcher = K8sScalePlanWatcher(a.job_name, cli)

        def _manual_scaling():
            for plan in sp_watcher.watch(interval=a.loop_interval):
                m.job_manager.apply_scale_plan(plan)

        threading.Thread(target=_manual_scaling, daemon=True, name="dwamd-scaleplan-watcher").start()
    else:
        m = JobMaster(port=a.port, node_num=a.node_num, loop_interval=a.loop_interval)
    m.prepare()
    if a.port_file:
        with open(a.port_file, "w") as f:
            f.write(str(m.port))
    try:
        return m.run()
    finally:
        m.stop()


if __name__ == "__main__":
    raise SystemExit(main())
