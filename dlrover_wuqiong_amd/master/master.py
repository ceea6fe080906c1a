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
                 run_configs: Optional[Dict[str, str]] = None, max_relaunch_count: int = 3):
        self.port = port or find_free_port()
        self.node_num = node_num
        self.job_manager = JobManager(node_num, launcher, max_relaunch_count=max_relaunch_count)
        self.task_manager = TaskManager()
        self.speed_monitor = SpeedMonitor()
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
DistributedJobMaster = JobMaster


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
    a = p.parse_args(argv)
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
