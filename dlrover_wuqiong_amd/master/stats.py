"""Job metric collection and reporting.

Parity: reference ``master/stats/job_collector.py`` (``JobMetricCollector``),
``stats/reporter.py:55-233`` (``StatsReporter``, ``LocalStatsReporter``;
``BrainReporter`` posts to the Brain service -- out of scope) and
``stats/training_metrics.py``.  The local reporter keeps the records in
memory and, optionally, appends them as JSON lines to a file that job
dashboards can tail.
"""

import json
import threading
import time
from dataclasses import asdict, dataclass, field
from typing import Dict, List, Optional

from ..common.constants import NodeStatus


@dataclass
class DatasetMetric:
    name: str = ""
    size: int = 0
    storage_type: str = ""


@dataclass
class ModelMetric:
    num_params: int = 0
    flops: float = 0.0


@dataclass
class TrainingHyperParams:
    batch_size: int = 0
    epoch: int = 0
    max_steps: int = 0


@dataclass
class RuntimeMetric:
    timestamp: float = 0.0
    global_step: int = 0
    speed: float = 0.0
    running_nodes: List[Dict] = field(default_factory=list)


class StatsReporter:
    def report_dataset_metric(self, metric: DatasetMetric):
        ...

    def report_model_metrics(self, metric: ModelMetric):
        ...

    def report_training_hyper_params(self, params: TrainingHyperParams):
        ...

    def report_runtime_stats(self, stats: RuntimeMetric):
        ...

    def report_job_exit_reason(self, reason: str):
        ...


class LocalStatsReporter(StatsReporter):
    def __init__(self, path: str = ""):
        self.path = path
        self.records: List[Dict] = []
        self._lock = threading.Lock()

    def _add(self, kind: str, payload):
        rec = {"kind": kind, "time": time.time(), **(asdict(payload) if hasattr(payload, "__dataclass_fields__")
                                                     else {"value": payload})}
        with self._lock:
            self.records.append(rec)
            if self.path:
                with open(self.path, "a") as f:
                    f.write(json.dumps(rec) + "\n")

    def report_dataset_metric(self, metric):
        self._add("dataset", metric)

    def report_model_metrics(self, metric):
        self._add("model", metric)

    def report_training_hyper_params(self, params):
        self._add("hyper_params", params)

    def report_runtime_stats(self, stats):
        self._add("runtime", stats)

    def report_job_exit_reason(self, reason):
        self._add("exit_reason", reason)


class JobMetricCollector:
    def __init__(self, job_manager, speed_monitor, reporter: Optional[StatsReporter] = None):
        self._jm = job_manager
        self._speed = speed_monitor
        self.reporter = reporter or LocalStatsReporter()

    def collect_dataset_metric(self, name: str, size: int, storage_type: str = ""):
        self.reporter.report_dataset_metric(DatasetMetric(name, size, storage_type))

    def collect_model_metric(self, num_params: int, flops: float = 0.0):
        self.reporter.report_model_metrics(ModelMetric(num_params, flops))

    def collect_training_hyper_params(self, batch_size: int = 0, epoch: int = 0, max_steps: int = 0):
        self.reporter.report_training_hyper_params(TrainingHyperParams(batch_size, epoch, max_steps))

    def collect_runtime_stats(self) -> RuntimeMetric:
        nodes = [{"id": n.id, "type": n.type, "rank": n.rank_index, "cpu": n.used_cpu, "mem": n.used_memory,
                  "gpus": [vars(g) if hasattr(g, "__dict__") else g for g in n.gpu_stats]}
                 for n in self._jm.nodes.values() if n.status == NodeStatus.RUNNING]
        m = RuntimeMetric(timestamp=time.time(), global_step=getattr(self._speed, "completed_global_step", 0),
                          speed=self._speed.running_speed(), running_nodes=nodes)
        self.reporter.report_runtime_stats(m)
        return m

    def collect_job_exit_reason(self, reason: str):
        self.reporter.report_job_exit_reason(reason)
