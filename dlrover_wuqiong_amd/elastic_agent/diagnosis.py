"""Agent-side diagnosis collectors + periodic reporter.

Collectors (parity: reference ``elastic_agent/datacollector/*.py`` and
``monitor/diagnosis.py:28-112``, which are stubs there):

* ``TrainingLogCollector`` -- tail of each worker log file;
* ``GpuLogCollector`` -- HIP / RCCL / amdgpu-KFD error signatures in the worker
  logs (memory access faults, RCCL async errors, ECC ...), i.e. evidence
  for a *hardware* (node-level) failure vs. a code error;
* ``ChipMetricsCollector`` -- per-GPU busy %, VRAM used, temperature and power
  from the amdgpu sysfs (no HIP initialisation in the agent).

``DiagnosisMonitor`` runs them every ``interval`` seconds and reports to the
master (``MasterClient.report_diagnosis``).  ``classify_failure`` turns a
failed worker's log into a ``TrainingExceptionLevel`` so the agent reports
NODE_ERROR (relaunch the node) for hardware signatures.
"""

import glob
import os
import re
import threading
from typing import Dict, List, Optional

from ..common.constants import TrainingExceptionLevel
from ..common.diagnosis import ChipMetrics, GpuRuntimeLog, TrainingLog
from ..common.log import logger

GPU_ERROR_PATTERNS = [
    r"Memory access fault by GPU",
    r"HSA_STATUS_ERROR\w*",
    r"hipErrorIllegalAddress|hipErrorLaunchFailure|hipErrorECCNotCorrectable|hipErrorNoDevice",
    r"RCCL (?:WARN|ERROR).*(?:timeout|error|abort)",
    r"NCCL (?:WARN|ERROR).*(?:timeout|error|abort)",
    r"amdgpu.*(?:GPU reset|ring .* timeout|ECC)",
    r"GPU Hang|gpu hang",
    r"uncorrectable ECC",
]
_GPU_RE = re.compile("|".join(f"(?:{p})" for p in GPU_ERROR_PATTERNS))


def _tail(path: str, nbytes: int = 16384) -> List[str]:
    try:
        with open(path, "rb") as f:
            f.seek(0, os.SEEK_END)
            size = f.tell()
            f.seek(max(0, size - nbytes))
            return f.read().decode("utf-8", errors="replace").splitlines()
    except OSError:
        return []


class TrainingLogCollector:
    def __init__(self, log_dir: str = "", n_lines: int = 50):
        self.log_dir = log_dir
        self.n_lines = n_lines

    def files(self) -> List[str]:
        return sorted(glob.glob(os.path.join(self.log_dir, "*.log"))) if self.log_dir else []

    def collect_data(self) -> TrainingLog:
        lines: List[str] = []
        for f in self.files():
            lines += [f"{os.path.basename(f)}: {x}" for x in _tail(f)[-self.n_lines:]]
        return TrainingLog(logs=lines)


class GpuLogCollector(TrainingLogCollector):
    def collect_data(self) -> GpuRuntimeLog:
        errors: List[str] = []
        for f in self.files():
            errors += [x for x in _tail(f, 65536) if _GPU_RE.search(x)]
        return GpuRuntimeLog(errors=errors[-50:])


class ChipMetricsCollector:
    SYSFS = "/sys/class/drm/card*/device"

    def collect_data(self) -> ChipMetrics:
        out: Dict[str, Dict[str, float]] = {}
        for i, dev in enumerate(sorted(glob.glob(self.SYSFS))):
            m: Dict[str, float] = {}
            for key, fname in (("busy_pct", "gpu_busy_percent"), ("vram_used", "mem_info_vram_used"),
                               ("vram_total", "mem_info_vram_total")):
                try:
                    m[key] = float(open(os.path.join(dev, fname)).read().strip())
                except (OSError, ValueError):
                    pass
            for hw in glob.glob(os.path.join(dev, "hwmon", "hwmon*")):
                for key, fname, scale in (("temp_c", "temp1_input", 1e-3), ("power_w", "power1_average", 1e-6)):
                    try:
                        m[key] = float(open(os.path.join(hw, fname)).read().strip()) * scale
                    except (OSError, ValueError):
                        pass
            if m:
                out[str(i)] = m
        return ChipMetrics(gpus=out)


def classify_failure(log_text: str) -> str:
    """NODE_ERROR for GPU/driver signatures (relaunch the node), else
    PROCESS_ERROR (restart the worker processes in place)."""
    if log_text and _GPU_RE.search(log_text):
        return TrainingExceptionLevel.NODE_ERROR
    return TrainingExceptionLevel.PROCESS_ERROR


class DiagnosisMonitor:
    def __init__(self, master_client, log_dir: str = "", interval: float = 60.0):
        self._mc = master_client
        self.collectors = [TrainingLogCollector(log_dir), GpuLogCollector(log_dir), ChipMetricsCollector()]
        self.interval = interval
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None

    def report_once(self):
        for c in self.collectors:
            data = c.collect_data()
            try:
                self._mc.report_diagnosis(type(data).__name__, data.to_json())
            except Exception as e:
                logger.debug(f"diagnosis report failed: {e}")

    def start(self):
        if self._thread is None:
            self._thread = threading.Thread(target=self._run, daemon=True, name="dwamd-diagnosis")
            self._thread.start()

    def _run(self):
        while not self._stop.wait(self.interval):
            self.report_once()

    def stop(self):
        self._stop.set()
