"""Agent-side monitors.

Parity: reference ``dlrover/python/elastic_agent/monitor/resource.py:28-180``
(psutil CPU/mem + GPU stats; the reference reads NVML - here AMD GPU stats
come from the amdgpu sysfs nodes, so the agent never initialises HIP) and
``monitor/training.py:77-134`` (``TorchTrainingMonitor``: reports the global
step that the training process writes to ``runtime_metrics.json``).
"""

import glob
import json
import os
import threading
import time
from typing import Dict, Iterable, List, Optional, Set, Tuple

from ..common.comm import GPUStats
from ..common.constants import ConfigPath
from ..common.log import logger


class ResourceMonitor:
    def __init__(self):
        try:
            import psutil

            self._proc = psutil
            psutil.cpu_percent(None)
        except Exception:  # pragma: no cover
            self._proc = None

    def sample(self) -> Tuple[float, int]:
        if self._proc is None:
            return 0.0, 0
        cpu = self._proc.cpu_percent(None) / 100.0 * (os.cpu_count() or 1)
        mem = self._proc.virtual_memory().used
        return cpu, int(mem)

    @staticmethod
    def gpu_stats(pdevs: Optional[Set[str]] = None) -> List[GPUStats]:
        """amdgpu sysfs counters of every GPU of the host, or only of the
        ``pdevs`` PCI addresses (e.g. ``process_gpu_pdevs`` of this job's
        processes: other tenants' GPUs on a shared host do not count)."""
        out = []
        for i, dev in enumerate(sorted(glob.glob("/sys/class/drm/card*/device"))):
            if pdevs and os.path.basename(os.path.realpath(dev)) not in pdevs:
                continue
            try:
                total = int(open(os.path.join(dev, "mem_info_vram_total")).read())
                used = int(open(os.path.join(dev, "mem_info_vram_used")).read())
                busy = float(open(os.path.join(dev, "gpu_busy_percent")).read())
            except (OSError, ValueError):
                continue
            out.append(GPUStats(index=i, total_memory_mb=total >> 20, used_memory_mb=used >> 20,
                                gpu_utilization=busy))
        return out

    @staticmethod
    def process_gpu_usage(pids: Iterable[int]) -> Tuple[Set[str], Dict[int, int]]:
        """(PCI addresses of the GPUs the given processes hold DRM file
        descriptors on, {pid: VRAM bytes}) from /proc/<pid>/fdinfo/* --
        amdgpu publishes ``drm-pdev`` and ``drm-memory-vram`` per open render
        node, HIP allocations included (checked on MI355X:
        scripts/probe/drm_vram_probe.py); no HIP call."""
        found: Set[str] = set()
        vram: Dict[int, int] = {}
        for pid in pids:
            for fi in glob.glob(f"/proc/{int(pid)}/fdinfo/*"):
                try:
                    with open(fi) as f:
                        txt = f.read()
                except OSError:
                    continue
                if "drm-pdev" not in txt:
                    continue
                for line in txt.splitlines():
                    if line.startswith("drm-pdev:"):
                        found.add(line.split(":", 1)[1].strip())
                    elif line.startswith("drm-memory-vram:"):
                        parts = line.split()
                        try:
                            n = int(parts[1]) << {"KiB": 10, "MiB": 20, "GiB": 30}.get(parts[2] if len(parts) > 2
                                                                                       else "", 0)
                        except (IndexError, ValueError):
                            continue
                        vram[int(pid)] = vram.get(int(pid), 0) + n
        return found, vram

    @staticmethod
    def process_gpu_pdevs(pids: Iterable[int]) -> Set[str]:
        return ResourceMonitor.process_gpu_usage(pids)[0]


class TorchTrainingMonitor:
    """Node 0's agent forwards the training step (written by ElasticTrainer
    into ``runtime_metrics.json``) to the master every ``interval`` seconds."""

    def __init__(self, client, metrics_path: str = "", interval: float = 15.0):
        self.client = client
        self.path = metrics_path or os.getenv(ConfigPath.ENV_RUNTIME_METRICS, ConfigPath.RUNTIME_METRICS)
        self.interval = interval
        self._stop = threading.Event()
        self._last_step = -1

    def report_step(self) -> bool:
        try:
            with open(self.path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            return False
        step = int(d.get("step", 0))
        if step > self._last_step:
            self.client.report_global_step(step, d.get("timestamp", time.time()))
            self._last_step = step
            return True
        return False

    def start(self):
        def loop():
            while not self._stop.wait(self.interval):
                try:
                    self.report_step()
                except Exception as e:
                    logger.debug(f"step report failed: {e}")

        threading.Thread(target=loop, daemon=True, name="dwamd-train-monitor").start()

    def stop(self):
        self._stop.set()
