"""Throughput timer and lightweight GPU-event timers.

``ThroughputTimer(batch_size, start_step=2, steps_per_output=50)``: call
``start()`` / ``stop()`` around each step; it reports samples/s (and
TFLOP/s when ``flops_per_sample`` is given) averaged over the steps after
the warm-up, synchronising the device only when a report is due.
``Timers`` keeps named ``hipEvent`` intervals without host syncs until
``elapsed()`` is read.

Parity: ATorch ``atorch/utils/timer.py`` (``ThroughputTimer``) and
``atorch/utils/prof.py`` timers.
"""

import time
from typing import Dict, Optional

import torch

from ...common.log import logger


class ThroughputTimer:
    def __init__(self, batch_size: int, start_step: int = 2, steps_per_output: int = 50, monitor_memory: bool = False,
                 logging_fn=None, flops_per_sample: Optional[float] = None):
        self.batch_size = batch_size
        self.start_step = start_step
        self.steps_per_output = steps_per_output
        self.monitor_memory = monitor_memory
        self.logging = logging_fn or logger.info
        self.flops_per_sample = flops_per_sample
        self.epoch_count = 0
        self.local_step_count = 0
        self.total_step_count = 0
        self.total_elapsed_time = 0.0
        self.step_elapsed_time = 0.0
        self.started = False
        self._t0 = 0.0

    def update_epoch(self):
        self.epoch_count += 1
        self.local_step_count = 0

    def _sync(self):
        if torch.cuda.is_available():
            torch.cuda.synchronize()

    def start(self):
        self.started = True
        if self.total_step_count >= self.start_step:
            self._sync()
            self._t0 = time.perf_counter()

    def stop(self, end_train: bool = True, report_speed: bool = True):
        if not self.started:
            return
        self.started = False
        self.total_step_count += 1
        self.local_step_count += 1
        if self.total_step_count > self.start_step:
            self._sync()
            dt = time.perf_counter() - self._t0
            self.total_elapsed_time += dt
            self.step_elapsed_time += dt
            if report_speed and self.local_step_count % self.steps_per_output == 0:
                msg = (f"epoch={self.epoch_count}/step={self.local_step_count}: "
                       f"samples/s={self.avg_samples_per_sec():.2f}, last {self.steps_per_output} steps "
                       f"{self.step_elapsed_time:.3f}s")
                if self.flops_per_sample:
                    msg += f", TFLOP/s={self.avg_samples_per_sec() * self.flops_per_sample / 1e12:.1f}"
                if self.monitor_memory and torch.cuda.is_available():
                    msg += f", max_mem={torch.cuda.max_memory_allocated() / 2 ** 30:.1f}GiB"
                self.logging(msg)
                self.step_elapsed_time = 0.0

    def avg_samples_per_sec(self) -> float:
        steps = self.total_step_count - self.start_step
        if steps <= 0 or self.total_elapsed_time <= 0:
            return float("-inf")
        return self.batch_size / (self.total_elapsed_time / steps)


class Timers:
    """Named device-event intervals (no host sync until read)."""

    def __init__(self):
        self._ev: Dict[str, list] = {}
        self._cpu: Dict[str, list] = {}

    def start(self, name: str):
        if torch.cuda.is_available():
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self._ev.setdefault(name, []).append([e, None])
        else:
            self._cpu.setdefault(name, []).append([time.perf_counter(), None])

    def stop(self, name: str):
        if torch.cuda.is_available():
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self._ev[name][-1][1] = e
        else:
            self._cpu[name][-1][1] = time.perf_counter()

    def elapsed(self, name: str, reset: bool = True) -> float:
        """Total milliseconds of completed intervals."""
        tot = 0.0
        if name in self._ev:
            for s, e in self._ev[name]:
                if e is not None:
                    e.synchronize()
                    tot += s.elapsed_time(e)
        for s, e in self._cpu.get(name, []):
            if e is not None:
                tot += 1000 * (e - s)
        if reset:
            self._ev.pop(name, None)
            self._cpu.pop(name, None)
        return tot
