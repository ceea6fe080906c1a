"""Worker-side hang detection and relaunch requests.

A worker talks to its node's elastic agent through a small control directory
(``DWAMD_AGENT_CTL_DIR``, created per agent):

* ``hb.<local_rank>``        -- heartbeat file; its mtime is the last time the
  worker reported progress (``HangingDetector.report_normal``, or the
  ElasticTrainer step hook).  With ``--hang-timeout`` the agent treats a stale
  heartbeat as a hang;
* ``relaunch.<local_rank>``  -- written (atomically) by ``request_relaunch``:
  the agent kills the worker group, persists the in-memory checkpoint and
  restarts it, exactly like a crash.

The worker's own detector (``HangingDetector``) also fires from inside the
process, so a hang in a collective that leaves the Python thread blocked
still gets reported by the detector's thread -- and ``xpu_timer`` reports
device-side hangs through the same ``request_relaunch``.

Parity: ATorch ``atorch/fault_tolerance/hanging_detector.py``
(``HangingDetector(timeout, monitor_interval)``: ``start/stop/report_normal``;
``RelaunchStatus`` worker/agent relaunch ids over a TCPStore) and
``fault_tolerance/custom_agent.py`` (agent restarts workers on request).
"""

import faulthandler
import os
import threading
import time
from typing import Optional

from ..common.log import logger

CTL_ENV = "DWAMD_AGENT_CTL_DIR"


def ctl_dir() -> Optional[str]:
    d = os.getenv(CTL_ENV)
    return d if d and os.path.isdir(d) else None


def _local_rank() -> int:
    return int(os.getenv("LOCAL_RANK", "0"))


def heartbeat():
    """Touch this worker's heartbeat file (cheap: one utime syscall)."""
    d = ctl_dir()
    if d is None:
        return
    p = os.path.join(d, f"hb.{_local_rank()}")
    try:
        os.utime(p, None)
    except FileNotFoundError:
        with open(p, "w"):
            pass


def request_relaunch(reason: str) -> bool:
    """Ask the agent to restart the worker group.  Returns False when not
    running under the agent."""
    d = ctl_dir()
    if d is None:
        logger.warning(f"relaunch requested ({reason}) but no agent control dir")
        return False
    lr = _local_rank()
    tmp = os.path.join(d, f".relaunch.{lr}.{os.getpid()}")
    with open(tmp, "w") as f:
        f.write(reason)
    os.replace(tmp, os.path.join(d, f"relaunch.{lr}"))
    logger.error(f"worker {lr}: relaunch requested: {reason}")
    return True


class HangingDetector:
    """Call ``report_normal()`` every step; if no report arrives for
    ``timeout`` seconds while running, dump all Python stacks to the log and
    request a relaunch of the worker group."""

    def __init__(self, timeout: float = 300.0, monitor_interval: float = 15.0, rank: Optional[int] = None,
                 dump_stacks: bool = True):
        self.timeout = timeout
        self.monitor_interval = monitor_interval
        self.rank = rank if rank is not None else int(os.getenv("RANK", "0"))
        self.dump_stacks = dump_stacks
        self._last = time.time()
        self._running = False
        self._enabled = True
        self._thread: Optional[threading.Thread] = None
        self.fired = threading.Event()

    def start(self):
        if not self._enabled:
            return
        self._last = time.time()
        self._running = True
        heartbeat()
        if self._thread is None:
            self._thread = threading.Thread(target=self._loop, daemon=True, name="dwamd-hang-detector")
            self._thread.start()

    def stop(self, finalize: bool = False):
        self._running = False
        if finalize:
            self._enabled = False

    def report_normal(self):
        self._last = time.time()
        heartbeat()

    def _loop(self):
        while self._enabled:
            time.sleep(min(self.monitor_interval, max(self.timeout / 4, 0.05)))
            if self._running and time.time() - self._last > self.timeout:
                msg = f"rank {self.rank}: no progress for {time.time() - self._last:.0f}s"
                logger.error(f"hang detected: {msg}")
                if self.dump_stacks:
                    try:
                        faulthandler.dump_traceback(all_threads=True)
                    except Exception:  # pragma: no cover
                        pass
                request_relaunch(f"hang: {msg}")
                self.fired.set()
                break
