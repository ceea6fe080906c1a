"""Network throughput monitor: a daemon thread sampling the host's RDMA
(``/sys/class/infiniband/<dev>/ports/<p>/counters/port_{xmit,rcv}_data``,
in 4-byte words) and Ethernet (``/sys/class/net/<if>/statistics/
{tx,rx}_bytes``) counters and keeping per-device send / receive rates --
the scale-out links of an MI355X node (its scale-up xGMI traffic is visible
to RCCL only).  ``snapshot()`` returns the latest rates; the elastic
agent's resource monitor and the diagnosis collectors can export them.

Parity: ATorch ``atorch/utils/ib_monitor.py`` (IBStat thread).
"""

import os
import threading
import time
from typing import Dict, Optional


def _read_int(path: str) -> Optional[int]:
    try:
        with open(path) as f:
            return int(f.read().strip())
    except (OSError, ValueError):
        return None


class NetStat(threading.Thread):
    def __init__(self, interval: float = 1.0, sysfs_root: str = "/sys/class", include_eth: bool = True):
        super().__init__(daemon=True, name="dwamd-netstat")
        self.interval = interval
        self.root = sysfs_root
        self.include_eth = include_eth
        self._stop_ev = threading.Event()
        self._lock = threading.Lock()
        self._rates: Dict[str, Dict[str, float]] = {}
        self._last: Dict[str, tuple] = {}

    def counters(self) -> Dict[str, tuple]:
        """{device: (tx_bytes, rx_bytes)} now."""
        out = {}
        ib = os.path.join(self.root, "infiniband")
        if os.path.isdir(ib):
            for dev in sorted(os.listdir(ib)):
                ports = os.path.join(ib, dev, "ports")
                for p in sorted(os.listdir(ports)) if os.path.isdir(ports) else ():
                    c = os.path.join(ports, p, "counters")
                    tx, rx = _read_int(os.path.join(c, "port_xmit_data")), _read_int(os.path.join(c, "port_rcv_data"))
                    if tx is not None and rx is not None:
                        out[f"{dev}:{p}"] = (4 * tx, 4 * rx)  # counters are in 4-byte words
        net = os.path.join(self.root, "net")
        if self.include_eth and os.path.isdir(net):
            for dev in sorted(os.listdir(net)):
                if dev == "lo":
                    continue
                s = os.path.join(net, dev, "statistics")
                tx, rx = _read_int(os.path.join(s, "tx_bytes")), _read_int(os.path.join(s, "rx_bytes"))
                if tx is not None and rx is not None:
                    out[dev] = (tx, rx)
        return out

    def sample(self, now: Optional[float] = None):
        now = time.monotonic() if now is None else now
        cur = self.counters()
        rates = {}
        for dev, (tx, rx) in cur.items():
            prev = self._last.get(dev)
            if prev is not None and now > prev[0]:
                dt = now - prev[0]
                rates[dev] = {"tx_gbps": max(0, tx - prev[1]) / dt / 1e9, "rx_gbps": max(0, rx - prev[2]) / dt / 1e9}
            self._last[dev] = (now, tx, rx)
        with self._lock:
            self._rates.update(rates)
        return rates

    def snapshot(self) -> Dict[str, Dict[str, float]]:
        with self._lock:
            return {k: dict(v) for k, v in self._rates.items()}

    def run(self):
        while not self._stop_ev.is_set():
            self.sample()
            self._stop_ev.wait(self.interval)

    def stop(self):
        self._stop_ev.set()
