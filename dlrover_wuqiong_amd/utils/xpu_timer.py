"""xpu_timer: per-shape GEMM / per-collective device timing, Prometheus
export and device-hang detection.

    from dlrover_wuqiong_amd.utils.xpu_timer import XpuTimer
    timer = XpuTimer(hang_timeout=300).install()      # mm/bmm/linear + collectives
    timer.start_exporter(port=38888 + local_rank)      # GET /metrics
    ...
    print(timer.report())

Interposition: a ``TorchFunctionMode`` catches ``mm/bmm/matmul/addmm/linear``
(key = kind + m/n/k, work = 2mnk FLOPs), the ``torch.distributed``
collectives are wrapped (key = collective + dtype + bytes, work = bytes,
reported as algorithm and bus bandwidth), and every launch of the
framework's own HIP kernel library (flash attention, norms, RoPE, fused
optimizers, grouped GEMM, hipBLASLt epilogue GEMMs, checkpoint copies) is
bracketed at its single entry point (``ops/_hip.lib()``; key = ``kernel:``
+ entry point, i.e. ``kernel|dw_attn_fwd_strided``) -- the same coverage the reference gets from LD_PRELOAD
hooks of the vendor libraries, without a preload.  On a GPU, each op is bracketed by
two pooled hipEvents recorded on the current stream (``csrc/kernels/
xpu_timer.hip``); a native poller thread turns them into statistics without
ever synchronising the training stream, and flags a device hang when an op
does not finish within ``hang_timeout``.  On the CPU (gloo) the same API times
ops with the host clock (they are synchronous there).

Hang handling: ``on_hang`` callbacks run once per hang; the default dumps all
Python stacks (faulthandler) and, under the elastic agent, asks the agent to
relaunch the worker group (``fault_tolerance.request_relaunch``).

Parity: ATorch ``atorch/dev/xpu_timer`` (README metric names
``atorch_mm_mnk_*`` / ``*_avg_latency`` / ``*_p99_latency`` on a Prometheus
port, hang detection in ``common/manager.cc``).
"""

import ctypes
import faulthandler
import functools
import os
import sys
import threading
import time
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional

import torch
import torch.distributed as dist
from torch.overrides import TorchFunctionMode

from ..common.log import logger

_COLLECTIVES = ("all_reduce", "all_gather", "all_gather_into_tensor", "reduce_scatter", "reduce_scatter_tensor",
                "broadcast", "all_to_all", "all_to_all_single", "reduce", "send", "recv", "barrier")


@dataclass
class OpStat:
    key: str
    count: int
    avg_us: float
    max_us: float
    p50_us: float
    p99_us: float
    work_per_us: float  # FLOPs/us (GEMM) or bytes/us (collective)

    @property
    def kind(self) -> str:
        return self.key.split("|", 1)[0]

    def rate(self) -> Dict[str, float]:
        if self.kind == "kernel":
            return {}  # framework kernels: latency statistics only
        if self.kind in ("mm", "bmm", "linear", "matmul", "addmm"):
            return {"tflops": self.work_per_us * 1e-6}
        return {"algbw_gbps": self.work_per_us * 1e-3}


class _HostBackend:
    """CPU timing backend (ops are synchronous: wall clock is op time)."""

    def __init__(self):
        self.lock = threading.Lock()
        self.keys: Dict[str, int] = {}
        self.stats: List[list] = []  # [n, sum, max, samples[], work]
        self.open: Dict[int, tuple] = {}
        self.tok = 0

    def key(self, name: str) -> int:
        with self.lock:
            if name not in self.keys:
                self.keys[name] = len(self.stats)
                self.stats.append([0, 0.0, 0.0, [], 0.0, name])
            return self.keys[name]

    def begin(self, k: int, stream=None) -> int:
        with self.lock:
            self.tok += 1
            self.open[self.tok] = (k, time.perf_counter())
            return self.tok

    def end(self, tok: int, work: float, stream=None):
        t1 = time.perf_counter()
        with self.lock:
            k, t0 = self.open.pop(tok)
            us = (t1 - t0) * 1e6
            st = self.stats[k]
            st[0] += 1
            st[1] += us
            st[2] = max(st[2], us)
            st[3].append(us)
            if len(st[3]) > 1024:
                del st[3][0]
            st[4] += work

    def snapshot(self) -> List[OpStat]:
        out = []
        with self.lock:
            for n, s, m, samples, work, name in self.stats:
                if n == 0:
                    continue
                v = sorted(samples)
                pct = lambda p: v[min(len(v) - 1, int(p * (len(v) - 1) + 0.5))]  # noqa: E731
                out.append(OpStat(name, n, s / n, m, pct(0.5), pct(0.99), work / s if s > 0 else 0.0))
        return out

    def hang(self):
        return 0, "", 0.0

    def flush(self, timeout=10.0):
        return True

    def reset(self):
        with self.lock:
            for st in self.stats:
                st[:5] = [0, 0.0, 0.0, [], 0.0]

    def start(self, hang_timeout, poll_ms):
        pass

    def stop(self):
        pass


class _HipBackend:
    """Native HIP-event backend (``libdw_kernels.so``: dw_xt_*)."""

    def __init__(self):
        from .._native import kernels

        self.lib = kernels(required=True)
        self._keys: Dict[str, int] = {}

    def key(self, name: str) -> int:
        k = self._keys.get(name)
        if k is None:
            k = self._keys[name] = self.lib.dw_xt_key(name.encode())
        return k

    def begin(self, k: int, stream) -> int:
        return self.lib.dw_xt_begin(k, stream)

    def end(self, tok: int, work: float, stream):
        if tok >= 0:
            self.lib.dw_xt_end(tok, float(work), stream)

    def snapshot(self) -> List[OpStat]:
        n = self.lib.dw_xt_snapshot(None, 0)
        buf = ctypes.create_string_buffer(n + 1)
        self.lib.dw_xt_snapshot(buf, n + 1)
        out = []
        for line in buf.value.decode().splitlines():
            f = line.split("\t")
            out.append(OpStat(f[0], int(f[1]), float(f[2]), float(f[3]), float(f[4]), float(f[5]), float(f[6])))
        return out

    def hang(self):
        buf = ctypes.create_string_buffer(512)
        sec = ctypes.c_double(0)
        h = self.lib.dw_xt_hang(buf, 512, ctypes.byref(sec))
        return h, buf.value.decode(), sec.value

    def flush(self, timeout=10.0):
        return self.lib.dw_xt_flush(float(timeout)) == 0

    def reset(self):
        self.lib.dw_xt_reset()

    def start(self, hang_timeout, poll_ms):
        self.lib.dw_xt_start(float(hang_timeout), int(poll_ms))

    def stop(self):
        self.lib.dw_xt_stop()


def _stream_ptr(t: torch.Tensor):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream) if t.is_cuda else None


def _gemm_key(func_name: str, args) -> Optional[tuple]:
    """(kind, shape string, flops) or None for ops we do not time."""
    try:
        if func_name == "mm":
            a, b = args[0], args[1]
            m, k = a.shape
            n = b.shape[1]
            return "mm", f"{m}_{n}_{k}", 2.0 * m * n * k, a
        if func_name == "addmm":
            a, b = args[1], args[2]
            m, k = a.shape
            n = b.shape[1]
            return "mm", f"{m}_{n}_{k}", 2.0 * m * n * k, a
        if func_name == "bmm":
            a, b = args[0], args[1]
            bs, m, k = a.shape
            n = b.shape[2]
            return "bmm", f"{bs}_{m}_{n}_{k}", 2.0 * bs * m * n * k, a
        if func_name == "linear":
            x, w = args[0], args[1]
            k = x.shape[-1]
            m = x.numel() // max(k, 1)
            n = w.shape[0]
            return "linear", f"{m}_{n}_{k}", 2.0 * m * n * k, x
        if func_name == "matmul":
            a, b = args[0], args[1]
            if a.dim() < 2 or b.dim() < 2:
                return None
            k = a.shape[-1]
            m = a.numel() // max(k, 1)
            n = b.shape[-1]
            return "matmul", f"{m}_{n}_{k}", 2.0 * m * n * k, a
    except (AttributeError, ValueError, IndexError, TypeError):
        return None
    return None


class _GemmMode(TorchFunctionMode):
    _names = {"mm", "addmm", "bmm", "linear", "matmul"}

    def __init__(self, timer: "XpuTimer"):
        super().__init__()
        self.timer = timer

    def __torch_function__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        name = getattr(func, "__name__", "")
        if name in self._names:
            info = _gemm_key(name, args)
            if info is not None:
                kind, shape, flops, t = info
                with self.timer.timed(f"{kind}|{shape}", flops, t):
                    return func(*args, **kwargs)
        return func(*args, **kwargs)


class XpuTimer:
    def __init__(self, hang_timeout: float = 300.0, poll_ms: int = 50, device: Optional[str] = None,
                 on_hang: Optional[List[Callable[[str, float], None]]] = None, dump_dir: Optional[str] = None):
        use_gpu = (device or ("cuda" if torch.cuda.is_available() else "cpu")) != "cpu"
        self.backend = _HipBackend() if use_gpu else _HostBackend()
        self.hang_timeout = hang_timeout
        self.poll_ms = poll_ms
        self.on_hang = list(on_hang) if on_hang is not None else [self._default_on_hang]
        self.dump_dir = dump_dir or os.getenv("DWAMD_XPU_TIMER_DIR", "/tmp/dwamd_xpu_timer")
        self._mode: Optional[_GemmMode] = None
        self._orig: Dict[str, Callable] = {}
        self._watch: Optional[threading.Thread] = None
        self._stop = threading.Event()
        self._hang_reported = False
        self._server = None
        self.labels = {"rank": os.getenv("RANK", "0"), "job_name": os.getenv("DWAMD_JOB_NAME", "unknown"),
                       "host_name": os.uname().nodename}

    # ------------------------------------------------------------ timing
    def timed(self, key: str, work: float = 0.0, like: Optional[torch.Tensor] = None):
        return _Timed(self, key, work, like)

    def kernel(self, name: str):
        """Bracket one launch of a framework kernel on torch's current stream."""
        return _TimedStream(self, "kernel|" + name)

    # ------------------------------------------------------------ install
    def install(self, gemm: bool = True, collectives: bool = True, kernels: bool = True) -> "XpuTimer":
        self.backend.start(self.hang_timeout, self.poll_ms)
        if kernels:
            from ..ops import _hip

            _hip._TIMER = self
        if gemm and self._mode is None:
            self._mode = _GemmMode(self)
            self._mode.__enter__()
        if collectives:
            self._wrap_collectives()
        if self._watch is None:
            self._stop.clear()
            self._watch = threading.Thread(target=self._watch_loop, daemon=True, name="dwamd-xpu-timer")
            self._watch.start()
        return self

    def uninstall(self):
        from ..ops import _hip

        if _hip._TIMER is self:
            _hip._TIMER = None
        if self._mode is not None:
            self._mode.__exit__(None, None, None)
            self._mode = None
        for name, fn in self._orig.items():
            setattr(dist, name, fn)
        self._orig.clear()
        self._stop.set()
        if self._watch is not None:
            self._watch.join(timeout=5)
            self._watch = None
        self.backend.stop()
        if self._server is not None:
            self._server.shutdown()
            self._server = None

    def _wrap_collectives(self):
        for name in _COLLECTIVES:
            fn = getattr(dist, name, None)
            if fn is None or name in self._orig:
                continue
            self._orig[name] = fn
            setattr(dist, name, self._wrap(name, fn))

    def _wrap(self, name: str, fn: Callable) -> Callable:
        timer = self

        @functools.wraps(fn)
        def wrapper(*args, **kwargs):
            t = _first_tensor(args, kwargs)
            if t is None or kwargs.get("async_op"):
                return fn(*args, **kwargs)
            nbytes = _payload_bytes(name, args, kwargs)
            ws = 1
            try:
                ws = dist.get_world_size(kwargs.get("group"))
            except Exception:
                pass
            key = f"{name}|{str(t.dtype).replace('torch.', '')}|{nbytes}|ws{ws}"
            with timer.timed(key, float(nbytes), t):
                return fn(*args, **kwargs)

        return wrapper

    # ------------------------------------------------------------ results
    def flush(self, timeout: float = 10.0) -> bool:
        return self.backend.flush(timeout)

    def stats(self) -> List[OpStat]:
        return self.backend.snapshot()

    def reset(self):
        self.backend.reset()

    def report(self) -> str:
        rows = sorted(self.stats(), key=lambda s: -s.avg_us * s.count)
        lines = [f"{'op':60s} {'count':>7s} {'avg_us':>9s} {'p99_us':>9s} {'max_us':>9s}  rate"]
        for s in rows:
            rate = ", ".join(f"{k}={v:.1f}" for k, v in s.rate().items())
            lines.append(f"{s.key:60s} {s.count:7d} {s.avg_us:9.1f} {s.p99_us:9.1f} {s.max_us:9.1f}  {rate}")
        return "\n".join(lines)

    def prometheus_text(self) -> str:
        """Prometheus exposition text: one gauge family per statistic with
        kind/shape labels (shape-in-label rather than the reference's
        shape-in-metric-name keeps the series count bounded per family)."""
        lab = ",".join(f'{k}="{v}"' for k, v in self.labels.items())
        fams = {"avg_latency_us": [], "max_latency_us": [], "p50_latency_us": [], "p99_latency_us": [],
                "count": [], "tflops": [], "algbw_gbps": [], "busbw_gbps": []}
        for s in self.stats():
            kind, rest = s.key.split("|", 1)
            base = f'{lab},kind="{kind}",shape="{rest}"'
            fams["avg_latency_us"].append((base, s.avg_us))
            fams["max_latency_us"].append((base, s.max_us))
            fams["p50_latency_us"].append((base, s.p50_us))
            fams["p99_latency_us"].append((base, s.p99_us))
            fams["count"].append((base, s.count))
            r = s.rate()
            if "tflops" in r:
                fams["tflops"].append((base, r["tflops"]))
            elif "algbw_gbps" in r:
                fams["algbw_gbps"].append((base, r["algbw_gbps"]))
                n = _ws_from_key(s.key)
                factor = {"all_reduce": 2.0 * (n - 1) / n}.get(kind, (n - 1) / n if n > 1 else 1.0)
                fams["busbw_gbps"].append((base, r["algbw_gbps"] * factor))
        h, desc, sec = self.backend.hang()
        out = []
        for fam, vals in fams.items():
            name = f"dwamd_xpu_timer_{fam}"
            out.append(f"# TYPE {name} gauge")
            out.extend(f"{name}{{{b}}} {v}" for b, v in vals)
        out.append("# TYPE dwamd_xpu_timer_hang gauge")
        out.append(f"dwamd_xpu_timer_hang{{{lab}}} {h}")
        return "\n".join(out) + "\n"

    def start_exporter(self, port: int = 0, addr: str = "127.0.0.1") -> int:
        """Serve ``/metrics`` (Prometheus text).  Returns the bound port."""
        from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

        timer = self

        class H(BaseHTTPRequestHandler):
            def do_GET(self):
                if self.path.startswith("/metrics"):
                    body = timer.prometheus_text().encode()
                    ctype = "text/plain; version=0.0.4"
                elif self.path.startswith("/report"):
                    body = timer.report().encode()
                    ctype = "text/plain"
                else:
                    self.send_response(404)
                    self.end_headers()
                    return
                self.send_response(200)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def log_message(self, *a):
                pass

        self._server = ThreadingHTTPServer((addr, port), H)
        threading.Thread(target=self._server.serve_forever, daemon=True, name="dwamd-xpu-exporter").start()
        return self._server.server_address[1]

    # ------------------------------------------------------------ hang
    def hang_status(self):
        return self.backend.hang()

    def _watch_loop(self):
        while not self._stop.wait(max(0.05, min(5.0, self.hang_timeout / 10))):
            h, desc, sec = self.backend.hang()
            if h and not self._hang_reported:
                self._hang_reported = True
                logger.error(f"xpu_timer: device hang suspected ({desc}, {sec:.0f}s)")
                for cb in self.on_hang:
                    try:
                        cb(desc, sec)
                    except Exception as e:  # pragma: no cover
                        logger.warning(f"hang callback failed: {e}")
            elif not h:
                self._hang_reported = False

    def _default_on_hang(self, desc: str, seconds: float):
        os.makedirs(self.dump_dir, exist_ok=True)
        path = os.path.join(self.dump_dir, f"hang_rank{self.labels['rank']}_{int(time.time())}.txt")
        with open(path, "w") as f:
            f.write(f"{desc} ({seconds:.0f}s)\n\n")
            f.flush()
            faulthandler.dump_traceback(file=f, all_threads=True)
            f.write("\n" + self.report() + "\n")
        from ..atorch.fault_tolerance import request_relaunch

        request_relaunch(f"xpu_timer: {desc}")


class _Timed:
    __slots__ = ("timer", "key", "work", "like", "tok", "stream")

    def __init__(self, timer, key, work, like):
        self.timer, self.key, self.work, self.like = timer, key, work, like
        self.tok = -1

    def __enter__(self):
        b = self.timer.backend
        self.stream = _stream_ptr(self.like) if (self.like is not None and isinstance(b, _HipBackend)) else None
        if isinstance(b, _HipBackend) and self.stream is None:
            return self
        self.tok = b.begin(b.key(self.key), self.stream)
        return self

    def __exit__(self, *exc):
        if self.tok is not None and self.tok >= 0:
            self.timer.backend.end(self.tok, self.work, self.stream)
        return False


class _TimedStream:
    """Like _Timed, on torch's current stream (framework kernel launches)."""

    __slots__ = ("timer", "key", "tok", "stream")

    def __init__(self, timer, key):
        self.timer, self.key, self.tok = timer, key, -1

    def __enter__(self):
        b = self.timer.backend
        self.stream = None
        if isinstance(b, _HipBackend):
            self.stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        self.tok = b.begin(b.key(self.key), self.stream)
        return self

    def __exit__(self, *exc):
        if self.tok is not None and self.tok >= 0:
            self.timer.backend.end(self.tok, 0.0, self.stream)
        return False


def _first_tensor(args, kwargs):
    for a in list(args) + list(kwargs.values()):
        if isinstance(a, torch.Tensor):
            return a
        if isinstance(a, (list, tuple)) and a and isinstance(a[0], torch.Tensor):
            return a[0]
    return None


def _payload_bytes(name, args, kwargs) -> int:
    def nb(x):
        if isinstance(x, torch.Tensor):
            return x.numel() * x.element_size()
        if isinstance(x, (list, tuple)):
            return sum(nb(y) for y in x)
        return 0

    if name in ("all_gather", "all_gather_into_tensor"):
        return nb(args[1] if len(args) > 1 else kwargs.get("input_tensor", kwargs.get("tensor")))
    if name in ("reduce_scatter", "reduce_scatter_tensor", "all_to_all", "all_to_all_single"):
        return nb(args[1] if len(args) > 1 else kwargs.get("input", kwargs.get("input_list")))
    return nb(args[0] if args else kwargs.get("tensor"))


def _ws_from_key(key: str) -> int:
    try:
        return int(key.rsplit("|ws", 1)[1])
    except (IndexError, ValueError):
        return 1


_GLOBAL: Optional[XpuTimer] = None


def maybe_install_from_env() -> Optional[XpuTimer]:
    """``DWAMD_XPU_TIMER=1`` (set by ``dwamd-run --xpu-timer``) installs the
    timer in a worker; the exporter listens on ``DWAMD_XPU_TIMER_PORT`` +
    local rank (default 38888)."""
    global _GLOBAL
    if _GLOBAL is not None or os.getenv("DWAMD_XPU_TIMER", "0") != "1":
        return _GLOBAL
    _GLOBAL = XpuTimer(hang_timeout=float(os.getenv("DWAMD_HANG_TIMEOUT", "300"))).install()
    base = int(os.getenv("DWAMD_XPU_TIMER_PORT", "38888"))
    try:
        _GLOBAL.start_exporter(base + int(os.getenv("LOCAL_RANK", "0")), addr="0.0.0.0")
    except OSError as e:
        logger.warning(f"xpu_timer exporter not started: {e}")
    print(f"xpu_timer installed (pid {os.getpid()})", file=sys.stderr)
    return _GLOBAL
