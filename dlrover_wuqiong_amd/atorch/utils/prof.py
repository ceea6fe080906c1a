"""Per-module FLOPs / latency profiler with MFU against the MI355X peak.

``AProfiler(model)`` attaches forward pre/post hooks to every module,
counts FLOPs with ``torch.utils.flop_counter.FlopCounterMode`` (the
aten-level formulas: matmul / conv / SDPA -- the GEMMs our fused ops issue
are counted; work inside a custom HIP kernel such as flash attention is
credited with ``add_flops(flash_attn_flops(...))``) and times each module with device events (host timers on CPU).

    prof = AProfiler(model)
    prof.start_profile()
    loss = model(x); loss.backward()
    prof.stop_profile()
    prof.print_model_profile()       # per-module table + totals, MFU
    prof.get_total_flops(), prof.get_total_duration()

Peak defaults to 2.5e15 (MI355X dense bf16, no sparsity).

Parity: ATorch ``atorch/utils/prof.py`` (AProfiler: start/stop/end_profile,
get_total_flops / params / duration, print_model_profile; per-op FLOP
formulas).
"""

import time
from collections import defaultdict
from typing import Dict, Optional

import torch
import torch.nn as nn

MI355X_BF16_PEAK = 2.5e15


def flash_attn_flops(q_shape, causal: bool = True) -> int:
    """Forward FLOPs of flash attention on q [B, S, H, D] (for ``add_flops``)."""
    B, S, H, D = q_shape
    f = 4 * B * H * S * S * D
    return f // 2 if causal else f


class AProfiler:
    def __init__(self, model: nn.Module, peak_flops: float = MI355X_BF16_PEAK):
        self.model = model
        self.peak = peak_flops
        self._handles = []
        self._mode = None
        self._t0: Dict[int, object] = {}
        self.duration: Dict[str, float] = defaultdict(float)
        self.calls: Dict[str, int] = defaultdict(int)
        self._pending = []
        self.total_duration = 0.0
        self._start = None
        self.extra_flops = 0

    # -- timing ------------------------------------------------------------
    def _now(self):
        if torch.cuda.is_available():
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            return e
        return time.perf_counter()

    def _pre(self, name):
        def hook(mod, args):
            self._t0[id(mod)] = self._now()
        return hook

    def _post(self, name):
        def hook(mod, args, out):
            t0 = self._t0.pop(id(mod), None)
            if t0 is not None:
                self._pending.append((name, t0, self._now()))
            self.calls[name] += 1
        return hook

    def start_profile(self):
        from torch.utils.flop_counter import FlopCounterMode

        for name, m in self.model.named_modules():
            name = name or type(self.model).__name__
            self._handles.append(m.register_forward_pre_hook(self._pre(name)))
            self._handles.append(m.register_forward_hook(self._post(name)))
        self._mode = FlopCounterMode(display=False)
        self._mode.__enter__()
        self._start = self._now()

    def add_flops(self, flops: int):
        """Credit work the aten counter cannot see (custom HIP ops)."""
        self.extra_flops += int(flops)

    def stop_profile(self):
        end = self._now()
        if self._mode is not None:
            self._mode.__exit__(None, None, None)
        for h in self._handles:
            h.remove()
        self._handles = []
        if torch.cuda.is_available():
            torch.cuda.synchronize()
            el = lambda a, b: a.elapsed_time(b) * 1e-3  # noqa: E731
        else:
            el = lambda a, b: b - a  # noqa: E731
        for name, a, b in self._pending:
            self.duration[name] += el(a, b)
        self._pending = []
        self.total_duration = el(self._start, end) if self._start is not None else 0.0

    def end_profile(self):
        self._mode = None
        self.duration.clear()
        self.calls.clear()

    # -- results -----------------------------------------------------------
    def module_flops(self) -> Dict[str, int]:
        if self._mode is None:
            return {}
        counts = self._mode.get_flop_counts()
        root = type(self.model).__name__
        out = {}
        for mod, ops in counts.items():
            out[mod] = sum(ops.values())
        if "Global" in out:
            out[root] = out.pop("Global")
        return out

    def get_total_flops(self) -> int:
        return (self._mode.get_total_flops() if self._mode is not None else 0) + self.extra_flops

    def get_total_params(self) -> int:
        return sum(p.numel() for p in self.model.parameters())

    def get_total_duration(self) -> float:
        return self.total_duration

    def mfu(self, n_devices: int = 1) -> Optional[float]:
        t = self.total_duration
        return self.get_total_flops() / t / (self.peak * n_devices) if t > 0 else None

    def print_model_profile(self, top: int = 20, file=None):
        fl = self.module_flops()
        rows = sorted(self.duration.items(), key=lambda kv: -kv[1])[:top]
        lines = [f"{'module':48s} {'calls':>6s} {'time ms':>10s} {'GFLOP':>12s}"]
        for name, d in rows:
            lines.append(f"{name[:48]:48s} {self.calls[name]:6d} {1e3 * d:10.3f} {fl.get(name, 0) / 1e9:12.3f}")
        m = self.mfu()
        lines.append(f"total: {self.get_total_params() / 1e6:.2f} M params, {self.get_total_flops() / 1e9:.3f} GFLOP, "
                     f"{1e3 * self.total_duration:.3f} ms" + (f", MFU {100 * m:.2f}%" if m is not None else ""))
        print("\n".join(lines), file=file)
        return lines
