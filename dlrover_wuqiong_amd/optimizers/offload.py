"""CPU-offloaded AdamW over a flat parameter buffer (ZeRO-Offload style).

The GPU keeps only the bf16 weights and gradients of a ``FlatParams``; the
fp32 master weights and both Adam moments (12 bytes/parameter) live in
pinned host memory and are updated by the native host kernel
``dw_cpu_adamw`` (``csrc/runtime/cpu_adam.cpp``: std::threads x AVX2/FMA).
``step()`` pipelines the buffer in chunks over two HIP side streams:

    D2H stream : grad chunk i  -> pinned host (bf16)
    host cores : AdamW on chunk i-1 (GIL released inside the ctypes call)
    H2D stream : updated bf16 weights of chunk i-2 -> GPU

so host<->device traffic in both directions overlaps the CPU math; the
compute stream waits for the last H2D before the next forward.  On an
MI355X (288 GB HBM) offload is rarely needed for memory -- it is for
models whose optimizer state would otherwise crowd out activations, or for
keeping the optimizer state host-resident next to the flash-checkpoint shm.

Parity: ATorch ``atorch/optimizers/adam_offload.py`` (``PartitionAdam``:
optimizer state swapped between host and device around the step).
"""

import math
import os
from typing import Optional

import torch

from ..parallel.flat import ALIGN, FlatParams


class CPUOffloadAdamW(torch.optim.Optimizer):
    def __init__(self, flat: FlatParams, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01,
                 max_grad_norm: Optional[float] = None, chunk_elems: int = 32 << 20, threads: Optional[int] = None):
        if flat.dtype not in (torch.bfloat16, torch.float32):
            raise TypeError("CPUOffloadAdamW needs bf16 or fp32 flat parameters")
        super().__init__([flat.data], dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self.flat = flat
        self.max_grad_norm = max_grad_norm
        self.grad_scale = 1.0
        self.chunk = max(ALIGN, chunk_elems // ALIGN * ALIGN)
        self.threads = threads or max(1, min(32, (os.cpu_count() or 8) // 2))
        self.cuda = flat.data.is_cuda
        pin = self.cuda
        n = flat.numel
        self.master = torch.empty(n, dtype=torch.float32, pin_memory=pin)
        self.master.copy_(flat.data.float().cpu() if self.cuda else flat.data.float())
        self.exp_avg = torch.zeros(n, dtype=torch.float32, pin_memory=pin)
        self.exp_avg_sq = torch.zeros(n, dtype=torch.float32, pin_memory=pin)
        if self.cuda:
            self.grad_host = torch.empty(n, dtype=flat.grad.dtype, pin_memory=True)
            self.param_host = torch.empty(n, dtype=flat.dtype, pin_memory=True)
            self.d2h = torch.cuda.Stream(flat.data.device)
            self.h2d = torch.cuda.Stream(flat.data.device)
        self.step_count = 0
        # decay mask: one byte per 64-element block (FlatParams convention)
        self._mask = flat.decay_mask.cpu()

    def zero_grad(self, set_to_none: bool = False):
        self.flat.zero_grad()

    def _runs(self, s: int, e: int):
        """Split [s, e) into maximal runs with a constant weight-decay flag."""
        m = self._mask
        b0, b1 = s // ALIGN, (e + ALIGN - 1) // ALIGN
        out, start, cur = [], s, int(m[b0]) if b0 < m.numel() else 1
        for b in range(b0 + 1, b1):
            flag = int(m[b]) if b < m.numel() else 1
            if flag != cur:
                out.append((start, b * ALIGN, cur))
                start, cur = b * ALIGN, flag
        out.append((start, e, cur))
        return out

    def _grad_scale(self) -> float:
        scale = self.grad_scale
        if self.max_grad_norm:
            g = self.flat.grad
            norm = float(torch.linalg.vector_norm(g.float() if g.dtype != torch.float32 else g)) * scale
            if math.isfinite(norm) and norm > self.max_grad_norm:
                scale *= self.max_grad_norm / (norm + 1e-6)
        return scale

    @torch.no_grad()
    def step(self, closure=None):
        from .. import _native

        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        lib = _native.runtime()
        grp = self.param_groups[0]
        b1, b2 = grp["betas"]
        self.step_count += 1
        t = self.step_count
        bc1, bc2 = 1 - b1 ** t, 1 - b2 ** t
        gscale = self._grad_scale()
        n = self.flat.numel
        chunks = [(s, min(n, s + self.chunk)) for s in range(0, n, self.chunk)]
        gsrc = self.grad_host if self.cuda else self.flat.grad
        g_bf16 = int(gsrc.dtype == torch.bfloat16)
        out_bf16 = self.flat.dtype == torch.bfloat16
        if self.cuda:
            cur = torch.cuda.current_stream()
            self.d2h.wait_stream(cur)
            evs = []
            with torch.cuda.stream(self.d2h):
                for s, e in chunks:
                    self.grad_host[s:e].copy_(self.flat.grad[s:e], non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(self.d2h)
                    evs.append(ev)
            # weights must not be overwritten while the compute stream may still read them
            self.h2d.wait_stream(cur)
        esz_g = gsrc.element_size()
        for ci, (s, e) in enumerate(chunks):
            if self.cuda:
                evs[ci].synchronize()
            pout = self.param_host if (self.cuda and out_bf16) else None
            for rs, re_, decay in self._runs(s, e):
                lib.dw_cpu_adamw(self.master.data_ptr() + 4 * rs, gsrc.data_ptr() + esz_g * rs, g_bf16,
                                 self.exp_avg.data_ptr() + 4 * rs, self.exp_avg_sq.data_ptr() + 4 * rs,
                                 (pout.data_ptr() + 2 * rs) if pout is not None else None, re_ - rs,
                                 float(grp["lr"]), float(b1), float(b2), float(grp["eps"]),
                                 float(grp["weight_decay"]) if decay else 0.0, float(bc1), float(bc2),
                                 float(gscale), self.threads)
            if self.cuda:
                with torch.cuda.stream(self.h2d):
                    src = self.param_host[s:e] if out_bf16 else self.master[s:e]
                    self.flat.data[s:e].copy_(src, non_blocking=True)
            else:
                self.flat.data[s:e].copy_(self.master[s:e])
        if self.cuda:
            torch.cuda.current_stream().wait_stream(self.h2d)
        return loss

    def state_dict(self):
        return {"step": self.step_count, "master": self.master, "exp_avg": self.exp_avg,
                "exp_avg_sq": self.exp_avg_sq, "param_groups": [{k: v for k, v in g.items() if k != "params"}
                                                                for g in self.param_groups]}

    def load_state_dict(self, sd):
        self.step_count = int(sd["step"])
        self.master.copy_(sd["master"])
        self.exp_avg.copy_(sd["exp_avg"])
        self.exp_avg_sq.copy_(sd["exp_avg_sq"])
        for g, s in zip(self.param_groups, sd["param_groups"]):
            g.update(s)
        self.flat.data.copy_(self.master.to(self.flat.data.device, self.flat.dtype))
