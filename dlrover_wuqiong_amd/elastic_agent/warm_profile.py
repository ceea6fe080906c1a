"""Warm profile: what a replacement worker's first training step will need,
recorded by the live worker and replayed by the import-mode standby.

An import-mode standby (``standby.py``) has imported torch, initialised HIP
and pinned the checkpoint shm, but it does not know the training script's
model.  A restarted worker's first step then pays, on top of its compute:

* the GEMM library's first call per problem (hipBLASLt heuristic query and
  the lazy load of each kernel's code object);
* fresh device memory for every activation / gradient / workspace block
  (the driver clears new VRAM pages before handing them out);
* the first launch of every code object of this package's kernel library.

The live worker records those once -- every distinct GEMM signature
(op, shapes, strides, dtypes) of ONE optimizer step, observed through a
``TorchDispatchMode`` that is only active for that step, plus its peak
caching-allocator footprint -- into ``warm_profile.<local_rank>.json`` in the
agent's control directory.  The standby replays the GEMMs on scratch tensors,
touches every kernel code object, and reserves the recorded footprint in its
caching allocator, all while it waits.  Activated, it trains its first step
from a warm allocator and warm GEMM/kernel caches.

Recording starts after the worker's first flash-checkpoint save (the model
and optimizer exist, warm-up is over) and stops at the end of the next
optimizer step; ``DWAMD_WARM_PROFILE=0`` disables it.  The reference's agent
always cold-starts workers (``training.py:580-645,704``); this is an MI355X
restart-latency optimisation measured by ``bench.py`` (``import_mode``).
"""

import json
import os
import sys
import threading
import time
from typing import Dict, List, Optional

PROFILE_PREFIX = "warm_profile."
_VERSION = 1

_state = {"saves": 0, "recorder": None, "hook": None, "done": False}
_lock = threading.Lock()


def profile_path(ctl: str, local_rank) -> str:
    return os.path.join(ctl, f"{PROFILE_PREFIX}{local_rank}.json")


def _enabled() -> bool:
    return (os.environ.get("DWAMD_WARM_PROFILE", "1") == "1" and bool(os.environ.get("DWAMD_AGENT_CTL_DIR"))
            and os.environ.get("DWAMD_STANDBY", "0") != "1")


def _gemm_ops():
    import torch

    aten = torch.ops.aten
    ops = [aten.mm.default, aten.addmm.default, aten.bmm.default, aten.baddbmm.default, aten.addmm_.default,
           aten.mm.out, aten.addmm.out, aten.bmm.out]
    if hasattr(aten, "_scaled_mm"):
        ops.append(aten._scaled_mm.default)
    return {op: (op._overloadpacket.__name__, op._overloadname) for op in ops}


def _enc(x, device_type: str = "cuda"):
    import torch

    if isinstance(x, torch.Tensor):
        if x.device.type != device_type:
            return {"cpu_scalar": float(x.item())} if x.numel() == 1 else None
        return {"t": list(x.shape), "s": list(x.stride()), "d": str(x.dtype).replace("torch.", ""),
                "o": int(x.storage_offset())}
    if isinstance(x, (bool, int, float)) or x is None:
        return {"v": x}
    if isinstance(x, torch.dtype):
        return {"dt": str(x).replace("torch.", "")}
    if isinstance(x, (list, tuple)) and all(isinstance(v, (int, float)) for v in x):
        return {"l": list(x)}
    return None  # not replayable


# Non-GEMM aten ops are recorded too (their kernels' code objects load at the
# first launch) -- except ops whose replay on scratch data could do harm or
# is pointless: random number generation, host syncs, pure views /
# metadata, collectives (other namespaces are never recorded).
_SKIP_WORDS = ("rand", "normal", "uniform", "bernoulli", "dropout", "exponential", "multinomial", "random",
               "_local_scalar_dense", "nonzero", "unique", "masked_select", "item", "resize", "set_",
               "record_stream", "_foreach")
_VIEW_OPS = {"view", "_unsafe_view", "as_strided", "t", "transpose", "permute", "expand", "slice", "select",
             "unsqueeze", "squeeze", "reshape", "alias", "detach", "unbind", "split", "split_with_sizes",
             "chunk", "narrow", "lift_fresh", "view_as_real", "view_as_complex", "_reshape_alias",
             "empty", "empty_like", "empty_strided", "new_empty", "new_empty_strided", "is_same_size"}


def _warm_op(name: str) -> bool:
    return name not in _VIEW_OPS and not any(w in name for w in _SKIP_WORDS)


def _make_recorder(device_type: str = "cuda"):
    import torch
    from torch.utils._python_dispatch import TorchDispatchMode

    ops = _gemm_ops()

    class GemmRecorder(TorchDispatchMode):
        """Records the distinct GEMM calls of the step it is active for."""

        def __init__(self):
            super().__init__()
            self.seen: Dict[str, dict] = {}
            self.other: Dict[str, dict] = {}
            self.calls = 0

        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            kwargs = kwargs or {}
            name = ops.get(func)
            gemm = name is not None
            if name is None and getattr(func, "namespace", "") == "aten":
                pk = func._overloadpacket.__name__
                name = (pk, func._overloadname) if _warm_op(pk) else None
            if name is not None and name[1] != "out":
                self.calls += gemm
                ea = [_enc(a, device_type) for a in args]
                ek = {k: _enc(v, device_type) for k, v in kwargs.items()}
                # at least one device tensor (a kernel runs), everything encodable
                dev = any(isinstance(e, dict) and "t" in e for e in ea + list(ek.values()))
                if dev and all(e is not None for e in ea) and all(e is not None for e in ek.values()):
                    key = json.dumps([name, ea, ek], sort_keys=True)
                    table = self.seen if gemm else self.other
                    if key not in table:
                        table[key] = {"op": name[0], "ov": name[1], "args": ea, "kwargs": ek}
            return func(*args, **kwargs)

    return GemmRecorder()


def _write(rec, t0: float):
    import torch

    ctl = os.environ.get("DWAMD_AGENT_CTL_DIR", "")
    lr = os.environ.get("LOCAL_RANK", "0")
    dev = torch.cuda.current_device()
    prof = {"version": _VERSION, "pid": os.getpid(), "device": dev, "recorded_s": round(time.time() - t0, 3),
            "gemm_calls": rec.calls, "gemms": list(rec.seen.values()), "ops": list(rec.other.values()),
            "max_reserved": int(torch.cuda.max_memory_reserved(dev)),
            "reserved": int(torch.cuda.memory_reserved(dev)),
            "max_allocated": int(torch.cuda.max_memory_allocated(dev)),
            # checkpoint staging inside max_reserved (the standby holds its own)
            "staging_reserved": int(_state.get("staging", 0))}
    path = profile_path(ctl, lr)
    with open(path + ".tmp", "w") as f:
        json.dump(prof, f)
    os.replace(path + ".tmp", path)


def _stop(*_a, **_k):
    """Optimizer post-step hook: end the recording after one full step."""
    import torch

    with _lock:
        rec = _state["recorder"]
        if rec is None:
            return
        top = _top_mode()
        if top is not rec:
            return  # someone else's mode is on top (unbalanced): retry at the next step
        rec.__exit__(None, None, None)
        _state["recorder"] = None
        _state["done"] = True
        if _state["hook"] is not None:
            _state["hook"].remove()
            _state["hook"] = None
    try:
        _write(rec, _state.get("t0", time.time()))
    except Exception as e:  # never fatal
        print(f"[warm_profile] not written: {e}", file=sys.stderr)


def _top_mode():
    from torch.utils._python_dispatch import _get_current_dispatch_mode

    return _get_current_dispatch_mode()


def on_save(staging_bytes: int = 0):
    """Called by the checkpoint engine after every flash save (training
    thread): the first save arms the recorder for the next optimizer step.
    ``staging_bytes``: snapshot staging the caching allocator holds for the
    copier (subtracted from the recorded footprint)."""
    if _state["done"] or not _enabled():
        return
    _state["staging"] = max(int(staging_bytes), int(_state.get("staging", 0)))
    import torch

    if not torch.cuda.is_available():
        return
    with _lock:
        _state["saves"] += 1
        if _state["saves"] != 1 or _state["recorder"] is not None:
            return
        from torch.optim.optimizer import register_optimizer_step_post_hook

        rec = _make_recorder()
        rec.__enter__()
        _state["recorder"] = rec
        _state["t0"] = time.time()
        _state["hook"] = register_optimizer_step_post_hook(_stop)


# ------------------------------------------------------------------ replay
def _dec(e, device):
    import torch

    if "t" in e:
        dt = getattr(torch, e["d"])
        need = e["o"] + 1 + sum((n - 1) * s for n, s in zip(e["t"], e["s"]) if n > 0)
        base = torch.empty(max(need, 1), dtype=dt, device=device) if dt.is_floating_point else torch.zeros(
            max(need, 1), dtype=dt, device=device)
        if dt.is_floating_point and dt.itemsize >= 2:
            base.normal_()
        elif dt.is_floating_point:
            base.view(torch.uint8).fill_(0x38)  # fp8: a finite value (1.0-ish)
        return base.as_strided(e["t"], e["s"], e["o"])
    if "cpu_scalar" in e:
        return torch.tensor(e["cpu_scalar"])
    if "dt" in e:
        return getattr(torch, e["dt"])
    if "l" in e:
        return e["l"]
    return e.get("v")


def replay(prof: dict, device=None, repeats: int = 2) -> dict:
    """Run every recorded GEMM ``repeats`` times, and every other recorded
    op once, on scratch tensors (floats random, integers zero -- so index
    operands stay in range): loads the GEMM library's heuristics and the
    kernels' code objects in this process.
    Returns ``{"gemms": n, "ops": m, "failed": k, "sec": s}``."""
    import torch

    device = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    t0 = time.perf_counter()
    n = failed = m = 0
    for g in prof.get("ops", []):
        try:
            op = getattr(getattr(torch.ops.aten, g["op"]), g.get("ov", "default"))
            args = [_dec(a, device) for a in g["args"]]
            kwargs = {k: _dec(v, device) for k, v in g["kwargs"].items()}
            op(*args, **kwargs)
            m += 1
            del args, kwargs
        except Exception:
            failed += 1
    for g in prof.get("gemms", []):
        try:
            op = getattr(getattr(torch.ops.aten, g["op"]), g.get("ov", "default"))
        except AttributeError:
            failed += 1
            continue
        try:
            args = [_dec(a, device) for a in g["args"]]
            kwargs = {k: _dec(v, device) for k, v in g["kwargs"].items()}
            for _ in range(repeats):
                op(*args, **kwargs)
            n += 1
            del args, kwargs
        except Exception:
            failed += 1
    if torch.device(device).type == "cuda":
        torch.cuda.synchronize(device)
    return {"gemms": n, "ops": m, "failed": failed, "sec": round(time.perf_counter() - t0, 3)}


def preload_kernel_library() -> float:
    """Force-load every code object of this package's kernel library (with
    deferred loading a fat binary is loaded at its first launch)."""
    t0 = time.perf_counter()
    try:
        from .._native import kernels

        L = kernels(required=False)
        if L is not None and hasattr(L, "dw_preload_code_objects"):
            L.dw_preload_code_objects()
    except Exception as e:  # never fatal
        print(f"[warm_profile] kernel preload skipped: {e}", file=sys.stderr)
    return time.perf_counter() - t0


def load(ctl: str, local_rank) -> Optional[dict]:
    try:
        with open(profile_path(ctl, local_rank)) as f:
            prof = json.load(f)
        return prof if prof.get("version") == _VERSION else None
    except (OSError, ValueError):
        return None


def reserve_bytes(prof: Optional[dict], state_bytes: int, factor: float = 1.25) -> int:
    """Bytes the standby should hold in its caching allocator: the worker's
    recorded peak footprint, else ~its checkpoint payload (model + optimizer)."""
    if prof and prof.get("max_reserved"):
        return max(0, int(prof["max_reserved"]) - int(prof.get("staging_reserved", 0)))
    return int(state_bytes * factor)


def summary(prof: Optional[dict]) -> List:
    if not prof:
        return []
    return [g["op"] for g in prof.get("gemms", [])]
