"""Direct gradient accumulation into flat gradient buffers.

Parameters managed by ``parallel.flat.FlatParams`` (with
``direct_grads=True``) carry ``_dwamd_direct``: their ``.grad`` is a view of
the flat gradient buffer, zeroed lazily once per step (``claim()``: the
first contribution after ``zero_grad`` overwrites, ``parallel/flat.py``).  The fused ops accumulate
into it themselves -- weight GEMMs with ``addmm_`` (beta = 1: the hipBLASLt
epilogue does the add), bias / norm-weight reductions with an accumulating
finish kernel -- and return ``None`` to autograd.  That removes one
elementwise ``grad += g`` pass per parameter per micro-batch (hundreds of
kernels per step) and the temporary ``g``.  Autograd still fires the
parameter's post-accumulate hook after the op's backward returns (the grad
it hands over is undefined), which is what ``FlatDDP`` counts.  The optional
``_dwamd_grad_ready`` callback is an extra, earlier readiness signal for
code that wants it; ``FlatDDP`` deliberately does not use it (it would count
each parameter twice).
"""

from typing import Optional

import torch


def direct_grad(p: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    if p is None or not getattr(p, "_dwamd_direct", False):
        return None
    g = p.grad
    if g is None or not g.is_contiguous():
        return None
    return g


def claim(p: Optional[torch.Tensor]) -> bool:
    """The caller is about to write ``p``'s direct gradient: True when the
    write must OVERWRITE (first contribution since a lazy ``zero_grad``,
    ``parallel/flat.py``), False when it accumulates."""
    st = getattr(p, "_dwamd_flat", None)
    return st.claim(p._dwamd_idx) if st is not None else False


def claim_all(*ps) -> bool:
    """One writer for several parameters (e.g. a norm's weight and bias):
    True (overwrite) only if all are fresh; a mixed set zeroes its fresh
    members and accumulates."""
    ps = [p for p in ps if p is not None]
    fresh = [claim(p) for p in ps]
    if all(fresh):
        return bool(fresh)
    for p, f in zip(ps, fresh):
        if f:
            p.grad.zero_()
    return False


def notify(p: Optional[torch.Tensor]):
    if p is None:
        return
    cb = getattr(p, "_dwamd_grad_ready", None)
    if cb is not None:
        cb(p)
