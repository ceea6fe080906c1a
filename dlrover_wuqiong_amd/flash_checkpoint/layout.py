"""State-dict -> shared-memory layout planning.

A checkpoint "shard" is one byte payload in a POSIX shm segment plus a small
metadata tree.  The tree mirrors the user's nested state dict (dicts, lists,
tuples) with every tensor replaced by a :class:`TensorMeta` (shape, dtype,
byte offset into the payload) and every other leaf kept as-is.

MI355X-first detail: tensors are *coalesced by storage*.  Every parameter /
optimizer state of a model trained by this framework is a view into a few
large flat buffers, so the ~N hundred tensors of a state dict collapse into a
handful of contiguous byte extents.  A snapshot is then a few long HBM->HBM
(or HBM->pinned-host) streams instead of one copy per tensor, and the same
extents are what the agent persists.

Parity: reference ``ckpt_saver.py:94-206`` (``_traverse_state_dict``,
``TensorMeta``, ``_create_tensor_meta``) - same tree semantics, different
packing.
"""

from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Tuple

import torch

ALIGN = 4096  # extents start on a page boundary (pinned DMA + O_DIRECT friendly)


def _align(x: int, a: int = ALIGN) -> int:
    return (x + a - 1) // a * a


@dataclass
class TensorMeta:
    shape: Tuple[int, ...] = ()
    dtype: torch.dtype = torch.float32
    element_size: int = 0
    numel: int = 0
    offset: int = 0  # byte offset in the shard payload
    device: str = "cpu"  # device type at save time ("cuda" / "cpu")

    @property
    def nbytes(self) -> int:
        return self.numel * self.element_size


@dataclass
class Extent:
    """A contiguous byte range of one source storage mapped to the payload."""

    src_ptr: int  # address of the first byte in the source storage
    nbytes: int
    offset: int  # payload offset
    device: str  # "cuda" or "cpu"
    keepalive: Any = None  # the tensor whose storage this is (for CPU copies)


@dataclass
class Layout:
    meta_tree: Any = None
    extents: List[Extent] = field(default_factory=list)
    total_bytes: int = 0
    signature: Tuple = ()  # identifies a layout that can be reused

    def gpu_extents(self):
        return [e for e in self.extents if e.device == "cuda"]

    def cpu_extents(self):
        return [e for e in self.extents if e.device != "cuda"]

    @property
    def gpu_end(self) -> int:
        """End of the device region: plan_layout places every device storage
        before every host one, so [0, gpu_end) is what a staging buffer's
        PCIe flush may write -- host tensors (copied to shm directly) lie
        beyond it and are never overwritten by staging bytes."""
        return max((e.offset + e.nbytes for e in self.extents if e.device == "cuda"), default=0)


def traverse(value: Any, visitor: Callable[[Any], Any]) -> Any:
    """Rebuild ``value`` with ``visitor`` applied to every non-container leaf."""
    if isinstance(value, dict):
        items = [(k, traverse(v, visitor)) for k, v in value.items()]
        try:
            return type(value)(items)
        except Exception:
            return dict(items)
    if isinstance(value, list):
        return [traverse(v, visitor) for v in value]
    if isinstance(value, tuple) and not hasattr(value, "_fields"):
        return tuple(traverse(v, visitor) for v in value)
    return visitor(value)


def iter_leaves(value: Any, out: Optional[list] = None) -> list:
    if out is None:
        out = []
    if isinstance(value, dict):
        for v in value.values():
            iter_leaves(v, out)
    elif isinstance(value, (list, tuple)) and not hasattr(value, "_fields"):
        for v in value:
            iter_leaves(v, out)
    else:
        out.append(value)
    return out


def _storage_key(t: torch.Tensor):
    st = t.untyped_storage()
    return (t.device.type, t.device.index, st.data_ptr())


MERGE_GAP = 1 << 20  # bridge gaps (alignment padding) up to 1 MiB inside one storage


class LayoutCache:
    """Re-plans only when the tensor set changes.

    A training loop checkpoints the same tensors every time (same storages,
    same addresses); only non-tensor leaves (step counters, lr, ...) change.
    The cache key is the (address, numel, dtype) sequence of the tensor
    leaves; on a hit the TensorMetas and extents are reused and only the
    meta tree is rebuilt (cheap, no allocation per tensor).
    """

    def __init__(self):
        self._key = None
        self._layout: Optional[Layout] = None
        self._metas: List[TensorMeta] = []

    def cached(self) -> Optional[Layout]:
        """The layout of the previous plan (its tensors are kept alive by the
        caller), for a speculative snapshot enqueued before :meth:`plan`
        verifies that ``state_dict`` still matches it."""
        return self._layout

    def plan(self, state_dict: Any) -> Tuple[Layout, List[torch.Tensor]]:
        if self._layout is not None:
            try:
                tree, tensors = self._hit(state_dict)
                lay = self._layout
                return Layout(meta_tree=tree, extents=lay.extents, total_bytes=lay.total_bytes,
                              signature=lay.signature), tensors
            except _Miss:
                pass
        key: List[Tuple] = []

        def collect(v):
            if torch.is_tensor(v):
                key.append((v.data_ptr(), v.numel(), v.dtype, v.is_contiguous()))
            return v

        traverse(state_dict, collect)
        layout, tens = plan_layout(state_dict)
        # temporaries of non-contiguous leaves are never reused
        all_contig = all(k[3] for k in key)
        self._key = key if all_contig else None
        self._layout = layout if all_contig else None
        self._metas = [m for m in iter_leaves(layout.meta_tree) if isinstance(m, TensorMeta)]
        return layout, tens

    def _hit(self, state_dict: Any):
        """One pass over ``state_dict``: verify every tensor leaf against the
        cached key and rebuild the meta tree (same shape rules as
        :func:`traverse`).  Raises ``_Miss`` on the first mismatch.  Lists of
        plain scalars (optimizer ``param_groups[...]["params"]``) are copied
        without per-element recursion -- a state dict of a few thousand
        tensors is re-planned in about a millisecond."""
        key, metas = self._key, self._metas
        n = len(key)
        tensors: List[torch.Tensor] = []
        T = torch.Tensor
        append = tensors.append

        def leaf(v):
            # a tensor leaf: verified against the cached key, replaced by its meta
            i = len(tensors)
            if i >= n:
                raise _Miss
            k = key[i]
            if v.data_ptr() != k[0] or v.numel() != k[1] or v.dtype != k[2] or not v.is_contiguous():
                raise _Miss
            append(v)
            return metas[i]

        def rec_dict(v, tv):
            # tensors handled inline (no call per leaf): the bulk of a state dict
            out = {}
            for k, x in v.items():
                tx = type(x)
                out[k] = leaf(x) if (tx is T or tx is torch.nn.Parameter) else (
                    x if tx in _SCALARS else rec(x))
            if tv is dict:
                return out
            try:
                return tv(out.items())
            except Exception:
                return out

        def rec(v):
            tv = type(v)
            if tv is T or tv is torch.nn.Parameter:
                return leaf(v)
            if tv in _SCALARS:
                return v
            if tv is dict or isinstance(v, dict):
                return rec_dict(v, tv)
            if tv is list or isinstance(v, list):
                if all(type(x) in _SCALARS for x in v):
                    return list(v)
                return [rec(x) for x in v]
            if isinstance(v, tuple) and not hasattr(v, "_fields"):
                return tuple(rec(x) for x in v)
            if isinstance(v, T):
                return leaf(v)
            return v

        tree = rec(state_dict)
        if len(tensors) != n:
            raise _Miss
        return tree, tensors


_SCALARS = frozenset((int, float, str, bool, type(None)))


class _Miss(Exception):
    pass


def plan_layout(state_dict: Any) -> Tuple[Layout, List[torch.Tensor]]:
    """Plan where every tensor of ``state_dict`` lives in the payload.

    Returns the layout and the list of tensors in leaf order (contiguous
    versions of non-contiguous tensors are created here and must be kept alive
    until the copy is done).
    """
    tensors: List[torch.Tensor] = []

    def collect(v):
        if torch.is_tensor(v):
            t = v.detach()
            if not t.is_contiguous():
                t = t.contiguous()
            tensors.append(t)
        return v

    traverse(state_dict, collect)

    # group byte ranges per storage
    groups: Dict[Any, List[Tuple[int, int, int]]] = {}  # key -> [(start_addr, end_addr, idx)]
    for i, t in enumerate(tensors):
        if t.numel() == 0:
            continue
        start = t.data_ptr()
        end = start + t.numel() * t.element_size()
        groups.setdefault(_storage_key(t), []).append((start, end, i))

    extents: List[Extent] = []
    tensor_offset: Dict[int, int] = {}
    cursor = 0
    # deterministic order: device storages first (the staging buffers' PCIe
    # flush covers one contiguous device region and must not write over
    # host tensors), then host ones; each by first appearance in the dict
    order = sorted(groups.items(), key=lambda kv: (kv[0][0] != "cuda", min(x[2] for x in kv[1])))
    for key, ranges in order:
        ranges.sort()
        merged: List[List[int]] = []  # [start, end, [idx...]]
        for s, e, i in ranges:
            if merged and s <= merged[-1][1] + MERGE_GAP:
                merged[-1][1] = max(merged[-1][1], e)
                merged[-1][2].append(i)
            else:
                merged.append([s, e, [i]])
        for s, e, idxs in merged:
            off = _align(cursor)
            dev = key[0]
            extents.append(Extent(src_ptr=s, nbytes=e - s, offset=off, device=dev,
                                  keepalive=tensors[idxs[0]]))
            for i in idxs:
                tensor_offset[i] = off + (tensors[i].data_ptr() - s)
            cursor = off + (e - s)

    counter = [0]

    def to_meta(v):
        if torch.is_tensor(v):
            i = counter[0]
            counter[0] += 1
            t = tensors[i]
            return TensorMeta(shape=tuple(t.shape), dtype=t.dtype, element_size=t.element_size(),
                              numel=t.numel(), offset=tensor_offset.get(i, 0), device=t.device.type)
        return v

    meta_tree = traverse(state_dict, to_meta)
    total = _align(cursor) if cursor else 0
    sig = tuple((m.shape, str(m.dtype), m.offset) for m in iter_leaves(meta_tree)
                if isinstance(m, TensorMeta))
    return Layout(meta_tree=meta_tree, extents=extents, total_bytes=total, signature=sig), tensors


def split_ranges(total: int, parts: int, align: int = ALIGN) -> List[Tuple[int, int]]:
    """Split [0, total) into ``parts`` page-aligned contiguous slices."""
    per = _align((total + parts - 1) // parts, align) if total else 0
    out = []
    for p in range(parts):
        b = min(total, p * per)
        e = min(total, b + per)
        out.append((b, e))
    return out


def intersect_extents(extents: List[Extent], lo: int, hi: int):
    """Yield (extent, payload_lo, payload_hi) pieces of extents inside [lo, hi)."""
    for e in extents:
        a = max(lo, e.offset)
        b = min(hi, e.offset + e.nbytes)
        if a < b:
            yield e, a, b


def tensors_from_payload(meta_tree: Any, buf, base_offset: int = 0) -> Any:
    """Zero-copy CPU tensors viewing a payload buffer (memoryview / bytes-like)."""

    def read(v):
        if isinstance(v, TensorMeta):
            if v.numel == 0:
                return torch.empty(v.shape, dtype=v.dtype)
            t = torch.frombuffer(buf, dtype=v.dtype, count=v.numel, offset=base_offset + v.offset)
            return t.view(v.shape)
        return v

    return traverse(meta_tree, read)
