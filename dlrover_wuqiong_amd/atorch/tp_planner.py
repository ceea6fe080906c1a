"""Automatic tensor-parallel plans for arbitrary models (graph-traced).

``auto_accelerate``'s tensor_parallel used to match a fixed list of Linear
leaf names (q_proj, up_proj, ...), silently leaving any other naming
unsharded.  This planner traces the model with ``torch.fx`` and finds the
Megatron pattern structurally:

  * a *column* Linear's output may only flow through feature-local ops --
    elementwise activations / products of other column outputs of the same
    block (SwiGLU), head views / transposes / splits, attention (matmul,
    softmax, SDPA, dropout), dtype casts -- and must end in *row* Linears;
  * a row Linear's input must come only from column Linears of the block
    (so its input features are exactly the concatenated column shards).

Every such block becomes ``ColwiseParallel`` for its column Linears and
``RowwiseParallel`` for its sinks (DTensor, torch.distributed.tensor.parallel):
one all-reduce per block in forward, one in backward.  Anything the tracer
cannot prove safe (layer norms, residual adds, reductions over features,
data-dependent control flow) is left replicated.

Parity: ATorch ``modules/distributed_modules/compilers/tp_compiler/
tp_compiler.py`` (graph-traced sharding planner); re-designed on torch.fx +
DTensor instead of ATorch's own tracer and TP layers.
"""

import operator
from typing import Dict, List, Optional, Set

import torch
import torch.fx as fx
import torch.nn as nn
import torch.nn.functional as F

from ..common.log import logger

# ops whose output features are a function of the SAME features of their
# inputs (shard-local when the feature dimension is split across ranks)
_LOCAL_FUNCS = {
    F.relu, F.gelu, F.silu, F.sigmoid, F.tanh, F.softmax, F.dropout, torch.relu, torch.sigmoid, torch.tanh,
    torch.softmax, F.scaled_dot_product_attention, torch.matmul, torch.bmm, torch.transpose, torch.permute,
    torch.reshape, torch.flatten, torch.chunk, torch.split, torch.unbind, torch.exp, operator.getitem,
    operator.mul, operator.truediv, torch.mul, torch.div, torch.einsum, F.leaky_relu, F.elu, F.mish,
}
_LOCAL_METHODS = {"view", "reshape", "transpose", "permute", "contiguous", "split", "chunk", "unbind",
                  "softmax", "float", "to", "type_as", "half", "bfloat16", "relu", "sigmoid", "tanh", "mul",
                  "div", "flatten", "unflatten", "matmul", "masked_fill", "exp", "__getitem__"}
_LOCAL_MODULES = (nn.ReLU, nn.GELU, nn.SiLU, nn.Sigmoid, nn.Tanh, nn.Dropout, nn.Softmax, nn.Identity,
                  nn.LeakyReLU, nn.Mish)


def _is_linear(gm: fx.GraphModule, n: fx.Node) -> bool:
    return n.op == "call_module" and isinstance(gm.get_submodule(n.target), nn.Linear)


def _is_local(gm: fx.GraphModule, n: fx.Node) -> bool:
    if n.op == "call_function":
        return n.target in _LOCAL_FUNCS
    if n.op == "call_method":
        return n.target in _LOCAL_METHODS
    if n.op == "call_module":
        return isinstance(gm.get_submodule(n.target), _LOCAL_MODULES)
    return False


def _tensor_inputs(n: fx.Node) -> List[fx.Node]:
    out = []

    def visit(a):
        if isinstance(a, fx.Node):
            out.append(a)
        elif isinstance(a, (list, tuple)):
            for x in a:
                visit(x)
        elif isinstance(a, dict):
            for x in a.values():
                visit(x)

    visit(n.args)
    visit(n.kwargs)
    return out


def _is_shape_query(gm: fx.GraphModule, n: fx.Node) -> bool:
    """x.size() / x.dim() / x.shape: read metadata, carry no feature data."""
    if n.op == "call_method" and n.target in ("size", "dim"):
        return True
    return n.op == "call_function" and n.target is getattr and len(n.args) > 1 and n.args[1] in ("shape",
                                                                                                 "dtype", "device")


def _is_constant(n: fx.Node) -> bool:
    return n.op == "get_attr" or (n.op == "call_function" and n.target in (torch.ones, torch.zeros, torch.full,
                                                                           torch.arange, torch.tril, torch.triu))


def _grow_block(gm: fx.GraphModule, seed: fx.Node, claimed: Set[fx.Node]):
    """(column Linears, row Linears) of the Megatron block around ``seed``,
    or None when any data flow would mix sharded and replicated features."""
    cols, rows, region = {seed}, set(), set()
    work = [seed]

    def back(a: fx.Node) -> bool:
        # make ``a`` column-derived: every path back ends in a fresh Linear
        # (a new column) or a constant, through feature-local ops only
        if a in cols or a in region:
            return True
        if _is_linear(gm, a):
            if a in rows or a in claimed:
                return False
            cols.add(a)
            work.append(a)
            return True
        if _is_constant(a):
            return True
        if _is_shape_query(gm, a):
            return True
        if _is_local(gm, a):
            region.add(a)
            work.append(a)
            return all(back(x) for x in _tensor_inputs(a))
        return False

    while work:
        n = work.pop()
        for u in list(n.users):
            if u in region or u in rows or u in cols or _is_shape_query(gm, u):
                continue
            if _is_linear(gm, u):
                rows.add(u)  # sharded features into a Linear: its input dim is split
                continue
            if not _is_local(gm, u):
                return None
            region.add(u)
            work.append(u)
            if not all(back(a) for a in _tensor_inputs(u)):
                return None
    if not rows:
        return None
    for r in rows:
        if any(a not in region and a not in cols for a in _tensor_inputs(r)):
            return None
    # head counts baked into views of the sharded features: view(B, S, nh, -1)
    # splits the (now 1/tp) feature dim -- nh must shrink with it
    heads = set()
    for n in region:
        if (n.op == "call_method" and n.target in ("view", "reshape")) or (
                n.op == "call_function" and n.target is torch.reshape):
            dims = n.args[1:] if n.op == "call_method" else (n.args[1] if len(n.args) > 1 else ())
            if len(dims) == 1 and isinstance(dims[0], (list, tuple)):
                dims = dims[0]
            if len(dims) >= 2 and isinstance(dims[-2], int) and dims[-2] > 1:
                heads.add(dims[-2])
    return cols, rows, heads


def trace_tp_plan(model: nn.Module, heads_out: Optional[Dict[str, Set[int]]] = None
                  ) -> Optional[Dict[str, str]]:
    """{linear module name: "colwise" | "rowwise"} or None if the model does
    not trace.  ``heads_out`` receives {owner module name: head counts its
    views hard-code} (divide those attributes by the TP degree)."""
    try:
        gm = fx.symbolic_trace(model)
    except Exception as e:  # data-dependent control flow, unsupported ops
        logger.info(f"tp planner: {type(model).__name__} does not trace ({type(e).__name__}); no structural plan")
        return None
    plan: Dict[str, str] = {}
    claimed: Set[fx.Node] = set()
    for seed in [n for n in gm.graph.nodes if _is_linear(gm, n)]:
        if seed in claimed:
            continue
        blk = _grow_block(gm, seed, claimed)
        if blk is None:
            continue
        cols, rows, heads = blk
        if heads_out is not None and heads:
            names = [n.target for n in cols | rows]
            owner = names[0].rsplit(".", 1)[0] if "." in names[0] else ""
            while owner and not all(x.startswith(owner + ".") for x in names):
                owner = owner.rsplit(".", 1)[0] if "." in owner else ""
            heads_out.setdefault(owner, set()).update(heads)
        for c in cols:
            plan[c.target] = "colwise"
        for r in rows:
            plan[r.target] = "rowwise"
        claimed |= cols | rows
    return plan


def auto_tp_plan(model: nn.Module, heads_out: Optional[Dict[str, Set[int]]] = None) -> Dict[str, object]:
    """DTensor parallelize plan {fully-qualified name: ColwiseParallel() |
    RowwiseParallel()} found structurally, per traceable submodule when the
    whole model does not trace (e.g. HF decoder layers under a generate loop)."""
    from torch.distributed.tensor.parallel import ColwiseParallel, RowwiseParallel

    def to_styles(p: Dict[str, str], prefix: str) -> Dict[str, object]:
        return {(prefix + "." + k) if prefix else k: (ColwiseParallel() if v == "colwise" else RowwiseParallel())
                for k, v in p.items()}

    def merge_heads(h: Dict[str, Set[int]], prefix: str):
        if heads_out is not None:
            for k, v in h.items():
                key = ".".join(x for x in (prefix, k) if x)
                heads_out.setdefault(key, set()).update(v)

    h: Dict[str, Set[int]] = {}
    whole = trace_tp_plan(model, h)
    if whole:
        merge_heads(h, "")
        return to_styles(whole, "")
    out: Dict[str, object] = {}
    done: List[str] = []
    for name, mod in model.named_modules():
        if not name or any(name.startswith(d + ".") for d in done):
            continue
        if not any(isinstance(c, nn.Linear) for c in mod.modules()) or isinstance(mod, nn.Linear):
            continue
        h = {}
        p = trace_tp_plan(mod, h)
        if p:
            out.update(to_styles(p, name))
            merge_heads(h, name)
            done.append(name)
    return out


def shrink_head_attributes(model: nn.Module, heads: Dict[str, Set[int]], tp: int) -> int:
    """Divide the integer attributes of each owner module that equal a head
    count its views hard-code (``self.nh``, ``self.num_heads`` ...)."""
    n = 0
    for owner, counts in heads.items():
        mod = model.get_submodule(owner) if owner else model
        for sub in mod.modules():
            for k, v in list(vars(sub).items()):
                if isinstance(v, int) and not isinstance(v, bool) and v in counts and v % tp == 0:
                    setattr(sub, k, v // tp)
                    n += 1
    return n
