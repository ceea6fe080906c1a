"""Maximal-update parametrization (muP): hyper-parameters tuned on a narrow
proxy model transfer to the wide production model.

How it works here:

1. ``set_base_shapes(model, base, delta)`` compares parameter shapes of the
   target model with a base-width model (and a delta-width model that tells
   which dimensions scale with width) and attaches ``p.infshape`` -- per
   dimension the base size and the actual size.
2. Parameters are classified by how many of their dims are "infinite"
   (scale with width): hidden matrices (2), vector-likes (1: embeddings,
   biases, norm weights, readout with a finite fan-out) and scalars (0).
3. Initialisation (``normal_``, ``xavier_*``, ``kaiming_*`` here, or
   ``MupLinear.mup_initial``) and the optimizers (``MuAdam``, ``MuSGD``)
   rescale per class with the width multiplier ``m = width / base_width``:

   ==============  ====================  =====================
   class           Adam lr               SGD lr
   ==============  ====================  =====================
   hidden (2 inf)  lr / m_fanin          lr * m_fanout/m_fanin
   vector (1 inf)  lr                    lr * m
   ==============  ====================  =====================

   Hidden-weight init std shrinks by ``1/sqrt(m_fanin)`` for constant-std
   samplers, and the readout (``MuReadout`` / ``OutputLayer``) divides its
   logits by ``m`` (initialised to zero by default).

Parity: ATorch ``atorch/mup`` (``infshape.py`` InfDim/InfShape, ``shape.py``
set_base_shapes/make_base_shapes/save/load, ``init.py`` samplers,
``module.py`` MupModule/MupLinear/QKVLayer/QLayer/OutputLayer, ``optim.py``
MuAdam/MuSGD).
"""

import math
from copy import copy
from typing import Dict, Iterable, Optional, Union

import torch
import torch.nn as nn
import torch.nn.functional as F
import yaml


# ------------------------------------------------------------- shapes
class InfDim:
    """One dimension: ``base_dim`` None means finite (does not scale)."""

    __slots__ = ("base_dim", "dim")

    def __init__(self, base_dim: Optional[int], dim: int):
        self.base_dim, self.dim = base_dim, dim

    def isinf(self) -> bool:
        return self.base_dim is not None

    def width_mult(self) -> float:
        return self.dim / self.base_dim if self.isinf() else 1.0

    def __eq__(self, other):
        return isinstance(other, InfDim) and (self.base_dim, self.dim) == (other.base_dim, other.dim)

    def __repr__(self):
        return f"InfDim({self.base_dim}, {self.dim})"


class InfShape(tuple):
    def ninf(self) -> int:
        return sum(d.isinf() for d in self)

    def fanin_fanout(self):
        """Linear/conv convention: weight [out, in, ...]."""
        if len(self) < 2:
            return None, self[0]
        return self[1], self[0]

    def width_mult(self) -> float:
        """Fan-in width multiplier for matrices, else the infinite dim's."""
        fi, fo = self.fanin_fanout()
        if fi is not None and fi.isinf():
            return fi.width_mult()
        for d in self:
            if d.isinf():
                return d.width_mult()
        return 1.0

    def fanin_fanout_mult_ratio(self) -> float:
        fi, fo = self.fanin_fanout()
        return (fi.width_mult() if fi is not None else 1.0) / fo.width_mult()

    @property
    def shape(self):
        return tuple(d.dim for d in self)

    @property
    def base_shape(self):
        return tuple(d.base_dim for d in self)

    def serialize(self):
        return {"base_shape": list(self.base_shape), "shape": list(self.shape)}

    @classmethod
    def deserialize(cls, d):
        return cls(InfDim(b, s) for b, s in zip(d["base_shape"], d["shape"]))

    @classmethod
    def from_base_shape(cls, bsh):
        return cls(InfDim(b, None) for b in bsh)


def zip_infshape(base_dims, dims, fin_if_same: bool = True) -> InfShape:
    out = []
    for b, d in zip(base_dims, dims):
        if isinstance(b, InfDim):
            b = b.base_dim
        out.append(InfDim(None if (fin_if_same and b == d) or b is None else b, d))
    return InfShape(out)


def get_shapes(model: nn.Module) -> Dict[str, tuple]:
    return {n: tuple(p.shape) for n, p in model.named_parameters()}


def get_infshapes(model: nn.Module) -> Dict[str, InfShape]:
    return {n: p.infshape for n, p in model.named_parameters()}


def make_base_shapes(base_shapes, delta_shapes, savefile: Optional[str] = None) -> Dict[str, list]:
    """Base shapes with the dims that differ between base and delta marked
    infinite; finite dims are stored as None."""
    base = base_shapes if isinstance(base_shapes, dict) else get_shapes(base_shapes)
    delta = delta_shapes if isinstance(delta_shapes, dict) else get_shapes(delta_shapes)
    out = {}
    for n, bs in base.items():
        ds = delta[n]
        out[n] = [b if b != d else None for b, d in zip(bs, ds)]
    if savefile:
        save_base_shapes(out, savefile)
    return out


def save_base_shapes(model_or_shapes, file: str):
    shapes = model_or_shapes if isinstance(model_or_shapes, dict) else {
        n: list(s.base_shape) for n, s in get_infshapes(model_or_shapes).items()}
    with open(file, "w") as f:
        yaml.safe_dump({k: list(v) for k, v in shapes.items()}, f)


def load_base_shapes(filename: str) -> Dict[str, list]:
    with open(filename) as f:
        return yaml.safe_load(f)


def set_base_shapes(model: nn.Module, base, delta=None, savefile: Optional[str] = None, rescale_params: bool = True,
                    do_assert: bool = True) -> nn.Module:
    """Attach ``infshape`` to every parameter of ``model``.

    ``base``: a model / shape dict of the base width, a YAML file written by
    ``save_base_shapes``, or None (model treated as its own base: SP).
    ``delta``: a model/shape dict at another width; when omitted, dims that
    differ between ``base`` and ``model`` are the infinite ones.
    """
    shapes = get_shapes(model)
    if base is None:
        base_shapes = {n: [None] * len(s) for n, s in shapes.items()}
    elif isinstance(base, str):
        base_shapes = load_base_shapes(base)
    elif delta is not None:
        base_shapes = make_base_shapes(base, delta)
    else:
        bs = base if isinstance(base, dict) else get_shapes(base)
        base_shapes = {n: [b if b != s else None for b, s in zip(bs[n], shapes[n])] for n in shapes}
    for n, p in model.named_parameters():
        if do_assert and len(base_shapes[n]) != p.dim():
            raise ValueError(f"base shape of {n} has rank {len(base_shapes[n])}, param has {p.dim()}")
        p.infshape = InfShape(InfDim(b, d) for b, d in zip(base_shapes[n], p.shape))
    for m in model.modules():
        if isinstance(m, MuReadout):
            m._rescale_parameters(rescale_params)
    if savefile:
        save_base_shapes(base_shapes, savefile)
    return model


def assert_hidden_size_inf(model: nn.Module):
    for n, m in model.named_modules():
        if isinstance(m, nn.Linear) and not isinstance(m, MuReadout):
            if not m.weight.infshape.fanin_fanout()[0].isinf() and not m.weight.infshape.fanin_fanout()[1].isinf():
                raise AssertionError(f"{n}: neither dim of this Linear scales with width")


# --------------------------------------------------------------- init
def _check(t):
    if not hasattr(t, "infshape"):
        raise AssertionError("call set_base_shapes(model, ...) before muP initialisation")


@torch.no_grad()
def _const_std(tensor, sample):
    _check(tensor)
    scale = tensor.infshape.width_mult() ** -0.5 if tensor.infshape.ninf() == 2 else 1.0
    sample(tensor, scale)
    return tensor


def normal_(tensor, mean: float = 0.0, std: float = 1.0):
    return _const_std(tensor, lambda t, s: t.normal_(mean * s, std * s))


def uniform_(tensor, a: float = 0.0, b: float = 1.0):
    return _const_std(tensor, lambda t, s: t.uniform_(a * s, b * s))


def trunc_normal_(tensor, mean: float = 0.0, std: float = 1.0, a: float = -2.0, b: float = 2.0):
    return _const_std(tensor, lambda t, s: nn.init.trunc_normal_(t, mean * s, std * s, a * s, b * s))


def ones_(tensor):
    return _const_std(tensor, lambda t, s: t.fill_(s))


def eye_(tensor):
    _check(tensor)
    return nn.init.eye_(tensor)


def _fan_adjust(tensor) -> float:
    """Standard fan-based inits already give 1/fan_in variance; muP wants
    hidden weights unchanged and vector-likes with an infinite fan-out
    (input embeddings) at constant scale."""
    _check(tensor)
    sh = tensor.infshape
    fi, fo = sh.fanin_fanout()
    if sh.ninf() == 1 and fo.isinf() and (fi is None or not fi.isinf()):
        # fan-based std shrinks like 1/sqrt(fan_in + fan_out): undo the fan_out part
        fan_in = fi.dim if fi is not None else 1
        return math.sqrt((fan_in + fo.dim) / (fan_in + fo.base_dim))
    return 1.0


@torch.no_grad()
def xavier_uniform_(tensor, gain: float = 1.0):
    nn.init.xavier_uniform_(tensor, gain)
    return tensor.mul_(_fan_adjust(tensor))


@torch.no_grad()
def xavier_normal_(tensor, gain: float = 1.0):
    nn.init.xavier_normal_(tensor, gain)
    return tensor.mul_(_fan_adjust(tensor))


@torch.no_grad()
def kaiming_uniform_(tensor, a=0, mode="fan_in", nonlinearity="leaky_relu"):
    nn.init.kaiming_uniform_(tensor, a, mode, nonlinearity)
    if mode == "fan_out":
        tensor.mul_(_fan_adjust(tensor))
    return tensor


@torch.no_grad()
def kaiming_normal_(tensor, a=0, mode="fan_in", nonlinearity="leaky_relu"):
    nn.init.kaiming_normal_(tensor, a, mode, nonlinearity)
    if mode == "fan_out":
        tensor.mul_(_fan_adjust(tensor))
    return tensor


# ------------------------------------------------------------ modules
class MupModule(nn.Module):
    """Base class: ``mup_initial(mode)`` initialises every Mup* submodule."""

    def mup_initial(self, mode: str = "mup"):
        for m in self.modules():
            if m is not self and hasattr(m, "mup_initial") and not isinstance(m, MupModule):
                m.mup_initial(mode)


class MupLinear(nn.Linear):
    """``nn.Linear`` whose initialisation is muP-aware (``mup_initial``)."""

    _SAMPLERS = ("uniform", "normal", "xavier_uniform", "xavier_normal", "kaiming_uniform", "kaiming_normal")

    def __init__(self, in_features, out_features, bias=True, sampler: str = "normal", bias_zero_init: bool = True,
                 init_weight_method=None, init_bias_method=None, device=None, dtype=None, **kwargs):
        super().__init__(in_features, out_features, bias=bias, device=device, dtype=dtype)
        if sampler not in self._SAMPLERS:
            raise ValueError(f"sampler must be one of {self._SAMPLERS}")
        self._sampler = sampler
        self._bias_zero_init = bias_zero_init
        self._init_w, self._init_b = init_weight_method, init_bias_method
        self._kw = kwargs

    def _sample(self, w, mup: bool):
        kw = self._kw
        s = self._sampler
        if s == "normal":
            (normal_ if mup else nn.init.normal_)(w, kw.get("mean", 0.0), kw.get("std", 1.0))
        elif s == "uniform":
            (uniform_ if mup else nn.init.uniform_)(w, kw.get("a", 0.0), kw.get("b", 1.0))
        elif s.startswith("xavier"):
            f = {"xavier_uniform": (xavier_uniform_, nn.init.xavier_uniform_),
                 "xavier_normal": (xavier_normal_, nn.init.xavier_normal_)}[s][0 if mup else 1]
            f(w, kw.get("gain", 1.0))
        else:
            f = {"kaiming_uniform": (kaiming_uniform_, nn.init.kaiming_uniform_),
                 "kaiming_normal": (kaiming_normal_, nn.init.kaiming_normal_)}[s][0 if mup else 1]
            f(w, kw.get("a", 0.0), kw.get("mode", "fan_in"), kw.get("nonlinearity", "leaky_relu"))

    def _mup_init_weight(self):
        self._sample(self.weight, True)

    def _sp_init_weight(self):
        self._sample(self.weight, False)

    @torch.no_grad()
    def mup_initial(self, mode: str = "mup"):
        if mode not in ("mup", "sp"):
            raise ValueError("mode must be 'mup' or 'sp'")
        if self._init_w is not None:
            self._init_w(self.weight)
        elif mode == "mup":
            self._mup_init_weight()
        else:
            self._sp_init_weight()
        if self.bias is not None:
            if self._init_b is not None:
                self._init_b(self.bias)
            elif self._bias_zero_init:
                self.bias.zero_()
            elif mode == "mup":
                self.bias.mul_(self.weight.infshape[1].width_mult() ** 0.5)


class QKVLayer(MupLinear):
    """Fused Q/K/V projection.  ``attn_mult``: muP uses 1/d (not 1/sqrt(d))
    attention scaling; the query weights are zero-initialised under muP so
    attention starts uniform (Tensor Programs V, sec. 6)."""

    def __init__(self, in_features, out_features, bias=True, zero_query: bool = True, **kw):
        super().__init__(in_features, out_features, bias=bias, **kw)
        self.zero_query = zero_query

    @torch.no_grad()
    def _mup_init_weight(self):
        super()._mup_init_weight()
        if self.zero_query:
            self.weight[: self.out_features // 3].zero_()


class QLayer(QKVLayer):
    @torch.no_grad()
    def _mup_init_weight(self):
        MupLinear._mup_init_weight(self)
        if self.zero_query:
            self.weight.zero_()


class MuReadout(nn.Linear):
    """Output layer: logits = (x W^T + b) * output_mult / width_mult."""

    def __init__(self, in_features, out_features, bias=True, output_mult: float = 1.0, readout_zero_init: bool = True,
                 device=None, dtype=None):
        self.output_mult = output_mult
        self.readout_zero_init = readout_zero_init
        self._rescaled = False
        super().__init__(in_features, out_features, bias=bias, device=device, dtype=dtype)

    def reset_parameters(self):
        if self.readout_zero_init:
            nn.init.zeros_(self.weight)
            if self.bias is not None:
                nn.init.zeros_(self.bias)
        else:
            super().reset_parameters()

    def width_mult(self) -> float:
        _check(self.weight)
        return self.weight.infshape.width_mult()

    @torch.no_grad()
    def _rescale_parameters(self, enable: bool = True):
        """Undo the 1/width_mult output scaling at init (the first
        set_base_shapes only) so the initial function matches SP."""
        if self._rescaled or not enable:
            return
        m = self.width_mult()
        if self.bias is not None:
            self.bias.mul_(m)
        self.weight.mul_(m ** 0.5)
        self._rescaled = True

    def forward(self, x):
        return F.linear(x * (self.output_mult / self.width_mult()), self.weight, self.bias)


OutputLayer = MuReadout


class MuSharedReadout(MuReadout):
    """Readout tied to the input embedding weight."""

    def __init__(self, weight: nn.Parameter, bias=True, **kw):
        super().__init__(weight.shape[1], weight.shape[0], bias=bias, readout_zero_init=False, **kw)
        self.weight = weight


# --------------------------------------------------------- optimizers
def _groups(params):
    params = list(params)
    if params and isinstance(params[0], dict):
        return params
    return [{"params": params}]


def _split(params, scale_fn, defaults, scaled_wd: bool):
    out = []
    for g in _groups(params):
        buckets: Dict[tuple, dict] = {}
        for p in g["params"]:
            _check(p)
            lr_mult, wd_mult = scale_fn(p.infshape)
            key = (lr_mult, wd_mult)
            if key not in buckets:
                ng = {k: v for k, v in g.items() if k != "params"}
                ng["params"] = []
                lr = ng.get("lr", defaults.get("lr"))
                ng["lr"] = lr * lr_mult
                wd = ng.get("weight_decay", defaults.get("weight_decay", 0.0))
                if wd and scaled_wd:
                    ng["weight_decay"] = wd * wd_mult
                buckets[key] = ng
            buckets[key]["params"].append(p)
        out.extend(buckets.values())
    return out


def _adam_scale(sh: InfShape):
    if sh.ninf() == 2:
        m = sh.fanin_fanout()[0].width_mult()
        return 1.0 / m, m  # decoupled wd: lr*wd stays constant
    return 1.0, 1.0


def _sgd_scale(sh: InfShape):
    if sh.ninf() == 1:
        m = sh.width_mult()
        return m, 1.0 / m
    if sh.ninf() == 2:
        r = sh.fanin_fanout_mult_ratio()
        return 1.0 / r, r
    return 1.0, 1.0


def MuAdam(params, impl=torch.optim.AdamW, scaled_wd: bool = True, **kwargs):  # noqa: N802 (reference name)
    return impl(_split(params, _adam_scale, kwargs, scaled_wd), **kwargs)


def MuAdamW(params, **kwargs):  # noqa: N802
    return MuAdam(params, impl=torch.optim.AdamW, **kwargs)


def MuSGD(params, impl=torch.optim.SGD, scaled_wd: bool = True, **kwargs):  # noqa: N802
    return impl(_split(params, _sgd_scale, kwargs, scaled_wd), **kwargs)


def MuAdamParamGroupsAdjust(params, scaled_wd: bool = True, **kwargs):  # noqa: N802
    """Param groups with muP lr/wd applied, for any Adam-like optimizer
    (e.g. the fused HIP AdamW)."""
    return _split(params, _adam_scale, kwargs, scaled_wd)


def MuSGDParamGroupsAdjust(params, scaled_wd: bool = True, **kwargs):  # noqa: N802
    return _split(params, _sgd_scale, kwargs, scaled_wd)
