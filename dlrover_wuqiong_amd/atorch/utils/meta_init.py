"""Meta-device model construction and per-rank materialisation.

Building a 70B model eagerly on every rank wastes host RAM and time; build it
on the ``meta`` device (shapes only), shard / split it (FSDP, TP, pipeline
stages), then materialise just this rank's parameters on the GPU and either
run the modules' own initialisers or load the weights from a checkpoint.

    with init_empty_weights():
        model = Llama(LlamaConfig.named("llama3-70b"))        # 0 bytes
    stage = split_model(model, pp, rank)                       # still meta
    materialize(stage, device="cuda", init_fn=Llama._init)     # this stage only
    # or: load_state_dict_to_meta(stage, safetensors_file)

Tied weights (e.g. embedding / LM head) stay tied through materialisation.

Parity: ATorch ``atorch/utils/meta_model_utils.py`` (``init_empty_weights_with_disk_offload``,
``reload_meta_module``, ``_find_tied_weights`` / ``_retie_weights``,
``is_meta``) -- torch's native meta device replaces the reference's
constructor patching and disk offload.
"""

import contextlib
from typing import Callable, Dict, List, Optional

import torch
import torch.nn as nn


@contextlib.contextmanager
def init_empty_weights():
    with torch.device("meta"):
        yield


def is_meta(module: nn.Module) -> bool:
    return any(p.is_meta for p in module.parameters()) or any(b.is_meta for b in module.buffers())


def find_tied_parameters(model: nn.Module) -> List[List[str]]:
    seen: Dict[int, List[str]] = {}
    for name, p in model.named_parameters(remove_duplicate=False):
        seen.setdefault(id(p), []).append(name)
    return [names for names in seen.values() if len(names) > 1]


def _get(model, name):
    mod = model
    parts = name.split(".")
    for p in parts[:-1]:
        mod = getattr(mod, p)
    return mod, parts[-1]


def retie_parameters(model: nn.Module, groups: List[List[str]]):
    for names in groups:
        m0, a0 = _get(model, names[0])
        p = getattr(m0, a0)
        for n in names[1:]:
            m, a = _get(model, n)
            setattr(m, a, p)


def materialize(module: nn.Module, device="cuda", dtype: Optional[torch.dtype] = None,
                init_fn: Optional[Callable[[nn.Module], None]] = None) -> nn.Module:
    """Allocate this module's meta parameters/buffers on ``device`` (tied
    weights once) and initialise them with ``init_fn`` (applied per module)
    or each module's ``reset_parameters``."""
    ties = find_tied_parameters(module)
    module.to_empty(device=device)
    if dtype is not None:
        module.to(dtype)
    retie_parameters(module, ties)
    with torch.no_grad():
        if init_fn is not None:
            module.apply(init_fn)
        else:
            for m in module.modules():
                if hasattr(m, "reset_parameters"):
                    m.reset_parameters()
    return module


def load_state_dict_to_meta(module: nn.Module, path_or_sd, device="cuda", strict: bool = True):
    """Materialise from weights: a state dict or a safetensors file (read
    lazily tensor by tensor, only the keys this module owns)."""
    ties = find_tied_parameters(module)
    module.to_empty(device=device)
    retie_parameters(module, ties)
    own = dict(module.state_dict())
    if isinstance(path_or_sd, str):
        from safetensors import safe_open

        with safe_open(path_or_sd, framework="pt", device="cpu") as f:
            keys = set(f.keys())
            missing = [k for k in own if k not in keys]
            for k in own:
                if k in keys:
                    with torch.no_grad():
                        own[k].copy_(f.get_tensor(k))
    else:
        missing = [k for k in own if k not in path_or_sd]
        for k, v in own.items():
            if k in path_or_sd:
                with torch.no_grad():
                    v.copy_(path_or_sd[k])
    # a tied alias is satisfied when any member of its group was loaded
    alias = {n: g for g in ties for n in g}
    missing = [k for k in missing if not any(o not in missing for o in alias.get(k, []))]
    if strict and missing:
        raise KeyError(f"missing weights for {missing[:8]}{'...' if len(missing) > 8 else ''}")
    return module
