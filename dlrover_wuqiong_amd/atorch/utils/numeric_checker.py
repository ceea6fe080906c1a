"""Module-level numerics checker: record every patched module's outputs in a
reference run, then compare a second run (other kernels / parallelism /
precision) against them and report the first modules that diverge.

    module_numeric_checker(model, mode="save", dir="./check")   # run A
    module_numeric_checker(model, mode="compare", dir="./check")  # run B
    ... forward ...
    report = checker.report()  # [(module name, call index, max |diff|, ok)]

Parity: ATorch ``atorch/utils/numberic_checker.py`` (``patch_module`` save /
compare modes, ``check_allclose_and_save``, ``module_numberic_checker``).
"""

import os
from typing import Dict, List, Tuple

import torch


def _to_cpu(x):
    if torch.is_tensor(x):
        return x.detach().float().cpu()
    if isinstance(x, (list, tuple)):
        return type(x)(_to_cpu(v) for v in x)
    if isinstance(x, dict):
        return {k: _to_cpu(v) for k, v in x.items()}
    return x


def _flat(x) -> List[torch.Tensor]:
    if torch.is_tensor(x):
        return [x]
    if isinstance(x, (list, tuple)):
        return [t for v in x for t in _flat(v)]
    if isinstance(x, dict):
        return [t for v in x.values() for t in _flat(v)]
    if hasattr(x, "to_tuple"):
        return _flat(x.to_tuple())
    return []


class NumericChecker:
    def __init__(self, save_dir: str, mode: str = "save", atol: float = 0.0, rtol: float = 1e-2):
        if mode not in ("save", "compare"):
            raise ValueError("mode must be save or compare")
        self.save_dir, self.mode, self.atol, self.rtol = save_dir, mode, atol, rtol
        os.makedirs(save_dir, exist_ok=True)
        self.counters: Dict[str, int] = {}
        self.results: List[Tuple[str, int, float, bool]] = []
        self._handles = []

    def _hook(self, name):
        def hook(mod, args, out):
            i = self.counters.get(name, 0)
            self.counters[name] = i + 1
            path = os.path.join(self.save_dir, f"{name or 'root'}.{i}.pt")
            tensors = [t.detach().float().cpu() for t in _flat(out)]
            if self.mode == "save":
                torch.save(tensors, path)
                return
            ref = torch.load(path, weights_only=True)
            worst, ok = 0.0, len(ref) == len(tensors)
            for a, b in zip(ref, tensors):
                if a.shape != b.shape:
                    ok = False
                    continue
                d = (a - b).abs()
                worst = max(worst, float(d.max()) if d.numel() else 0.0)
                ok &= bool(torch.allclose(b, a, atol=self.atol, rtol=self.rtol))
            self.results.append((name, i, worst, ok))
        return hook

    def attach(self, model: torch.nn.Module, leaf_only: bool = False):
        for name, m in model.named_modules():
            if leaf_only and any(True for _ in m.children()):
                continue
            self._handles.append(m.register_forward_hook(self._hook(name)))
        return self

    def detach(self):
        for h in self._handles:
            h.remove()
        self._handles = []

    def report(self) -> List[Tuple[str, int, float, bool]]:
        return list(self.results)

    def first_mismatch(self):
        return next((r for r in self.results if not r[3]), None)


def module_numeric_checker(model, mode: str = "save", dir: str = "./logs/check_numeric", **kw) -> NumericChecker:
    return NumericChecker(dir, mode, **kw).attach(model)
