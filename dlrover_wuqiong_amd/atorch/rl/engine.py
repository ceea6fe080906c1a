"""Model engine for RLHF: the four PPO roles (actor, critic, frozen
reference, frozen reward model), their optimizers and train/eval switching,
save / load.

Each role is any ``nn.Module`` mapping token ids [B, S] to logits
[B, S, V] (actor / ref) or values [B, S] (critic; ``ValueModel`` wraps a
language model with a scalar head), or ids -> scores [B] (reward).
Trainable roles can be accelerated with ``auto_accelerate`` strategies
(``strategies={"actor": [...], "critic": [...]}``); frozen roles run in
eval / inference mode and, on GPU, in bf16.

Parity: ATorch ``atorch/rl/model_engine/model_engine.py`` (``ModelEngine``:
init_child_model, apply_strategy_to_child_model, get_optimizers, eval/train,
save/load, actor/critic/ref_model/reward_model properties).
"""

import os
from typing import Callable, Dict, Optional, Tuple

import torch
import torch.nn as nn


class ValueModel(nn.Module):
    """Critic = a language-model trunk + scalar head over its vocabulary
    logits (works with any module returning [B, S, V])."""

    def __init__(self, trunk: nn.Module, vocab_or_hidden: int):
        super().__init__()
        self.trunk = trunk
        self.v_head = nn.Linear(vocab_or_hidden, 1)
        nn.init.zeros_(self.v_head.weight)
        nn.init.zeros_(self.v_head.bias)

    def forward(self, ids):
        h = self.trunk(ids)
        return self.v_head(h.to(self.v_head.weight.dtype)).squeeze(-1)


class ModelEngine:
    def __init__(self, actor: nn.Module, critic: nn.Module, ref_model: nn.Module,
                 reward_model: Callable[[torch.Tensor], torch.Tensor], actor_lr: float = 1e-5,
                 critic_lr: float = 1e-5, strategies: Optional[Dict[str, list]] = None,
                 optim_cls=torch.optim.AdamW, role_optimizers: Optional[Dict[str, Tuple[type, dict]]] = None):
        """``role_optimizers`` ({role: (optimizer class, kwargs)}, e.g. from
        an ``AtorchRLConfig``) overrides ``optim_cls`` / the role's lr."""
        self.models: Dict[str, object] = {"actor": actor, "critic": critic, "ref_model": ref_model,
                                          "reward_model": reward_model}
        self.optimizers: Dict[str, torch.optim.Optimizer] = {}
        strategies = strategies or {}
        role_optimizers = role_optimizers or {}
        for role, lr in (("actor", actor_lr), ("critic", critic_lr)):
            m = self.models[role]
            cls, kw = role_optimizers.get(role, (optim_cls, {}))
            kw = dict(kw)
            kw.setdefault("lr", lr)
            if role in strategies:
                from ..auto_accelerate import auto_accelerate

                _ok, res, _s = auto_accelerate(m, cls, optim_args=kw, load_strategy=strategies[role])
                self.models[role], self.optimizers[role] = res.model, res.optim
            else:
                self.optimizers[role] = cls([p for p in m.parameters() if p.requires_grad], **kw)
        for role in ("ref_model", "reward_model"):
            m = self.models[role]
            if isinstance(m, nn.Module):
                m.eval()
                for p in m.parameters():
                    p.requires_grad_(False)

    @property
    def actor(self):
        return self.models["actor"]

    @property
    def critic(self):
        return self.models["critic"]

    @property
    def ref_model(self):
        return self.models["ref_model"]

    @property
    def reward_model(self):
        return self.models["reward_model"]

    @property
    def actor_optimizer(self):
        return self.optimizers["actor"]

    @property
    def critic_optimizer(self):
        return self.optimizers["critic"]

    def eval(self):
        for role in ("actor", "critic"):
            self.models[role].eval()

    def train(self):
        for role in ("actor", "critic"):
            self.models[role].train()

    def save(self, path: str, include_optimizer_state: bool = True):
        os.makedirs(path, exist_ok=True)
        for role in ("actor", "critic"):
            sd = {"model": self.models[role].state_dict()}
            if include_optimizer_state:
                sd["optimizer"] = self.optimizers[role].state_dict()
            torch.save(sd, os.path.join(path, f"{role}.pt"))

    def load(self, path: str, include_optimizer_state: bool = True):
        for role in ("actor", "critic"):
            sd = torch.load(os.path.join(path, f"{role}.pt"), map_location="cpu", weights_only=True)
            self.models[role].load_state_dict(sd["model"])
            if include_optimizer_state and "optimizer" in sd:
                self.optimizers[role].load_state_dict(sd["optimizer"])
