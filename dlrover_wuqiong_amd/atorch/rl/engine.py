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
init_child_model / apply_strategy_to_child_model per role under
``ParallelGroupContextManager`` :94-188, get_optimizers, eval/train,
save/load, actor / critic / ref_model / reward_model / cost_model /
actor_critic_ref properties :463-481).
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


class SharedCritic(nn.Module):
    """Critic that shares the actor's trunk (ATorch ``actor_critic_ref``):
    values = v_head(actor(ids)); only ``v_head`` is the critic's own
    parameter set -- the trunk is trained by the actor's optimizer from the
    combined PPO loss (policy + value terms)."""

    def __init__(self, actor: nn.Module, vocab_or_hidden: int):
        super().__init__()
        self.actor = [actor]  # not a submodule: its parameters belong to the actor
        self.v_head = nn.Linear(vocab_or_hidden, 1)
        nn.init.zeros_(self.v_head.weight)
        nn.init.zeros_(self.v_head.bias)

    def forward(self, ids):
        h = self.actor[0](ids)
        return self.v_head(h.to(self.v_head.weight.dtype)).squeeze(-1)


class ActorCriticRef(nn.Module):
    """One model object for the three policy-side roles (reference
    ``model_engine.py:463-481`` ``actor_critic_ref``): the actor, a critic
    sharing its trunk, and a frozen reference snapshot of the initial actor."""

    def __init__(self, actor: nn.Module, critic: nn.Module, ref: nn.Module):
        super().__init__()
        self.actor_model, self.critic_model, self.ref_model = actor, critic, ref

    def forward(self, ids):
        return self.actor_model(ids), self.critic_model(ids)


FROZEN_ROLES = ("ref_model", "reward_model", "cost_model")


class ModelEngine:
    def __init__(self, actor: nn.Module, critic: Optional[nn.Module], ref_model: Optional[nn.Module],
                 reward_model: Callable[[torch.Tensor], torch.Tensor], actor_lr: float = 1e-5,
                 critic_lr: float = 1e-5, strategies: Optional[Dict[str, list]] = None,
                 optim_cls=torch.optim.AdamW, role_optimizers: Optional[Dict[str, Tuple[type, dict]]] = None,
                 cost_model: Optional[Callable[[torch.Tensor], torch.Tensor]] = None,
                 shared_actor_critic: bool = False, value_width: Optional[int] = None):
        """``strategies``: {role: auto_accelerate strategy} for ANY role --
        trainable roles get their optimizer from it, frozen ones (ref / reward
        / cost) are only transformed (half, fsdp, tensor_parallel ...).  Each
        role is set up inside ``ParallelGroupContextManager(role)``, so roles
        may use different parallel layouts.  ``role_optimizers`` ({role:
        (optimizer class, kwargs)}, e.g. from an ``AtorchRLConfig``)
        overrides ``optim_cls`` / the role's lr.  ``shared_actor_critic``: the
        critic is a value head on the actor's trunk (``critic`` unused);
        ``ref_model`` None: a frozen copy of the initial actor."""
        import copy

        from ..distributed import ParallelGroupContextManager

        if ref_model is None:
            ref_model = copy.deepcopy(actor)
        if shared_actor_critic:
            width = value_width or getattr(critic, "v_head", nn.Linear(1, 1)).in_features
            if value_width is None and not hasattr(critic, "v_head"):
                raise ValueError("shared_actor_critic needs value_width (the actor's output width)")
        self.shared_actor_critic = shared_actor_critic
        self.models: Dict[str, object] = {"actor": actor, "critic": critic, "ref_model": ref_model,
                                          "reward_model": reward_model}
        if cost_model is not None:
            self.models["cost_model"] = cost_model
        self.optimizers: Dict[str, torch.optim.Optimizer] = {}
        self.strategies = dict(strategies or {})
        role_optimizers = role_optimizers or {}
        for role, lr in (("actor", actor_lr), ("critic", critic_lr)):
            if role == "critic" and shared_actor_critic:
                continue
            m = self.models[role]
            cls, kw = role_optimizers.get(role, (optim_cls, {}))
            kw = dict(kw)
            kw.setdefault("lr", lr)
            if role in self.strategies:
                from ..auto_accelerate import auto_accelerate

                with ParallelGroupContextManager(role):
                    _ok, res, _s = auto_accelerate(m, cls, optim_args=kw, load_strategy=self.strategies[role])
                self.models[role], self.optimizers[role] = res.model, res.optim
            else:
                self.optimizers[role] = cls([p for p in m.parameters() if p.requires_grad], **kw)
        if shared_actor_critic:
            # the head lives on the actor's device / dtype; its optimizer only
            # steps the head (the trunk belongs to the actor's)
            crit = SharedCritic(self.models["actor"], width)
            p0 = next(self.models["actor"].parameters())
            crit.v_head.to(p0.device)
            self.models["critic"] = crit
            cls, kw = role_optimizers.get("critic", (optim_cls, {}))
            kw = dict(kw)
            kw.setdefault("lr", critic_lr)
            self.optimizers["critic"] = cls(list(crit.v_head.parameters()), **kw)
        for role in FROZEN_ROLES:
            m = self.models.get(role)
            if not isinstance(m, nn.Module):
                continue
            m.eval()
            for p in m.parameters():
                p.requires_grad_(False)
            if role in self.strategies:
                from ..auto_accelerate import auto_accelerate

                with ParallelGroupContextManager(role):
                    _ok, res, _s = auto_accelerate(m, None, load_strategy=self.strategies[role])
                self.models[role] = res.model.eval()

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
    def cost_model(self):
        return self.models.get("cost_model")

    @property
    def actor_critic_ref(self) -> Optional[ActorCriticRef]:
        if not self.shared_actor_critic:
            return None
        return ActorCriticRef(self.actor, self.critic, self.ref_model)

    @property
    def actor_optimizer(self):
        return self.optimizers["actor"]

    @property
    def critic_optimizer(self):
        return self.optimizers["critic"]

    def trainable_parameters(self, role: str):
        """Parameters a role's gradient clipping covers (a shared critic: its head)."""
        m = self.models[role]
        if role == "critic" and self.shared_actor_critic:
            return list(m.v_head.parameters())
        return [p for p in m.parameters() if p.requires_grad]

    def eval(self):
        for role in ("actor", "critic"):
            self.models[role].eval()

    def train(self):
        for role in ("actor", "critic"):
            self.models[role].train()

    def save(self, path: str, include_optimizer_state: bool = True):
        os.makedirs(path, exist_ok=True)
        for role in ("actor", "critic"):
            m = self.models[role]
            sd = {"model": m.v_head.state_dict() if (role == "critic" and self.shared_actor_critic)
                  else m.state_dict()}
            if include_optimizer_state:
                sd["optimizer"] = self.optimizers[role].state_dict()
            torch.save(sd, os.path.join(path, f"{role}.pt"))

    def load(self, path: str, include_optimizer_state: bool = True):
        for role in ("actor", "critic"):
            sd = torch.load(os.path.join(path, f"{role}.pt"), map_location="cpu", weights_only=True)
            m = self.models[role]
            (m.v_head if (role == "critic" and self.shared_actor_critic) else m).load_state_dict(sd["model"])
            if include_optimizer_state and "optimizer" in sd:
                self.optimizers[role].load_state_dict(sd["optimizer"])
