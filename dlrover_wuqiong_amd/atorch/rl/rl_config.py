"""YAML-driven RLHF job description (``AtorchRLConfig``) and the builders that
turn it into a running PPO job: role models, optimizers, strategies, the
prompt dataset and the flat ``PPOConfig`` the trainer consumes.

The file layout follows ATorch's so its example configs load unchanged:

    model:                       # one entry per role
      actor:      {model_cls, model_path, model_params, train_strategy, optimizer: {name, kwargs}, ...}
      critic:     {...}          # an LM trunk gets a scalar value head (ValueModel)
      ref_model:  {model_cls, model_path, model_params, inference_strategy}
      reward_model: {...}        # LM / value trunk -> score of the last token
      cost_model: {...}          # optional (Safe-RLHF): score subtracted from the reward
      actor_critic_ref: {...}    # optional: ONE model for actor + critic (shared trunk) + frozen ref
    method:   {PPOConfig: {ppo_epoch, init_kl_coef, gamma, lam, cliprange, cliprange_value, vf_coef, ...}}
    train:    {seq_length, batch_size, epoch, num_rollouts, max_grad_norm, checkpoint_dir, ...}
    generation: {batch_size, gen_kwargs, gen_experience_kwargs: {max_new_tokens, temperature, top_k, ...}}
    tokenizer: {tokenizer_path, params}
    data:     {prompt_path, max_prompt_length, pad_token_id}   # extension: the reference leaves create_dataset empty

``model_cls`` is a dotted import path.  Our own model families take a config
object: ``model_params: {config: "llama-tiny"}`` (a ``named`` preset) or a
dict of config fields; HF classes with ``from_pretrained`` load
``model_path`` from local files (no network).  ``train_strategy`` is
``torch_native`` or a list of ``auto_accelerate`` strategy names.

Parity: ATorch ``atorch/rl/config.py:22-290`` (Optimizer /
GeneratationConfig / TrainConfig / TokenizerConfig / ModelConfig /
TrainableModelConfig / PPOConfig / AtorchRLConfig.load_yaml),
``atorch/rl/model_engine/model_engine.py`` (init_child_model /
get_optimizers from the config), ``atorch/rl/main.py``.
"""

import dataclasses
import importlib
import inspect
import json
import os
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

import torch
import torch.nn as nn

TRAINABLE_ROLES = ("actor", "critic", "actor_critic_ref")


def is_trainable_model(role: str) -> bool:
    return role in TRAINABLE_ROLES


def _fill(cfg: Optional[dict], defaults: dict) -> dict:
    """``cfg`` over ``defaults``; keys the dataclass does not know (e.g. the
    reference examples' ``generation.epoch``) are dropped."""
    out = {k: v for k, v in (cfg or {}).items() if k in defaults}
    for k, v in defaults.items():
        if out.get(k) is None:
            out[k] = v
    return out


class _Base:
    def to_dict(self) -> dict:
        return dataclasses.asdict(self)


@dataclass
class OptimizerSpec(_Base):
    name: str = "torch.optim.AdamW"
    kwargs: dict = field(default_factory=dict)

    def resolve(self):
        """Optimizer class from a dotted or bare name, case-insensitive on the
        last component (``torch.optim.adam`` -> ``torch.optim.Adam``)."""
        mod_name, _, cls_name = self.name.rpartition(".")
        mod = importlib.import_module(mod_name or "torch.optim")
        for k in dir(mod):
            if k.lower() == cls_name.lower() and inspect.isclass(getattr(mod, k)):
                return getattr(mod, k)
        raise ValueError(f"optimizer {self.name!r} not found in {mod.__name__}")


@dataclass
class GenerationConfig(_Base):
    batch_size: int = 4
    gen_kwargs: dict = field(default_factory=lambda: {"max_new_tokens": 512, "top_k": 0, "top_p": 1.0,
                                                      "do_sample": False})
    gen_experience_kwargs: dict = field(default_factory=lambda: {"max_new_tokens": 512, "do_sample": False,
                                                                 "temperature": 1.0, "top_k": 50, "top_p": 0.95})

    @classmethod
    def from_dict(cls, d: Optional[dict]) -> "GenerationConfig":
        base = cls()
        return cls(**_fill(d, base.to_dict()))


@dataclass
class TrainConfig(_Base):
    seq_length: int = 1024
    batch_size: int = 1024
    epoch: int = 100
    num_rollouts: int = 2048
    mode: str = "Concurrent"
    trainer: str = "PPOTrainer"
    logdir: str = "./tensorboard"
    scheduler: dict = field(default_factory=lambda: {"name": "cosine_warmup",
                                                     "kwargs": {"num_warmup_steps": 640, "num_training_steps": 6400}})
    eval_interval: int = 100
    checkpoint_interval: int = 100
    checkpoint_dir: str = "./checkpoint"
    gradient_accumulation_steps: int = 1
    max_grad_norm: Any = None
    seed: int = 0

    @classmethod
    def from_dict(cls, d: Optional[dict]) -> "TrainConfig":
        return cls(**_fill(d, cls().to_dict()))


@dataclass
class TokenizerConfig(_Base):
    tokenizer_path: Optional[str] = None
    params: dict = field(default_factory=dict)

    @classmethod
    def from_dict(cls, d: Optional[dict]) -> "TokenizerConfig":
        return cls(**_fill(d, cls().to_dict()))


@dataclass
class ModelConfig(_Base):
    model_cls: str = ""
    model_path: Optional[str] = None
    model_params: dict = field(default_factory=dict)
    train_strategy: Any = "torch_native"
    inference_strategy: Any = "torch_native"
    lazy_load: bool = False
    peft_config: Any = None

    @classmethod
    def from_dict(cls, d: dict) -> "ModelConfig":
        return cls(**_fill(d, cls().to_dict()))


@dataclass
class TrainableModelConfig(ModelConfig):
    optimizer: OptimizerSpec = field(default_factory=OptimizerSpec)
    loss: str = ""

    @classmethod
    def from_dict(cls, d: dict) -> "TrainableModelConfig":
        d = dict(d)
        opt = d.pop("optimizer", None) or {}
        base = ModelConfig.from_dict(d).to_dict()
        base["loss"] = d.get("loss", "") or ""
        return cls(optimizer=OptimizerSpec(name=opt.get("name", "torch.optim.AdamW"),
                                           kwargs=dict(opt.get("kwargs") or {})), **base)


@dataclass
class PPOMethodConfig(_Base):
    ppo_epoch: int = 4
    init_kl_coef: float = 0.05
    gamma: float = 1.0
    lam: float = 0.95
    cliprange: float = 0.2
    cliprange_value: float = 0.2
    vf_coef: float = 0.5
    cliprange_reward: float = 10.0
    ent_coef: float = 0.0
    horizon: float = 10000.0
    clip_ratio: bool = True
    scale_reward: Optional[str] = "running"
    ref_mean: Any = None
    ref_std: Any = None
    target: Optional[float] = None

    @classmethod
    def from_dict(cls, method: Optional[dict]) -> "PPOMethodConfig":
        d = (method or {}).get("PPOConfig", method or {})
        known = {f.name for f in dataclasses.fields(cls)}
        return cls(**{k: v for k, v in _fill(d, cls().to_dict()).items() if k in known})


@dataclass
class DataConfig(_Base):
    prompt_path: Optional[str] = None
    max_prompt_length: int = 64
    pad_token_id: int = 0

    @classmethod
    def from_dict(cls, d: Optional[dict]) -> "DataConfig":
        return cls(**_fill(d, cls().to_dict()))


class Model(_Base):
    """Role -> ModelConfig map with attribute access (``config.model.actor``)."""

    def __init__(self, model: Dict[str, ModelConfig]):
        self.model = model

    def __getattr__(self, key):
        try:
            return self.__dict__["model"][key]
        except KeyError:
            raise AttributeError(key)

    def to_dict(self) -> dict:
        return {k: v.to_dict() for k, v in self.model.items()}


@dataclass
class AtorchRLConfig(_Base):
    model: Model
    ppo_config: PPOMethodConfig
    train: TrainConfig
    generation: GenerationConfig
    model_keys: List[str]
    tokenizer: TokenizerConfig
    data: DataConfig = field(default_factory=DataConfig)

    @classmethod
    def load_yaml(cls, path: str) -> "AtorchRLConfig":
        import yaml

        with open(path) as f:
            return cls.from_dict(yaml.safe_load(f))

    @classmethod
    def from_dict(cls, config: dict) -> "AtorchRLConfig":
        keys = list(config["model"].keys())
        roles = {k: (TrainableModelConfig if is_trainable_model(k) else ModelConfig).from_dict(config["model"][k])
                 for k in keys}
        return cls(model=Model(roles), ppo_config=PPOMethodConfig.from_dict(config.get("method")),
                   train=TrainConfig.from_dict(config.get("train")),
                   generation=GenerationConfig.from_dict(config.get("generation")), model_keys=keys,
                   tokenizer=TokenizerConfig.from_dict(config.get("tokenizer")),
                   data=DataConfig.from_dict(config.get("data")))

    def to_dict(self) -> dict:
        return {"model": self.model.to_dict(), "method": {"PPOConfig": self.ppo_config.to_dict()},
                "train": self.train.to_dict(), "generation": self.generation.to_dict(),
                "tokenizer": self.tokenizer.to_dict(), "data": self.data.to_dict()}

    def to_ppo_config(self):
        """The trainer's flat hyper-parameters (``rl/config.py:PPOConfig``)."""
        from .config import PPOConfig

        m, t, g = self.ppo_config, self.train, self.generation.gen_experience_kwargs
        actor = self.model.model.get("actor")
        critic = self.model.model.get("critic")
        lr = lambda mc: float((mc.optimizer.kwargs or {}).get("lr", 1e-5)) if mc is not None else 1e-5  # noqa: E731
        return PPOConfig(
            max_new_tokens=int(g.get("max_new_tokens", 32)),
            temperature=float(g.get("temperature", 1.0)) if g.get("do_sample", True) else 0.0,
            top_k=int(g.get("top_k", 0) or 0),
            rollout_batch_size=int(self.generation.batch_size),
            mini_batch_size=int(min(t.batch_size, self.generation.batch_size)),
            ppo_epochs=int(m.ppo_epoch), init_kl_coef=float(m.init_kl_coef), target_kl=m.target,
            kl_horizon=int(m.horizon), cliprange=float(m.cliprange), cliprange_value=float(m.cliprange_value),
            vf_coef=float(m.vf_coef), ent_coef=float(m.ent_coef), gamma=float(m.gamma), lam=float(m.lam),
            scale_reward=m.scale_reward if m.scale_reward in ("running",) else None,
            max_grad_norm=float(t.max_grad_norm) if t.max_grad_norm else 0.0,
            actor_lr=lr(actor), critic_lr=lr(critic), seed=int(t.seed))


# ---------------------------------------------------------------------------
# builders
# ---------------------------------------------------------------------------
def load_py_file(path: str):
    """Import a user's model / strategy definition file (the reference's
    ``model_path: .../model_definition.py`` convention)."""
    import importlib.util

    name = "_dwamd_rl_" + os.path.splitext(os.path.basename(path))[0]
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _import(path: str, model_path: Optional[str] = None):
    if model_path and model_path.endswith(".py"):
        return getattr(load_py_file(model_path), path.rpartition(".")[2])
    mod, _, name = path.rpartition(".")
    if not mod:
        import transformers

        if hasattr(transformers, name):
            return getattr(transformers, name)
        raise ValueError(f"model_cls must be a dotted path (or a model_path .py file), got {path!r}")
    return getattr(importlib.import_module(mod), name)


def _config_class(cls):
    mod = importlib.import_module(cls.__module__)
    c = getattr(mod, cls.__name__ + "Config", None)
    if c is None:
        ann = inspect.signature(cls.__init__).parameters.get("cfg")
        c = ann.annotation if ann is not None and inspect.isclass(ann.annotation) else None
    return c


def build_role_model(mc: ModelConfig) -> nn.Module:
    cls = _import(mc.model_cls, mc.model_path)
    params = dict(mc.model_params or {})
    if mc.model_path and mc.model_path.endswith(".py"):
        return cls(**params)
    if mc.model_path and hasattr(cls, "from_pretrained"):
        if not os.path.exists(mc.model_path):
            raise FileNotFoundError(f"model_path {mc.model_path!r} does not exist (no network: local files only)")
        return cls.from_pretrained(mc.model_path, local_files_only=True, **params)
    if "config" in params:
        cfg = params.pop("config")
        ccls = _config_class(cls)
        if ccls is None:
            raise ValueError(f"{mc.model_cls}: cannot find its config class for model_params.config")
        cfg = ccls.named(cfg) if isinstance(cfg, str) else ccls(**cfg)
        model = cls(cfg, **params)
    else:
        model = cls(**params)
    if mc.model_path and os.path.isfile(mc.model_path):
        if mc.model_path.endswith(".safetensors"):
            from safetensors.torch import load_file

            sd = load_file(mc.model_path)
        else:
            sd = torch.load(mc.model_path, map_location="cpu", weights_only=True)
        model.load_state_dict(sd.get("model", sd) if isinstance(sd, dict) else sd)
    return model


def _out_width(model: nn.Module) -> int:
    for holder in (getattr(model, "cfg", None), getattr(model, "config", None)):
        v = getattr(holder, "vocab_size", None)
        if v:
            return int(v)
    raise ValueError("cannot infer the model's output width (vocab_size) for the value head")


class LastTokenScorer(nn.Module):
    """Reward model = a trunk mapping ids -> [B, S, V] (or a ValueModel's
    [B, S]) scored at the last position."""

    def __init__(self, trunk: nn.Module):
        super().__init__()
        self.trunk = trunk

    def forward(self, ids):
        out = self.trunk(ids)
        return out[:, -1] if out.dim() == 2 else out[:, -1].float().mean(-1)


def _strategy(s) -> Optional[list]:
    """None for torch-native training; a ``.py`` path names a file whose
    ``strategy`` attribute is the auto_accelerate strategy (reference
    convention); otherwise a strategy name or list."""
    if s in (None, "", "torch_native"):
        return None
    if isinstance(s, str) and s.endswith(".py"):
        return list(load_py_file(s).strategy)
    return list(s) if isinstance(s, (list, tuple)) else [s]


def build_engine(config: AtorchRLConfig, device: Optional[torch.device] = None, reward_fn=None):
    """ModelEngine for the config's roles.  ``reward_fn`` (ids -> [B])
    replaces a configured reward model (rule-based rewards).  Every role's
    ``train_strategy`` (trainable) / ``inference_strategy`` (frozen) is
    applied under its own parallel-group namespace."""
    from .engine import ModelEngine, ValueModel

    mm = config.model.model
    shared = "actor_critic_ref" in mm
    models = {}
    roles = ("actor_critic_ref",) if shared else ("actor", "critic")
    for role in roles + ("ref_model", "reward_model", "cost_model"):
        if role == "reward_model" and reward_fn is not None:
            models[role] = reward_fn
            continue
        if role not in mm:
            if role == "ref_model":
                src = models["actor_critic_ref" if shared else "actor"]
                models[role] = build_role_model(mm["actor_critic_ref" if shared else "actor"])
                models[role].load_state_dict(src.state_dict())
                continue
            if role == "cost_model":
                continue
            raise ValueError(f"config.model has no {role!r} entry")
        m = build_role_model(mm[role])
        if role == "critic" and not isinstance(m, ValueModel):
            m = ValueModel(m, _out_width(m))
        if role in ("reward_model", "cost_model"):
            m = LastTokenScorer(m)
        models[role] = m
    if device is not None:
        for role, m in models.items():
            if isinstance(m, nn.Module):
                m.to(device)
    if shared:
        models["actor"] = models.pop("actor_critic_ref")
        mm = dict(mm)
        mm["actor"] = mm["critic"] = mm["actor_critic_ref"]
    optim = {r: (mm[r].optimizer.resolve(), dict(mm[r].optimizer.kwargs)) for r in ("actor", "critic")}
    strategies = {r: s for r in ("actor", "critic") if (s := _strategy(mm[r].train_strategy)) is not None}
    for r in ("ref_model", "reward_model", "cost_model"):
        if r in config.model.model and (s := _strategy(config.model.model[r].inference_strategy)) is not None:
            strategies[r] = s
    if shared:
        strategies.pop("critic", None)
    return ModelEngine(models["actor"], models.get("critic"), models["ref_model"], models["reward_model"],
                       strategies=strategies or None, role_optimizers=optim, cost_model=models.get("cost_model"),
                       shared_actor_critic=shared, value_width=_out_width(models["actor"]) if shared else None)


class PromptDataset(torch.utils.data.Dataset):
    """Prompts as fixed-length id tensors: tokenized (``tokenizer`` callable
    returning ``input_ids``) unless already ids, truncated from the LEFT to
    ``max_prompt_length`` (the prompt's end is what the actor continues) and
    left-padded with ``pad_token_id`` so rollouts batch by stacking.

    Parity: ATorch ``atorch/rl/data/data_utils.py`` (BaseDataSet /
    PromptDataset: tokenize, truncate, create_loader)."""

    def __init__(self, prompts, max_prompt_length: int, tokenizer=None, pad_token_id: int = 0,
                 add_special_tokens: bool = False):
        self.max_prompt_length = int(max_prompt_length)
        self.pad_token_id = int(pad_token_id)
        ids = []
        for p in prompts:
            if isinstance(p, str):
                if tokenizer is None:
                    raise ValueError("string prompts need a tokenizer")
                p = tokenizer(p, add_special_tokens=add_special_tokens)["input_ids"]
            p = list(p)[-self.max_prompt_length:]
            ids.append([self.pad_token_id] * (self.max_prompt_length - len(p)) + p)
        self.gen_prompts = torch.tensor(ids, dtype=torch.long) if ids else torch.empty(0, self.max_prompt_length,
                                                                                          dtype=torch.long)

    def __len__(self):
        return self.gen_prompts.shape[0]

    def __getitem__(self, i):
        return self.gen_prompts[i]

    def create_loader(self, batch_size: int, shuffle: bool = False):
        return torch.utils.data.DataLoader(self, batch_size=batch_size, shuffle=shuffle, collate_fn=torch.stack)


def _load_tokenizer(tc: TokenizerConfig):
    if not tc.tokenizer_path:
        return None
    from transformers import AutoTokenizer

    return AutoTokenizer.from_pretrained(tc.tokenizer_path, local_files_only=True, **(tc.params or {}))


def read_prompts(path: str) -> list:
    """``.jsonl`` (objects with ``prompt`` text or ``input_ids``), ``.json``
    (a list of those / strings) or plain text (one prompt per line)."""
    def item(o):
        if isinstance(o, dict):
            return o.get("input_ids", o.get("prompt"))
        return o

    if path.endswith(".jsonl"):
        with open(path) as f:
            return [item(json.loads(line)) for line in f if line.strip()]
    if path.endswith(".json"):
        with open(path) as f:
            return [item(o) for o in json.load(f)]
    with open(path) as f:
        return [line.rstrip("\n") for line in f if line.strip()]


def create_dataset(config: AtorchRLConfig, prompts=None) -> PromptDataset:
    dc = config.data
    if prompts is None:
        if not dc.prompt_path:
            raise ValueError("config.data.prompt_path is not set and no prompts were given")
        prompts = read_prompts(dc.prompt_path)
    tok = _load_tokenizer(config.tokenizer)
    pad = dc.pad_token_id
    if tok is not None and getattr(tok, "pad_token_id", None) is not None:
        pad = tok.pad_token_id
    return PromptDataset(prompts, dc.max_prompt_length, tok, pad)
