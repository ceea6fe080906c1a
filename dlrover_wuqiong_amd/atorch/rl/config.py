"""PPO configuration.  Parity: ATorch ``atorch/rl/config.py`` (model
configs per role + PPO hyper-parameters: kl coefficient / adaptive target,
cliprange, cliprange_value, vf_coef, gamma, lam, ppo_epochs, whitening)."""

from dataclasses import dataclass
from typing import Optional


@dataclass
class PPOConfig:
    # generation
    max_new_tokens: int = 32
    temperature: float = 1.0
    top_k: int = 0
    # KV-cached generation from the training weights (Llama actors;
    # ``hybrid_engine.py``), HIP-graph decode on the GPU
    use_hybrid_engine: bool = True
    max_seq_len: Optional[int] = None   # cache length; default prompt + max_new_tokens
    # rollout / optimisation
    rollout_batch_size: int = 16
    mini_batch_size: int = 8
    ppo_epochs: int = 4
    # objective
    init_kl_coef: float = 0.05
    target_kl: Optional[float] = None   # adaptive KL controller when set
    kl_horizon: int = 10000
    cliprange: float = 0.2
    cliprange_value: float = 0.2
    vf_coef: float = 0.5
    ent_coef: float = 0.0
    gamma: float = 1.0
    lam: float = 0.95
    whiten_advantages: bool = True
    scale_reward: Optional[str] = None   # None | "running" (divide by running std)
    max_grad_norm: float = 1.0
    actor_lr: float = 1e-5
    critic_lr: float = 1e-5
    seed: int = 0
    # Safe-RLHF style: reward - cost_coef * cost when the engine has a cost model
    cost_coef: float = 1.0
