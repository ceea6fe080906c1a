"""PPO trainer: rollout (sample responses with the actor), score them with
the reward model, KL-penalise against the reference model, GAE, then
``ppo_epochs`` of clipped-objective updates over shuffled mini-batches.

    engine = ModelEngine(actor, ValueModel(critic_trunk, V), ref, reward_fn)
    trainer = PPOTrainer(engine, prompt_dataset, PPOConfig(...))
    trainer.train(num_rollouts=100)

Parity: ATorch ``atorch/rl/trainer/{rl_trainer,ppo_trainer}.py``
(``RLTrainer`` hooks: pre_make_experience / post_experience_generation /
pre_rl_training / post_rl_training, ``make_experience``, ``rl_training``,
``evaluate``, ``train``) and the replay buffer of ``rl/replay_buffer``.
"""

import os
from dataclasses import dataclass
from typing import Dict, List, Optional

import torch

from ...common.log import logger
from .config import PPOConfig
from .engine import ModelEngine
from .ppo_utils import (AdaptiveKLController, FixedKLController, entropy_from_logits, gae_advantages_and_returns,
                        kl_penalised_rewards, logprobs_of_labels, ppo_loss)


@torch.no_grad()
def sample(actor, prompts: torch.Tensor, max_new_tokens: int, temperature: float = 1.0, top_k: int = 0,
           generator: Optional[torch.Generator] = None) -> torch.Tensor:
    """Autoregressive sampling (full-sequence forward per token; use a
    KV-cached HF ``generate`` for long responses)."""
    ids = prompts
    for _ in range(max_new_tokens):
        logits = actor(ids)[:, -1, :].float()
        if temperature <= 0:
            nxt = logits.argmax(-1, keepdim=True)
        else:
            logits = logits / temperature
            if top_k:
                kth = logits.topk(top_k, dim=-1).values[:, -1:]
                logits = logits.masked_fill(logits < kth, float("-inf"))
            nxt = torch.multinomial(logits.softmax(-1), 1, generator=generator)
        ids = torch.cat([ids, nxt], 1)
    return ids


@dataclass
class Experience:
    sequences: torch.Tensor      # [B, P + R]
    logprobs: torch.Tensor       # [B, R]
    values: torch.Tensor         # [B, R]
    advantages: torch.Tensor     # [B, R]
    returns: torch.Tensor        # [B, R]
    mask: torch.Tensor           # [B, R]
    scores: torch.Tensor         # [B]


class ReplayBuffer:
    def __init__(self):
        self.items: List[Experience] = []

    def push(self, e: Experience):
        self.items.append(e)

    def clear(self):
        self.items = []

    def minibatches(self, size: int, generator: Optional[torch.Generator] = None):
        seqs = torch.cat([e.sequences for e in self.items])
        fields = {k: torch.cat([getattr(e, k) for e in self.items]) for k in
                  ("logprobs", "values", "advantages", "returns", "mask")}
        n = seqs.shape[0]
        perm = torch.randperm(n, generator=generator)
        for i in range(0, n, size):
            idx = perm[i:i + size]
            yield seqs[idx], {k: v[idx] for k, v in fields.items()}


class RLTrainer:
    def __init__(self, engine: ModelEngine, prompt_dataset, config: PPOConfig):
        self.engine, self.dataset, self.config = engine, prompt_dataset, config
        self.buffer = ReplayBuffer()
        self.stats_history: List[Dict[str, float]] = []

    # hooks (reference names)
    def pre_make_experience_hook(self):
        self.engine.eval()

    def post_experience_generation_hook(self):
        pass

    def pre_rl_training_hook(self):
        self.engine.train()

    def post_rl_training_hook(self):
        self.buffer.clear()

    def make_experience(self, prompts):
        raise NotImplementedError

    def rl_training(self):
        raise NotImplementedError

    def evaluate(self, prompts) -> float:
        self.engine.eval()
        seq = sample(self.engine.actor, prompts, self.config.max_new_tokens, temperature=0.0)
        return float(self.engine.reward_model(seq).float().mean())

    def _prompt_batches(self):
        n = len(self.dataset)
        g = torch.Generator().manual_seed(self.config.seed)
        while True:
            idx = torch.randperm(n, generator=g)
            for i in range(0, n - self.config.rollout_batch_size + 1, self.config.rollout_batch_size):
                yield torch.stack([self.dataset[int(j)] for j in idx[i:i + self.config.rollout_batch_size]])

    def train(self, num_rollouts: int, checkpoint_interval: int = 0,
              checkpoint_dir: Optional[str] = None) -> List[Dict[str, float]]:
        """``checkpoint_interval`` > 0 saves actor + critic (and their
        optimizers) to ``checkpoint_dir/rollout_{it}`` every that many
        rollouts (reference ``TrainConfig.checkpoint_interval``)."""
        batches = self._prompt_batches()
        for it in range(num_rollouts):
            self.pre_make_experience_hook()
            prompts = next(batches)
            dev = next(self.engine.actor.parameters()).device
            self.make_experience(prompts.to(dev))
            self.post_experience_generation_hook()
            self.pre_rl_training_hook()
            stats = self.rl_training()
            self.post_rl_training_hook()
            stats["rollout"] = it
            self.stats_history.append(stats)
            if checkpoint_interval and checkpoint_dir and (it + 1) % checkpoint_interval == 0:
                self.engine.save(os.path.join(checkpoint_dir, f"rollout_{it + 1}"))
            logger.info(f"rollout {it}: {stats}")
        return self.stats_history


class PPOTrainer(RLTrainer):
    def __init__(self, engine: ModelEngine, prompt_dataset, config: PPOConfig):
        super().__init__(engine, prompt_dataset, config)
        self.kl_ctl = (AdaptiveKLController(config.init_kl_coef, config.target_kl, config.kl_horizon)
                       if config.target_kl else FixedKLController(config.init_kl_coef))
        self.gen = torch.Generator(device="cpu").manual_seed(config.seed)
        self._last = {}

    def _hybrid(self, prompts):
        """The actor's hybrid (KV-cache) engine, or None to sample with full
        forwards (non-Llama or tensor/sequence-parallel actors)."""
        c = self.config
        if not c.use_hybrid_engine:
            return None
        need = (prompts.shape[0], c.max_seq_len or prompts.shape[1] + c.max_new_tokens)
        hy = getattr(self, "_hy", None)
        if hy is None or hy.max_batch < need[0] or hy.max_len < need[1]:
            from .hybrid_engine import HybridEngine, find_llama

            llama = find_llama(self.engine.actor)
            if llama is None:  # not a Llama-family actor: full-forward sampling
                self.config.use_hybrid_engine = False
                return None
            hy = self._hy = HybridEngine(self.engine.actor, need[0], need[1])
        return hy

    def _response_stats(self, model, seq, P):
        logits = model(seq)
        resp_logits = logits[:, P - 1:-1, :]
        return logits, logprobs_of_labels(resp_logits, seq[:, P:]), resp_logits

    @torch.no_grad()
    def make_experience(self, prompts: torch.Tensor):
        c, e = self.config, self.engine
        P = prompts.shape[1]
        g = self.gen if prompts.device.type == "cpu" else None
        hy = self._hybrid(prompts)
        if hy is not None:
            seq = hy.generate(prompts, c.max_new_tokens, c.temperature, c.top_k, generator=g)
        else:
            seq = sample(e.actor, prompts, c.max_new_tokens, c.temperature, c.top_k, generator=g)
        R = seq.shape[1] - P
        mask = torch.ones(seq.shape[0], R, device=seq.device)
        _, logprobs, _ = self._response_stats(e.actor, seq, P)
        _, ref_logprobs, _ = self._response_stats(e.ref_model, seq, P)
        values = e.critic(seq)[:, P - 1:-1].float()
        scores = e.reward_model(seq).float()
        if e.cost_model is not None:
            cost = e.cost_model(seq).float()
            self._cost = float(cost.mean())
            scores = scores - c.cost_coef * cost
        rewards, mean_kl = kl_penalised_rewards(logprobs, ref_logprobs, scores, mask, self.kl_ctl.value)
        adv, ret = gae_advantages_and_returns(values, rewards, mask, c.gamma, c.lam, c.whiten_advantages)
        self.buffer.push(Experience(seq, logprobs, values, adv, ret, mask, scores))
        self.kl_ctl.update(float(mean_kl), seq.shape[0])
        self._last = {"reward/mean": float(scores.mean()), "policy/mean_kl": float(mean_kl),
                      "kl_coef": self.kl_ctl.value}

    def rl_training(self) -> Dict[str, float]:
        c, e = self.config, self.engine
        P = self.buffer.items[0].sequences.shape[1] - self.buffer.items[0].logprobs.shape[1]
        agg: Dict[str, float] = {}
        n = 0
        for _ in range(c.ppo_epochs):
            for seq, mb in self.buffer.minibatches(c.mini_batch_size, self.gen):
                _, logprobs, resp_logits = self._response_stats(e.actor, seq, P)
                values = e.critic(seq)[:, P - 1:-1].float()
                ent = entropy_from_logits(resp_logits) if c.ent_coef else None
                loss, st = ppo_loss(logprobs, values, mb["logprobs"], mb["values"], mb["advantages"], mb["returns"],
                                    mb["mask"], c.cliprange, c.cliprange_value, c.vf_coef, ent, c.ent_coef)
                e.actor_optimizer.zero_grad(set_to_none=True)
                e.critic_optimizer.zero_grad(set_to_none=True)
                loss.backward()
                if c.max_grad_norm:
                    torch.nn.utils.clip_grad_norm_(e.trainable_parameters("actor"), c.max_grad_norm)
                    torch.nn.utils.clip_grad_norm_(e.trainable_parameters("critic"), c.max_grad_norm)
                e.actor_optimizer.step()
                e.critic_optimizer.step()
                for k, v in st.items():
                    agg[k] = agg.get(k, 0.0) + v
                n += 1
        out = {k: v / max(1, n) for k, v in agg.items()}
        out.update(self._last)
        return out
