"""PPO math: log-probs of sampled tokens, KL-penalised per-token rewards,
GAE advantages / returns, and the clipped policy + value objective.

Parity: ATorch ``atorch/rl/ppo_utils/ppo_util.py`` (``get_kl_penalty``,
``get_rewards``, ``loss``, ``get_advantages_and_returns``) and
``model_utils/model_util.py`` (``logprobs_of_labels``, ``whiten``).
"""

from typing import Dict, Tuple

import torch
import torch.nn.functional as F


def logprobs_of_labels(logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    """log softmax(logits)[label] per position, in fp32."""
    lp = F.log_softmax(logits.float(), dim=-1)
    return lp.gather(-1, labels.unsqueeze(-1)).squeeze(-1)


def entropy_from_logits(logits: torch.Tensor) -> torch.Tensor:
    lp = F.log_softmax(logits.float(), dim=-1)
    return -(lp.exp() * lp).sum(-1)


def masked_mean(x: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
    return (x * mask).sum() / mask.sum().clamp(min=1)


def whiten(x: torch.Tensor, mask: torch.Tensor = None, shift_mean: bool = True) -> torch.Tensor:
    if mask is None:
        mean, var = x.mean(), x.var(unbiased=False)
    else:
        mean = masked_mean(x, mask)
        var = masked_mean((x - mean) ** 2, mask)
    w = (x - mean) * torch.rsqrt(var + 1e-8)
    return w if shift_mean else w + mean


def kl_penalised_rewards(logprobs: torch.Tensor, ref_logprobs: torch.Tensor, scores: torch.Tensor,
                         mask: torch.Tensor, kl_coef: float) -> Tuple[torch.Tensor, torch.Tensor]:
    """Per-token reward = -kl_coef * (logp - logp_ref); the sequence score is
    added at the last valid response token.  Returns (rewards, mean KL)."""
    log_ratio = (logprobs - ref_logprobs) * mask
    rewards = -kl_coef * log_ratio
    last = (mask.sum(1).long() - 1).clamp(min=0)
    rewards = rewards.scatter_add(1, last.unsqueeze(1), scores.to(rewards.dtype).unsqueeze(1))
    mean_kl = masked_mean(log_ratio.exp() - 1 - log_ratio, mask)
    return rewards * mask, mean_kl


def gae_advantages_and_returns(values: torch.Tensor, rewards: torch.Tensor, mask: torch.Tensor, gamma: float,
                               lam: float, whiten_adv: bool = True) -> Tuple[torch.Tensor, torch.Tensor]:
    T = rewards.shape[1]
    lastgae = torch.zeros_like(rewards[:, 0])
    adv = torch.zeros_like(rewards)
    values = values * mask
    for t in reversed(range(T)):
        nextv = values[:, t + 1] if t < T - 1 else torch.zeros_like(values[:, 0])
        delta = rewards[:, t] + gamma * nextv - values[:, t]
        lastgae = (delta + gamma * lam * lastgae) * mask[:, t]
        adv[:, t] = lastgae
    returns = adv + values
    if whiten_adv:
        adv = whiten(adv, mask) * mask
    return adv.detach(), returns.detach()


def ppo_loss(logprobs, values, old_logprobs, old_values, advantages, returns, mask, cliprange: float,
             cliprange_value: float, vf_coef: float, entropy=None, ent_coef: float = 0.0
             ) -> Tuple[torch.Tensor, Dict[str, float]]:
    vclip = old_values + (values - old_values).clamp(-cliprange_value, cliprange_value)
    vf1 = (values - returns) ** 2
    vf2 = (vclip - returns) ** 2
    vf_loss = 0.5 * masked_mean(torch.max(vf1, vf2), mask)
    ratio = torch.exp((logprobs - old_logprobs) * mask)
    pg1 = -advantages * ratio
    pg2 = -advantages * ratio.clamp(1.0 - cliprange, 1.0 + cliprange)
    pg_loss = masked_mean(torch.max(pg1, pg2), mask)
    loss = pg_loss + vf_coef * vf_loss
    ent = masked_mean(entropy, mask) if entropy is not None else torch.zeros(())
    if ent_coef:
        loss = loss - ent_coef * ent
    with torch.no_grad():
        approx_kl = 0.5 * masked_mean((logprobs - old_logprobs) ** 2, mask)
        clipfrac = masked_mean((pg2 > pg1).float(), mask)
    stats = {"loss/policy": float(pg_loss.detach()), "loss/value": float(vf_loss.detach()),
             "loss/total": float(loss.detach()),
             "policy/approx_kl": float(approx_kl), "policy/clipfrac": float(clipfrac),
             "policy/entropy": float(ent)}
    return loss, stats


class AdaptiveKLController:
    """Ziegler et al.: adjust the KL coefficient toward a target KL."""

    def __init__(self, init_kl_coef: float, target: float, horizon: int):
        self.value, self.target, self.horizon = init_kl_coef, target, horizon

    def update(self, current: float, n_steps: int):
        err = max(min(current / self.target - 1, 0.2), -0.2)
        self.value *= 1 + err * n_steps / self.horizon


class FixedKLController:
    def __init__(self, kl_coef: float):
        self.value = kl_coef

    def update(self, current: float, n_steps: int):
        pass
