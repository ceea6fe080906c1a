"""PPO (RLHF) on tiny models: GAE / loss math and an end-to-end run whose
reward rises.  Parity: reference atorch/tests/rl/test_ppo_util.py and
test_rl_trainer.py."""

import copy

import torch


def test_gae_matches_reference_recursion():
    from dlrover_wuqiong_amd.atorch.rl.ppo_utils import gae_advantages_and_returns

    torch.manual_seed(0)
    v, r = torch.randn(3, 5), torch.randn(3, 5)
    m = torch.ones(3, 5)
    adv, ret = gae_advantages_and_returns(v, r, m, gamma=0.9, lam=0.8, whiten_adv=False)
    exp = torch.zeros(3, 5)
    for b in range(3):
        last = 0.0
        for t in reversed(range(5)):
            nv = v[b, t + 1] if t < 4 else 0.0
            last = r[b, t] + 0.9 * nv - v[b, t] + 0.9 * 0.8 * last
            exp[b, t] = last
    assert torch.allclose(adv, exp, atol=1e-6) and torch.allclose(ret, exp + v, atol=1e-6)


def test_ppo_loss_clips_ratio():
    from dlrover_wuqiong_amd.atorch.rl.ppo_utils import kl_penalised_rewards, ppo_loss

    old = torch.zeros(1, 2)
    new = torch.log(torch.tensor([[2.0, 0.5]]))  # ratios 2.0 and 0.5
    adv = torch.tensor([[1.0, -1.0]])
    z = torch.zeros(1, 2)
    loss, st = ppo_loss(new, z, old, z, adv, z, torch.ones(1, 2), 0.2, 0.2, vf_coef=0.0)
    # max(-A r, -A clip(r)): t0: max(-2, -1.2) = -1.2 ; t1: max(0.5, 0.8) = 0.8
    assert abs(float(loss) - (-1.2 + 0.8) / 2) < 1e-6 and st["policy/clipfrac"] == 1.0
    rew, kl = kl_penalised_rewards(torch.zeros(2, 3), torch.zeros(2, 3), torch.tensor([1.0, 2.0]),
                                   torch.ones(2, 3), 0.1)
    assert rew[0, -1] == 1.0 and rew[1, -1] == 2.0 and float(kl) == 0.0


def test_ppo_end_to_end_increases_reward():
    from dlrover_wuqiong_amd.atorch.rl import ModelEngine, PPOConfig, PPOTrainer, ValueModel
    from dlrover_wuqiong_amd.models.gpt2 import GPT2, GPT2Config

    torch.manual_seed(0)
    cfg = GPT2Config(vocab_size=16, n_positions=32, n_layer=2, n_head=2, n_embd=32)
    actor = GPT2(cfg)
    ref = copy.deepcopy(actor)
    critic = ValueModel(GPT2(cfg), 16)

    def reward(seq):  # fraction of response tokens equal to 3
        return (seq[:, 4:] == 3).float().mean(1)

    prompts = [torch.randint(0, 16, (4,)) for _ in range(64)]
    c = PPOConfig(max_new_tokens=6, rollout_batch_size=16, mini_batch_size=8, ppo_epochs=2, actor_lr=3e-3,
                  critic_lr=3e-3, init_kl_coef=0.01)
    eng = ModelEngine(actor, critic, ref, reward, c.actor_lr, c.critic_lr)
    tr = PPOTrainer(eng, prompts, c)
    hist = tr.train(num_rollouts=24)
    first = sum(h["reward/mean"] for h in hist[:4]) / 4
    last = sum(h["reward/mean"] for h in hist[-4:]) / 4
    assert last > first + 0.2, (first, last)
    assert all(k in hist[-1] for k in ("loss/policy", "loss/value", "policy/approx_kl", "kl_coef"))
