"""YAML-driven RLHF: AtorchRLConfig parsing (reference example layout),
role building (our Llama from a named preset, a user model_definition.py),
rl_train end to end with checkpoints, and the keyed replay buffer's
2-rank gloo sync.  Parity: reference atorch/rl/config.py, main.py,
replay_buffer/replay_buffer.py and tests/test_define_rl_models."""

import json
import os

import pytest
import torch
import yaml

REF_STYLE = """
model:
  actor:
      model_path: {defs}
      model_cls: FakeActor
      model_params: {{features_in: 10, features_out: 10}}
      train_strategy: null
      inference_strategy: null
      peft_config: {{peft_type: LORA, r: 8}}
  critic:
      model_path: {defs}
      model_cls: FakeCritic
      model_params: {{dims_in: 2, dims_out: 2}}
train: {{seq_length: 1024, batch_size: 4, epoch: 1, num_rollouts: 10}}
generation:
    batch_size: 4
    epoch: 10
    gen_kwargs: {{max_new_tokens: 512, top_k: 0, top_p: 1.0, do_sample: false}}
    gen_experience_kwargs: {{max_new_tokens: 512, do_sample: false, temperature: 1.0, top_k: 50, top_p: 0.95}}
tokenizer:
  tokenizer_path: /nonexistent/tokenizer
  params: {{truncation_side: right}}
method:
  PPOConfig: {{ppo_epoch: 2, init_kl_coef: 0.02, gamma: 1, lam: 0.95, cliprange: 0.2, cliprange_value: 0.2,
              vf_coef: 0.1, cliprange_reward: 50, clip_ratio: true, ent_coef: 0.01, scale_reward: running,
              ref_mean: null, ref_std: null}}
"""

DEFS = """
import torch


class FakeActor(torch.nn.Module):
    def __init__(self, features_in=10, features_out=10):
        super().__init__()
        self.linear = torch.nn.Linear(features_in, features_out)


class FakeCritic(torch.nn.Module):
    def __init__(self, dims_in=10, dims_out=10):
        super().__init__()
        self.linear = torch.nn.Linear(dims_in, dims_out)
"""


def test_reference_layout_parses(tmp_path):
    from atorch.rl.config import AtorchRLConfig, TrainableModelConfig
    from dlrover_wuqiong_amd.atorch.rl.rl_config import build_role_model

    defs = tmp_path / "model_definition.py"
    defs.write_text(DEFS)
    p = tmp_path / "model_def.yaml"
    p.write_text(REF_STYLE.format(defs=defs))
    c = AtorchRLConfig.load_yaml(str(p))
    assert c.model_keys == ["actor", "critic"]
    assert isinstance(c.model.actor, TrainableModelConfig)
    assert c.model.actor.optimizer.resolve() is torch.optim.AdamW
    assert c.ppo_config.ppo_epoch == 2 and c.ppo_config.vf_coef == 0.1 and c.ppo_config.horizon == 10000.0
    assert c.train.num_rollouts == 10 and c.train.trainer == "PPOTrainer"
    assert c.generation.gen_experience_kwargs["top_k"] == 50
    assert c.tokenizer.params == {"truncation_side": "right"}
    m = build_role_model(c.model.actor)
    assert m.linear.in_features == 10
    ppo = c.to_ppo_config()
    assert ppo.ppo_epochs == 2 and ppo.temperature == 0.0 and ppo.max_new_tokens == 512 and ppo.top_k == 50
    # round trip
    c2 = AtorchRLConfig.from_dict(c.to_dict())
    assert c2.to_dict() == c.to_dict()


def _llama_yaml(tmp_path, prompts_path):
    role = {"model_cls": "dlrover_wuqiong_amd.models.llama.Llama", "model_params": {"config": {
        "vocab_size": 64, "hidden_size": 32, "intermediate_size": 64, "num_hidden_layers": 1,
        "num_attention_heads": 2, "num_key_value_heads": 1, "max_position_embeddings": 64}}}
    cfg = {
        "model": {"actor": dict(role, optimizer={"name": "torch.optim.adam", "kwargs": {"lr": 1e-3}}),
                  "critic": dict(role, optimizer={"name": "AdamW", "kwargs": {"lr": 1e-3}}),
                  "ref_model": dict(role)},
        "train": {"batch_size": 4, "num_rollouts": 2, "checkpoint_interval": 1,
                  "checkpoint_dir": str(tmp_path / "ckpt"), "max_grad_norm": 1.0, "seed": 3},
        "generation": {"batch_size": 4, "gen_experience_kwargs": {"max_new_tokens": 4, "do_sample": True,
                                                                  "temperature": 1.0, "top_k": 0}},
        "method": {"PPOConfig": {"ppo_epoch": 1}},
        "data": {"prompt_path": str(prompts_path), "max_prompt_length": 6, "pad_token_id": 0},
    }
    p = tmp_path / "rl.yaml"
    p.write_text(yaml.safe_dump(cfg))
    return p


def test_rl_train_from_yaml(tmp_path):
    from dlrover_wuqiong_amd.atorch.rl.main import parse_args, rl_train
    from dlrover_wuqiong_amd.atorch.rl.rl_config import AtorchRLConfig, build_engine, create_dataset

    prompts = tmp_path / "prompts.jsonl"
    with open(prompts, "w") as f:
        for i in range(8):
            f.write(json.dumps({"input_ids": list(range(1 + i % 5, 4 + i % 5 + i % 3))}) + "\n")
    cfg_path = _llama_yaml(tmp_path, prompts)
    c = AtorchRLConfig.load_yaml(str(cfg_path))
    ds = create_dataset(c)
    assert len(ds) == 8 and ds[0].shape == (6,)
    assert ds[0][0] == 0 and ds[0][-1] == 3  # left-padded, prompt end kept
    eng = build_engine(c, reward_fn=lambda ids: (ids[:, -4:] % 2).float().mean(-1))
    assert isinstance(eng.actor_optimizer, torch.optim.Adam)
    assert isinstance(eng.critic_optimizer, torch.optim.AdamW)
    # the ref model starts as the actor's weights when it is built from the same role config
    hist = rl_train(parse_args(["--config_file", str(cfg_path)]),
                    reward_fn=lambda ids: (ids[:, -4:] % 2).float().mean(-1))
    assert len(hist) == 2 and all("reward/mean" in h for h in hist)
    for r in (1, 2):
        assert os.path.exists(tmp_path / "ckpt" / f"rollout_{r}" / "actor.pt")


def _sync_worker(rank, world, port, q):
    import torch.distributed as dist

    from dlrover_wuqiong_amd.atorch.rl.replay_buffer import SampleReplayBuffer

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b = SampleReplayBuffer()
    for i in range(rank + 1):
        b.add_sample({"seq": torch.full((2, 3 + i), float(10 * rank + i)), "tag": f"r{rank}s{i}"})
    assert b.add_sample({"tag": "r%d-updated" % rank}, index=0)
    assert not b.add_sample({"tag": "nope"}, index=99)
    b.sync()
    q.put((rank, len(b), [t.tolist() for t in b.data["seq"]], list(b.data["tag"])))
    dist.destroy_process_group()


def test_replay_buffer_sync_two_ranks():
    import torch.multiprocessing as mp

    from dlrover_wuqiong_amd.common.rpc import find_free_port

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = find_free_port()
    ps = [ctx.Process(target=_sync_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    (_, n0, seq0, tag0), (_, n1, seq1, tag1) = out
    assert n0 == n1 == 3
    assert seq0 == seq1 and tag0 == tag1 == ["r0-updated", "r1-updated", "r1s1"]
    assert seq0[0] == torch.full((2, 3), 0.0).tolist()
    assert seq0[2] == torch.full((2, 4), 11.0).tolist()


def test_replay_buffer_dataset():
    from atorch.rl.replay_buffer import ReplayBuffer

    b = ReplayBuffer(None, element_keys=["a", "b"])
    b.add_samples([{"a": 1, "b": 2}, {"a": 3, "b": 4}])
    with pytest.raises(KeyError):
        b.add_sample({"c": 0})
    ds = b.create_dataset()
    assert len(ds) == 2 and ds[1] == {"a": 3, "b": 4}
    b.reset()
    assert len(b) == 0


def test_atorch_compat_import_paths():
    """Reference ATorch import paths resolve onto this framework."""
    from atorch.fault_tolerance import HangingDetector  # noqa: F401
    from atorch.modules.distributed_transformer import context_parallel_attention  # noqa: F401
    from atorch.modules.moe import MoELayer, TopkGate  # noqa: F401
    from atorch.modules.transformer import CrossEntropyLoss  # noqa: F401
    from atorch.modules.transformer.layers import flash_attn_varlen_func  # noqa: F401
    from atorch.mup import MuAdam, OutputLayer, set_base_shapes  # noqa: F401
    from atorch.normalization import AtorchLayerNorm
    from atorch.ops.quantizer import CUDAQuantizer

    x = torch.randn(4, 16)
    ln = AtorchLayerNorm(16)
    assert ln(x).shape == x.shape
    c, p = CUDAQuantizer().quantize(torch.randn(8000))
    assert c.dtype == torch.int8 and p.shape[1] == 2


def test_actor_critic_ref_cost_model_and_role_strategies(tmp_path):
    """One ``actor_critic_ref`` model (critic = value head on the actor's
    trunk, frozen ref snapshot), a cost model subtracted from the reward,
    and per-role strategies (a frozen role transformed by its
    inference_strategy) -- reference model_engine.py:94-188,463-481."""
    import torch.nn as nn

    from dlrover_wuqiong_amd.atorch.rl.config import PPOConfig
    from dlrover_wuqiong_amd.atorch.rl.engine import SharedCritic
    from dlrover_wuqiong_amd.atorch.rl.rl_config import AtorchRLConfig, build_engine
    from dlrover_wuqiong_amd.atorch.rl.trainer import PPOTrainer

    role = {"model_cls": "dlrover_wuqiong_amd.models.llama.Llama", "model_params": {"config": {
        "vocab_size": 64, "hidden_size": 32, "intermediate_size": 64, "num_hidden_layers": 1,
        "num_attention_heads": 2, "num_key_value_heads": 1, "max_position_embeddings": 64}}}
    cfg = {"model": {"actor_critic_ref": dict(role, optimizer={"name": "AdamW", "kwargs": {"lr": 1e-3}}),
                     "cost_model": dict(role, inference_strategy=["half"])},
           "train": {"batch_size": 4}, "method": {"PPOConfig": {"ppo_epoch": 1}}}
    c = AtorchRLConfig.from_dict(cfg)
    eng = build_engine(c, reward_fn=lambda ids: (ids[:, -3:] % 2).float().mean(-1))
    assert isinstance(eng.critic, SharedCritic) and eng.actor_critic_ref is not None
    # the critic's optimizer owns only the value head; the trunk is the actor's
    head = {id(p) for p in eng.critic.v_head.parameters()}
    assert {id(p) for g in eng.critic_optimizer.param_groups for p in g["params"]} == head
    trunk = {id(p) for g in eng.actor_optimizer.param_groups for p in g["params"]}
    assert not (trunk & head) and len(trunk) == len(list(eng.actor.parameters()))
    assert not any(p.requires_grad for p in eng.ref_model.parameters())
    assert next(eng.cost_model.parameters()).dtype == torch.bfloat16  # its inference strategy ran
    assert isinstance(eng.actor_critic_ref, nn.Module)

    torch.manual_seed(0)
    prompts = torch.randint(1, 64, (4, 5))
    tr = PPOTrainer(eng, [prompts[i] for i in range(4)], PPOConfig(max_new_tokens=3, rollout_batch_size=4,
                                                                   mini_batch_size=2, ppo_epochs=1, cost_coef=0.5))
    before = [p.detach().clone() for p in eng.actor.parameters()]
    tr.make_experience(prompts)
    assert hasattr(tr, "_cost")
    stats = tr.rl_training()
    assert all(v == v for v in stats.values())
    assert any(not torch.equal(a, b) for a, b in zip(before, eng.actor.parameters()))
