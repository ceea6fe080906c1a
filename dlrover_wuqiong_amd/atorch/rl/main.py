"""RLHF entry point: ``python -m dlrover_wuqiong_amd.atorch.rl.main --config_file my_config.yml``
(also ``python -m atorch.rl.main``), launched per rank by ``dwamd-run``.

Loads the ``AtorchRLConfig``, initialises the process group when launched
distributed (RCCL on MI355X, gloo on CPU), builds the four role models and
their optimizers, the prompt dataset, and runs ``train.num_rollouts`` PPO
rollouts with checkpoints every ``train.checkpoint_interval``.

Parity: ATorch ``atorch/rl/main.py`` (rl_train).
"""

import argparse
import os

import torch


def parse_args(argv=None):
    p = argparse.ArgumentParser(description="ATorch-compatible PPO (RLHF) training")
    p.add_argument("--config_file", type=str, default="my_config.yml")
    return p.parse_args(argv)


def rl_train(args, reward_fn=None, prompts=None):
    from .rl_config import AtorchRLConfig, build_engine, create_dataset
    from .trainer import PPOTrainer

    config = AtorchRLConfig.load_yaml(args.config_file) if isinstance(args.config_file, str) else args.config_file
    device = torch.device("cpu")
    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) > 1:
        from ..distributed import init_distributed

        init_distributed("nccl" if torch.cuda.is_available() else "gloo")
    if torch.cuda.is_available():
        device = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
        torch.cuda.set_device(device)
    torch.manual_seed(config.train.seed)
    engine = build_engine(config, device=device, reward_fn=reward_fn)
    dataset = create_dataset(config, prompts=prompts)
    trainer = PPOTrainer(engine, dataset, config.to_ppo_config())
    return trainer.train(config.train.num_rollouts, checkpoint_interval=config.train.checkpoint_interval,
                         checkpoint_dir=config.train.checkpoint_dir)


def main(argv=None):
    rl_train(parse_args(argv))


if __name__ == "__main__":
    main()
