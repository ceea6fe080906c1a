"""Per-file ATorch import paths (reference module layout) resolve onto the
native implementations, and clip_grad_norm clips like torch."""

import importlib

import pytest
import torch
import torch.nn as nn

PATHS = {
    "atorch.optimizers.agd": ["AGD"],
    "atorch.optimizers.wsam": ["WeightedSAM"],
    "atorch.optimizers.bf16_optimizer": ["BF16Optimizer", "model_grads_to_master_grads"],
    "atorch.optimizers.adam_offload": ["PartitionAdam"],
    "atorch.utils.loss_spike_utils": ["TokenLossSpike", "LossSpikeBase"],
    "atorch.utils.numberic_checker": ["module_numberic_checker"],
    "atorch.data.elastic_dataset": ["ElasticDataset", "SimpleElasticDataset"],
    "atorch.data.unordered_dataloader": ["UnorderedDataLoader"],
    "atorch.data.shm_dataloader": ["ShmDataloader", "create_shm_dataloader"],
    "atorch.data.preloader": ["GpuPreLoader"],
    "atorch.fault_tolerance.hanging_detector": ["HangingDetector"],
    "atorch.trainer.atorch_args": ["AtorchArguments"],
    "atorch.trainer.atorch_trainer": ["AtorchTrainer", "count_model_params"],
    "atorch.mup.module": ["MupModule", "OutputLayer", "SharedOutputLayer"],
    "atorch.mup.optim": ["MuAdam", "MuSGD"],
    "atorch.mup.shape": ["set_base_shapes", "make_base_shapes"],
    "atorch.mup.init": ["normal_", "xavier_uniform_"],
    "atorch.normalization.layernorm": ["AtorchLayerNorm"],
    "atorch.auto.clip_grad_norm": ["clip_grad_norm"],
}


@pytest.mark.parametrize("mod", sorted(PATHS))
def test_reference_module_paths_import(mod):
    m = importlib.import_module(mod)
    for name in PATHS[mod]:
        assert getattr(m, name) is not None, f"{mod}.{name}"


def test_clip_grad_norm_matches_torch():
    from atorch.auto.clip_grad_norm import clip_grad_norm
    from atorch.trainer.atorch_trainer import count_model_params

    torch.manual_seed(0)
    a = nn.Sequential(nn.Linear(8, 16), nn.ReLU(), nn.Linear(16, 4))
    b = nn.Sequential(nn.Linear(8, 16), nn.ReLU(), nn.Linear(16, 4))
    b.load_state_dict(a.state_dict())
    x = torch.randn(5, 8)
    for m in (a, b):
        (m(x) ** 2).sum().mul(100).backward()
    n1 = clip_grad_norm(a, 0.5)
    n2 = torch.nn.utils.clip_grad_norm_(b.parameters(), 0.5)
    assert torch.allclose(n1, n2)
    for p, q in zip(a.parameters(), b.parameters()):
        assert torch.allclose(p.grad, q.grad)
    assert count_model_params(a) == sum(p.numel() for p in a.parameters())
    assert clip_grad_norm(nn.Linear(2, 2), 1.0) is None
