"""ElasticTrainer / ElasticDistributedSampler / ElasticDataLoader
(parity: reference trainer/tests/torch/elastic_test.py)."""

import json
import os

import torch
from torch.utils.data import TensorDataset


def test_grad_accum_keeps_global_batch(monkeypatch):
    from dlrover_wuqiong_amd.trainer.elastic import ElasticTrainer

    monkeypatch.setenv("WORKER_NUM", "4")
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "2")
    monkeypatch.setenv("WORLD_SIZE", "3")
    for rank, expect in ((0, 3), (1, 3), (2, 2)):
        monkeypatch.setenv("RANK", str(rank))
        t = ElasticTrainer(torch.nn.Linear(2, 2))
        t._set_gradient_accumulation_steps()
        assert t.gradient_accumulation_steps == expect  # 8 = 3 + 3 + 2


def test_step_context_only_syncs_every_accum(monkeypatch, tmp_path):
    from dlrover_wuqiong_amd.trainer.elastic import ElasticTrainer

    monkeypatch.setenv("WORKER_NUM", "2")
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "1")
    monkeypatch.setenv("WORLD_SIZE", "1")
    monkeypatch.setenv("RANK", "0")
    metrics = tmp_path / "m" / "runtime_metrics.json"
    monkeypatch.setenv("RUNTIME_METRICS_PATH", str(metrics))
    model = torch.nn.Linear(4, 1)
    trainer = ElasticTrainer(model, report_interval=0)
    opt = trainer.prepare(torch.optim.SGD(model.parameters(), lr=0.1))
    assert trainer.gradient_accumulation_steps == 2
    w0 = model.weight.detach().clone()
    with trainer.step(fix_total_batch_size=True):
        model(torch.ones(1, 4)).sum().backward()
        opt.step()
    assert torch.equal(model.weight, w0)  # accumulated, not stepped
    with trainer.step(fix_total_batch_size=True):
        model(torch.ones(1, 4)).sum().backward()
        opt.step()
    assert not torch.equal(model.weight, w0)
    assert trainer.num_steps == 1
    assert json.loads(metrics.read_text())["step"] == 1


def test_sampler_resumes_mid_epoch_with_new_world():
    from dlrover_wuqiong_amd.trainer.elastic import ElasticDistributedSampler

    ds = TensorDataset(torch.arange(100))
    samplers = [ElasticDistributedSampler(ds, num_replicas=2, rank=r, shuffle=True, seed=3) for r in range(2)]
    seen = [list(iter(s))[:10] for s in samplers]  # 10 local steps of batch 1
    state = samplers[0].state_dict(iter_step=10, micro_batch_size=1)
    assert state["completed_num"] == 20
    # resume with 4 replicas: the union of what remains is exactly the unseen samples
    new = [ElasticDistributedSampler(ds, num_replicas=4, rank=r, shuffle=True, seed=3) for r in range(4)]
    for s in new:
        s.load_state_dict(state)
    rest = set()
    for s in new:
        rest.update(iter(s))
    done = set(seen[0]) | set(seen[1])
    assert rest.isdisjoint(done) and rest | done == set(range(100))


def test_elastic_dataloader_reads_config(tmp_path):
    from dlrover_wuqiong_amd.trainer.elastic import ElasticDataLoader

    cfg = tmp_path / "paral.json"
    ds = TensorDataset(torch.arange(64))
    dl = ElasticDataLoader(ds, batch_size=4, config_file=str(cfg))
    assert next(iter(dl))[0].numel() == 4
    cfg.write_text(json.dumps({"dataloader": {"version": 1, "batch_size": 16}}))
    dl.update_batch_size()
    assert next(iter(dl))[0].numel() == 16
