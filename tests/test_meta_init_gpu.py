"""Meta-device FSDP2 init on the GPU (one rank over RCCL): a tiny Llama
built on the meta device is sharded by auto_accelerate, materialised on
cuda:0 with the deterministic per-shard init, equals the same init of the
unsharded model on the GPU, and trains."""

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_gpu_meta_llama_fsdp_init_and_step(monkeypatch):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import torch.distributed as dist

    from conftest import free_port
    from dlrover_wuqiong_amd.atorch.auto_accelerate import auto_accelerate
    from dlrover_wuqiong_amd.atorch.meta_init import deterministic_init_
    from dlrover_wuqiong_amd.models.llama import Llama, LlamaConfig, LlamaDecoderLayer

    for k, v in dict(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), RANK="0", WORLD_SIZE="1",
                     LOCAL_RANK="0", LOCAL_WORLD_SIZE="1").items():
        monkeypatch.setenv(k, v)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    try:
        cfg = LlamaConfig.named("llama-tiny")
        with torch.device("meta"):
            model = Llama(cfg)
        ok, res, _ = auto_accelerate(model, torch.optim.AdamW, optim_args={"lr": 1e-3},
                                     load_strategy=[("amp_native", {"dtype": torch.bfloat16}),
                                                    ("fsdp", {"wrap_cls": (LlamaDecoderLayer,)})])
        assert ok
        with torch.device("cuda"):
            ref = Llama(cfg)
        deterministic_init_(ref)
        for (n, p), (_n2, r) in zip(res.model.named_parameters(), ref.named_parameters()):
            assert p.to_local().is_cuda and torch.equal(p.full_tensor(), r), n
        ids = torch.randint(0, cfg.vocab_size, (2, 65), device="cuda")
        losses = []
        for _ in range(3):
            loss = res.model(ids[:, :-1], ids[:, 1:])
            loss.backward()
            res.optim.step()
            res.optim.zero_grad()
            losses.append(float(loss))
        assert all(v == v for v in losses) and losses[-1] < losses[0], losses
    finally:
        dist.destroy_process_group()
