"""Optimizer step inside the FSDP2 backward (optimizers/in_backward.py) on one
GPU over RCCL: a tiny Llama under auto_accelerate zero2 with
``optim_in_backward`` trains bit-identically to the plain multi-tensor step
(same kernel, same math), every unit's update is launched from its
post-backward, and a flash checkpoint taken between steps restores."""

import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(in_backward: bool, steps: int = 4):
    from dlrover_wuqiong_amd.atorch.auto_accelerate import auto_accelerate
    from dlrover_wuqiong_amd.models.llama import Llama, LlamaConfig, LlamaDecoderLayer

    torch.manual_seed(0)
    cfg = LlamaConfig.named("llama-tiny")
    with torch.device("cuda"):
        model = Llama(cfg)
    ok, res, _ = auto_accelerate(model, torch.optim.AdamW, optim_args={"lr": 1e-3, "weight_decay": 0.1},
                                 load_strategy=["half", ("zero2", {"wrap_cls": (LlamaDecoderLayer,),
                                                                   "optim_in_backward": in_backward})])
    assert ok
    m, opt = res.model, res.optim
    ib = getattr(opt, "_in_backward", None)
    assert (ib is not None) == in_backward
    g = torch.Generator(device="cpu").manual_seed(1)
    ids = torch.randint(0, cfg.vocab_size, (steps, 2, 65), generator=g).cuda()
    losses = []
    for i in range(steps):
        loss = m(ids[i, :, :-1], ids[i, :, 1:])
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
        losses.append(float(loss))
    torch.cuda.synchronize()
    state = [p.to_local().clone() for p in m.parameters()]
    bufs = {k: v.clone() for d in opt.flat_state_buffers().values() for k, v in d.items()}
    return losses, state, bufs, ib, opt.step_count


def test_gpu_optimizer_in_backward_matches_plain_step(monkeypatch):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import torch.distributed as dist

    from conftest import free_port

    for k, v in dict(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), RANK="0", WORLD_SIZE="1",
                     LOCAL_RANK="0", LOCAL_WORLD_SIZE="1").items():
        monkeypatch.setenv(k, v)
    monkeypatch.setenv("DWAMD_DETERMINISTIC", "1")  # bit-reproducible gradients: the runs compare bitwise
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    try:
        l0, s0, b0, _, n0 = _run(False)
        l1, s1, b1, ib, n1 = _run(True)
        assert n0 == n1 == 4
        units = len(ib.units)
        assert units >= 3 and ib.units_launched == 4 * units, (units, ib.units_launched)
        assert l0 == l1, (l0, l1)
        for a, b in zip(s0, s1):
            assert torch.equal(a, b)
        for k in b0:
            assert torch.equal(b0[k], b1[k]), k
    finally:
        dist.destroy_process_group()
