"""The user-facing examples (mirrors of the reference's atorch/examples and
examples/pytorch) run end to end on CPU / gloo with tiny configs: they are
the switching guide, so they must keep working as the APIs evolve."""

import os
import re
import subprocess
import sys

import pytest
import torch

from conftest import free_port

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EX = os.path.join(REPO, "examples")


def _run(args, cwd, nproc=1, timeout=300):
    env = dict(os.environ, PYTHONPATH=REPO, CUDA_VISIBLE_DEVICES="")
    if nproc > 1:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", str(nproc), "--master-addr",
               "127.0.0.1", "--master-port", str(free_port())] + args
    else:
        cmd = [sys.executable] + args
    p = subprocess.run(cmd, cwd=cwd, env=env, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    return p.stdout


def _losses(out):
    m = re.search(r"first_loss=([\d.]+) last_loss=([\d.]+)", out)
    assert m, out[-2000:]
    return float(m.group(1)), float(m.group(2))


@pytest.mark.parametrize("flags", [
    ["--model_type", "toy", "--load_strategy", "--epoch", "1"],
    ["--model_type", "toy", "--user_created_dataloader", "--optim_grouped_params", "--max_steps", "6"],
    ["--model_type", "toy", "--load_strategy", "--use_fp8", "--batchsize", "16", "--max_steps", "6"],
    ["--model_type", "gpt2", "--load_strategy", "--use_checkpointing", "--use_amp", "--max_steps", "4",
     "--layer_num", "2"],
])
def test_auto_accelerate_example_single(flags):
    out = _run(["train.py"] + flags, os.path.join(EX, "auto_accelerate"))
    first, last = _losses(out)
    assert last == last and first == first
    if flags[1] == "toy":
        assert last < first


def test_auto_accelerate_example_fsdp_two_ranks():
    out = _run(["train.py", "--model_type", "llama", "--distributed", "--load_strategy", "--use_fsdp",
                "--use_module_replace", "--max_steps", "3", "--layer_num", "2", "--log_interval", "1"],
               os.path.join(EX, "auto_accelerate"), nproc=2)
    assert "strategy: ['parallel_mode', 'module_replace', 'fsdp']" in out, out[-2000:]
    _losses(out)


def test_auto_accelerate_example_flat_fsdp_two_ranks():
    out = _run(["train.py", "--model_type", "llama", "--distributed", "--load_strategy", "--use_flat_fsdp",
                "--max_steps", "4", "--layer_num", "2", "--log_interval", "1"],
               os.path.join(EX, "auto_accelerate"), nproc=2)
    assert "strategy: ['parallel_mode', 'flat_fsdp']" in out, out[-2000:]
    first, last = _losses(out)
    assert abs(first) < 20 and abs(last) < 20


def test_llama2_fsdp_example():
    out = _run(["fsdp_llama2.py", "--max_steps", "3", "--gradient_checkpointing"], os.path.join(EX, "llama2"))
    assert out.count("iter ") == 3


def test_llama2_3d_example_tp2_pp2():
    out = _run(["ds_3d_llama2.py", "--model_parallel_size", "2", "--pipeline_parallel_size", "2", "--max_steps",
                "3", "--num_layers", "4"], os.path.join(EX, "llama2"), nproc=4)
    assert "3D parallel: tensor 2, pipeline 2, data 1" in out
    losses = [float(x) for x in re.findall(r"iter \d+: loss ([\d.]+)", out)]
    assert len(losses) == 3 and all(0 < x < 20 for x in losses), out[-2000:]


def test_nanogpt_example_saves_and_resumes(tmp_path):
    ck = str(tmp_path / "ck")
    cwd = os.path.join(EX, "nanogpt")
    out = _run(["train.py", "--max_iters", "4", "--save_memory_interval", "2", "--save_storage_interval", "4",
                "--save_dir", ck], cwd)
    assert "flash save (memory) step 4" in out
    assert open(os.path.join(ck, "dlrover_latest.txt")).read().strip() == "4"
    # a fresh process resumes at the persisted step, then LoRA fine-tunes on top
    out = _run(["train.py", "--max_iters", "6", "--save_memory_interval", "100", "--save_storage_interval", "100",
                "--save_dir", ck, "--lora_rank", "4", "--lora_targets", "c_attn"], cwd)
    assert "resumed at step 4" in out and "LoRA" in out and "iter 6:" in out, out[-2000:]


def test_lora_adapter_semantics():
    from dlrover_wuqiong_amd.atorch.lora import apply_lora, lora_state_dict, merge_lora
    from dlrover_wuqiong_amd.models.gpt2 import GPT2, GPT2Config

    torch.manual_seed(0)
    m = GPT2(GPT2Config.named("gpt2-tiny"))
    base_sd = {k: v.clone() for k, v in m.state_dict().items()}
    x = torch.randint(0, 1024, (2, 17))
    y0 = m(x).detach()
    names = apply_lora(m, ["c_attn", "c_fc"], rank=4, alpha=8)
    assert len(names) == 4 and torch.allclose(m(x), y0)  # B = 0: identical at start
    trainable = [n for n, p in m.named_parameters() if p.requires_grad]
    assert trainable and all("lora_" in n for n in trainable)
    opt = torch.optim.AdamW([p for p in m.parameters() if p.requires_grad], lr=1e-2)
    for _ in range(3):
        m(x[:, :-1], x[:, 1:]).backward()
        opt.step()
        opt.zero_grad()
    y1 = m(x).detach()
    assert not torch.allclose(y1, y0)
    merge_lora(m)
    assert torch.allclose(m(x), y1, atol=1e-5)
    assert set(lora_state_dict(m)) == {f"{n}.lora_{s}" for n in names for s in "AB"}
    # a plain checkpoint loads into an adapted model
    m2 = GPT2(GPT2Config.named("gpt2-tiny"))
    apply_lora(m2, ["c_attn"])
    m2.load_state_dict(base_sd)
    assert torch.allclose(m2(x), y0)


def test_optimizer_example_agd_and_wsam():
    cwd = os.path.join(EX, "optimizer")
    for opt, base, lr in (("vanilla", "agd", "1e-3"), ("wsam", "sgd", "0.05")):
        out = _run(["main.py", "--optimizer", opt, "--base_optimizer", base, "--lr", lr, "--max-steps", "15",
                    "--samples", "960"], cwd)
        first, last = _losses(out)
        assert last < first, (opt, base, out[-500:])


def test_mnist_elastic_example_resumes(tmp_path):
    ck = str(tmp_path / "ck")
    cwd = os.path.join(EX, "mnist")
    first = _run(["cnn_train.py", "--max_steps", "20", "--save_memory_interval", "10", "--save_storage_interval",
                  "20", "--checkpoint_dir", ck], cwd)
    _losses(first)
    out = _run(["cnn_train.py", "--max_steps", "25", "--checkpoint_dir", ck], cwd)
    assert "resumed at step 20" in out, out[-1500:]


def test_atorch_trainer_example(tmp_path):
    out_dir = str(tmp_path / "o")
    cwd = os.path.join(EX, "llama2_trainer")
    out = _run(["llama2_clm_atorch_trainer.py", "--output_dir", out_dir, "--max_steps", "4", "--save_steps", "2",
                "--lora_rank", "4"], cwd)
    assert "global_step=4" in out, out[-1500:]
    for f in ("model.safetensors", "adapter.pt", "strategy.json", "checkpoint-4"):
        assert os.path.exists(os.path.join(out_dir, f)), f


def test_shm_checkpoint_of_another_job_is_ignored(tmp_path):
    """Two jobs in one shm namespace (no launcher run id): the second never
    restores the first one's in-memory checkpoint."""
    from dlrover_wuqiong_amd.flash_checkpoint.checkpointer import StorageType
    from dlrover_wuqiong_amd.flash_checkpoint.ddp import DdpCheckpointer

    m = torch.nn.Linear(8, 8)
    a = DdpCheckpointer(str(tmp_path / "job_a"))
    assert a.save_checkpoint(5, {"model": m.state_dict(), "step": 5}, storage_type=StorageType.MEMORY)
    got = a.load_checkpoint()
    assert got.get("step") == 5
    a.close() if hasattr(a, "close") else None
    b = DdpCheckpointer(str(tmp_path / "job_b"))
    assert not b.load_checkpoint()  # foreign shm ignored, nothing on storage
    assert b.save_checkpoint(7, {"model": m.state_dict(), "step": 7}, storage_type=StorageType.MEMORY)
    assert b.load_checkpoint().get("step") == 7


def test_moe_example_upcycled_ep2_dp2():
    """Upcycled Llama MoE, EP 2 x DP 2 with capacity, MoE-aware DDP through
    auto_accelerate: the step-0 loss equals the dense model's (up to the
    expert noise) and training reduces it."""
    out = _run(["train_moe.py", "--ep", "2", "--capacity_factor", "1.25", "--steps", "5"],
               os.path.join(EX, "moe"), nproc=4)
    m = re.search(r"loss dense ([\d.]+) -> MoE ([\d.]+)", out)
    assert m and abs(float(m.group(1)) - float(m.group(2))) < 0.01, out[-1500:]
    first, last = _losses(out)
    assert last < first and "'ddp'" in out
