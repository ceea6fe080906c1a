"""Megatron-LM / DeepSpeed / HF-Trainer flash checkpointers on CPU.

Megatron-LM and DeepSpeed are not installed: a minimal stand-in package /
engine with their save/load call pattern (``torch.save`` to their file
layout + tracker files) drives the interception path.  Parity: reference
``dlrover/trainer/tests/torch/{megatron,deepspeed}_ckpt_test.py``."""

import os
import sys
import textwrap
import time

import pytest
import torch


def _wait_file(path, content=None, timeout=60):
    deadline = time.time() + timeout
    while time.time() < deadline:
        if os.path.exists(path):
            if content is None or open(path).read().strip() == content:
                return True
        time.sleep(0.05)
    return False


def test_megatron_native_layout(tmp_path):
    from dlrover_wuqiong_amd.flash_checkpoint.checkpointer import StorageType
    from dlrover_wuqiong_amd.flash_checkpoint.megatron import MegatronCheckpointer

    d = str(tmp_path / "mg")
    ck = MegatronCheckpointer(d)
    sd = {"model": {"w": torch.arange(10.0)}, "rng": torch.get_rng_state()}
    assert ck.save_checkpoint(4, sd, storage_type=StorageType.DISK)
    assert _wait_file(os.path.join(d, "latest_checkpointed_iteration.txt"), "4")
    assert open(os.path.join(d, "dlrover_latest.txt")).read() == "4"
    x = torch.load(os.path.join(d, "iter_0000004", "mp_rank_00", "model_optim_rng.pt"), weights_only=True)
    assert torch.equal(x["model"]["w"], torch.arange(10.0)) and x["iteration"] == 4
    sd["model"]["w"] += 1
    assert ck.save_checkpoint(6, sd, storage_type=StorageType.MEMORY)
    it, out = ck.load_checkpoint()
    assert it == 6 and torch.equal(out["model_states"]["model"]["w"], torch.arange(10.0) + 1)
    ck.close()


FAKE_MEGATRON = {
    "megatron/__init__.py": "",
    "megatron/training/__init__.py": """
        import types
        ARGS = types.SimpleNamespace(save=None, load=None, use_distributed_optimizer=False)
        def get_args():
            return ARGS
    """,
    "megatron/training/checkpointing.py": """
        import os
        import torch
        from megatron.training import get_args

        def _name(d, it):
            return os.path.join(d, f"iter_{it:07d}", "mp_rank_00", "model_optim_rng.pt")

        def save_checkpoint(iteration, model, optimizer, opt_param_scheduler,
                            num_floating_point_operations_so_far=0):
            args = get_args()
            path = _name(args.save, iteration)
            os.makedirs(os.path.dirname(path), exist_ok=True)
            torch.save({"model": model.state_dict(), "optimizer": optimizer.state_dict(),
                        "iteration": iteration}, path)
            with open(os.path.join(args.save, "latest_checkpointed_iteration.txt"), "w") as f:
                f.write(str(iteration))

        def load_checkpoint(model, optimizer, opt_param_scheduler, load_arg="load", strict=True):
            args = get_args()
            d = getattr(args, load_arg)
            t = os.path.join(d, "latest_checkpointed_iteration.txt")
            if not os.path.exists(t):
                return 0
            it = int(open(t).read())
            sd = torch.load(_name(d, it), map_location="cpu", weights_only=False)
            model.load_state_dict(sd["model"], strict=strict)
            optimizer.load_state_dict(sd["optimizer"])
            return sd["iteration"]
    """,
}


@pytest.fixture
def fake_megatron(tmp_path, monkeypatch):
    root = tmp_path / "fake_pkgs"
    for rel, src in FAKE_MEGATRON.items():
        p = root / rel
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_text(textwrap.dedent(src))
    monkeypatch.syspath_prepend(str(root))
    for m in [m for m in sys.modules if m == "megatron" or m.startswith("megatron.")]:
        monkeypatch.delitem(sys.modules, m)
    import megatron.training as mt

    yield mt
    for m in [m for m in sys.modules if m == "megatron" or m.startswith("megatron.")]:
        del sys.modules[m]


def test_megatron_lm_wrappers(tmp_path, fake_megatron):
    from dlrover_wuqiong_amd.flash_checkpoint import megatron as fm
    from dlrover_wuqiong_amd.flash_checkpoint.checkpointer import StorageType

    d = str(tmp_path / "mlm")
    fake_megatron.ARGS.save = fake_megatron.ARGS.load = d
    model = torch.nn.Linear(4, 4)
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    assert fm.save_checkpoint(10, model, opt, None, storage_type=StorageType.DISK)
    assert _wait_file(os.path.join(d, "dlrover_latest.txt"), "10")
    assert open(os.path.join(d, "latest_checkpointed_iteration.txt")).read() == "10"
    assert os.path.exists(os.path.join(d, "iter_0000010", "mp_rank_00", "model_optim_rng.pt"))
    w10 = model.weight.detach().clone()
    with torch.no_grad():
        model.weight.add_(1.0)
    w20 = model.weight.detach().clone()
    assert fm.save_checkpoint(20, model, opt, None, storage_type=StorageType.MEMORY)
    # a memory-only save leaves no directory and the tracker at the persisted step
    assert not os.path.exists(os.path.join(d, "iter_0000020"))
    assert open(os.path.join(d, "latest_checkpointed_iteration.txt")).read() == "10"
    with torch.no_grad():
        model.weight.zero_()
    it = fm.load_checkpoint(model, opt, None)
    assert it == 20 and torch.equal(model.weight, w20)  # served from memory
    assert not torch.equal(w10, w20)
    fm.MegatronCheckpointer.reset_instances()


class _FakeDeepSpeedEngine:
    """DeepSpeedEngine's checkpoint call pattern (ZeRO-1, one rank)."""

    def __init__(self, model, opt):
        self.module, self.optimizer = model, opt
        self.global_steps = 0
        self.save_non_zero_checkpoint = False

    def zero_optimization(self):
        return True

    def zero_optimization_stage(self):
        return 1

    def save_checkpoint(self, save_dir, tag, client_state, save_latest):
        d = os.path.join(save_dir, str(tag))
        os.makedirs(d, exist_ok=True)
        torch.save({"module": self.module.state_dict(), **client_state},
                   os.path.join(d, "mp_rank_00_model_states.pt"))
        torch.save({"optimizer_state_dict": self.optimizer.state_dict()},
                   os.path.join(d, "zero_pp_rank_0_mp_rank_00_optim_states.pt"))
        if save_latest:
            with open(os.path.join(save_dir, "latest"), "w") as f:
                f.write(str(tag))

    def load_checkpoint(self, load_dir, tag=None, **kw):
        if tag is None:
            tag = open(os.path.join(load_dir, "latest")).read().strip()
        d = os.path.join(load_dir, tag)
        m = torch.load(os.path.join(d, "mp_rank_00_model_states.pt"), weights_only=False)
        o = torch.load(os.path.join(d, "zero_pp_rank_0_mp_rank_00_optim_states.pt"), weights_only=False)
        self.module.load_state_dict(m["module"])
        self.optimizer.load_state_dict(o["optimizer_state_dict"])
        return d, {k: v for k, v in m.items() if k != "module"}


def test_deepspeed_checkpointer(tmp_path):
    from dlrover_wuqiong_amd.flash_checkpoint.checkpointer import StorageType
    from dlrover_wuqiong_amd.flash_checkpoint.deepspeed import DeepSpeedCheckpointer

    d = str(tmp_path / "ds")
    model = torch.nn.Linear(4, 4)
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    eng = _FakeDeepSpeedEngine(model, opt)
    ck = DeepSpeedCheckpointer(eng, d)
    assert eng.save_non_zero_checkpoint
    assert ck.save_checkpoint(d, "global_step4", {"epoch": 1}, storage_type=StorageType.DISK)
    assert _wait_file(os.path.join(d, "dlrover_latest.txt"), "4")
    assert open(os.path.join(d, "latest")).read() == "global_step4"
    assert os.path.exists(os.path.join(d, "global_step4", "zero_pp_rank_0_mp_rank_00_optim_states.pt"))
    with torch.no_grad():
        model.weight.add_(1.0)
    w8 = model.weight.detach().clone()
    assert ck.save_checkpoint(d, "global_step8", {"epoch": 2}, storage_type=StorageType.MEMORY)
    assert open(os.path.join(d, "latest")).read() == "global_step4"  # restored: step 8 is memory-only
    assert not os.path.exists(os.path.join(d, "global_step8"))
    with torch.no_grad():
        model.weight.zero_()
    path, client = ck.load_checkpoint(d)
    assert client["epoch"] == 2 and torch.equal(model.weight, w8)  # memory copy served
    ck.close()


def test_hf_flash_trainer(tmp_path):
    pytest.importorskip("transformers")
    from transformers import GPT2Config, GPT2LMHeadModel, TrainingArguments

    from dlrover_wuqiong_amd.flash_checkpoint.hf_trainer import FlashCkptTrainer

    torch.manual_seed(0)
    cfg = GPT2Config(n_layer=2, n_head=2, n_embd=32, vocab_size=64, n_positions=32)
    model = GPT2LMHeadModel(cfg)
    data = [{"input_ids": torch.randint(0, 64, (16,)), "labels": torch.randint(0, 64, (16,))} for _ in range(16)]
    out = str(tmp_path / "hf")
    args = TrainingArguments(output_dir=out, per_device_train_batch_size=4, max_steps=4, save_steps=2,
                             logging_steps=100, report_to=[], use_cpu=True, save_total_limit=3)
    tr = FlashCkptTrainer(model=model, args=args, train_dataset=data)
    tr.train()
    assert _wait_file(os.path.join(out, "dlrover_latest.txt"), "4")
    ck4 = os.path.join(out, "checkpoint-4")
    for f in ("model.safetensors", "optimizer.pt", "scheduler.pt", "trainer_state.json", "config.json"):
        assert os.path.exists(os.path.join(ck4, f)), f
    re = GPT2LMHeadModel.from_pretrained(ck4)
    for (k, a), (_, b) in zip(model.state_dict().items(), re.state_dict().items()):
        assert torch.equal(a, b), k
    opt = torch.load(os.path.join(ck4, "optimizer.pt"), weights_only=True)
    assert "state" in opt
