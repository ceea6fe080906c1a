"""AtorchTrainer: auto_accelerate-built training loop with HF callbacks,
flash-checkpoint saves, rotation and exact resume.
Parity: reference atorch/tests/.../test_atorch_trainer.py."""

import os

import pytest
import torch


class _DS(torch.utils.data.Dataset):
    def __init__(self, n=48, seq=16, vocab=64):
        g = torch.Generator().manual_seed(0)
        self.x = torch.randint(0, vocab, (n, seq + 1), generator=g)

    def __len__(self):
        return len(self.x)

    def __getitem__(self, i):
        return {"idx": self.x[i, :-1], "targets": self.x[i, 1:]}


def _model():
    from dlrover_wuqiong_amd.models.gpt2 import GPT2, GPT2Config

    torch.manual_seed(0)
    return GPT2(GPT2Config(vocab_size=64, n_positions=16, n_layer=2, n_head=2, n_embd=32))


def _args(out, **kw):
    from dlrover_wuqiong_amd.atorch.trainer import AtorchTrainingArgs

    base = dict(output_dir=str(out), per_device_train_batch_size=4, max_steps=6, save_steps=3, logging_steps=2,
                learning_rate=1e-3, shuffle=False, atorch_opt="none", atorch_module_replace=False,
                disable_tqdm=True, save_total_limit=1, seed=7, use_cpu=True, flash_checkpoint=True)
    base.update(kw)
    return AtorchTrainingArgs(**base)


@pytest.mark.parametrize("flash", [True, False])
def test_trainer_trains_saves_rotates_and_resumes_exactly(tmp_path, flash):
    from transformers import TrainerCallback

    from dlrover_wuqiong_amd.atorch.trainer import AtorchTrainer

    events = []

    class Rec(TrainerCallback):
        def on_save(self, args, state, control, **kw):
            events.append(("save", state.global_step))

        def on_log(self, args, state, control, logs=None, **kw):
            events.append(("log", state.global_step))

    a = AtorchTrainer(_model(), _args(tmp_path / "a", flash_checkpoint=flash), train_dataset=_DS(),
                      callbacks=[Rec()])
    m = a.train()
    assert m["global_step"] == 6
    assert ("save", 3) in events and ("save", 6) in events and ("log", 2) in events
    a.close()
    cks = sorted(os.listdir(tmp_path / "a"))
    assert "checkpoint-6" in cks and "checkpoint-3" not in cks  # save_total_limit=1
    assert any(h.get("loss") is not None for h in a.state.log_history)
    final_a = {k: v.clone() for k, v in a.model.state_dict().items()}

    # run b: stop at step 3 (checkpoint), then resume in a fresh trainer to step 6
    class Stop(TrainerCallback):
        def on_step_end(self, args, state, control, **kw):
            if state.global_step == 3:
                control.should_training_stop = True

    b = AtorchTrainer(_model(), _args(tmp_path / "b", save_total_limit=None, flash_checkpoint=flash),
                      train_dataset=_DS(), callbacks=[Stop()])
    assert b.train()["global_step"] == 3
    b.close()
    c = AtorchTrainer(_model(), _args(tmp_path / "b", flash_checkpoint=flash), train_dataset=_DS())
    c.train(resume_from_checkpoint=True)
    c.close()
    for k, v in c.model.state_dict().items():
        assert torch.allclose(v, final_a[k], atol=1e-6), k
    c.save_model(str(tmp_path / "final"))
    from safetensors.torch import load_file

    w = load_file(str(tmp_path / "final" / "model.safetensors"))
    assert torch.equal(w["wte.weight"], final_a["wte.weight"])
