"""ATorch utilities: activation offload checkpoint, numerics checker, loss
spike recorder/decoder, throughput timer, meta-device init.
Parity: reference atorch/tests/... test_selective_offloading_checkpoint.py,
test_numberic_checker.py, test_loss_spike_utils.py, test_meta_model_utils.py."""

import numpy as np
import torch


def _gpt2():
    from dlrover_wuqiong_amd.models.gpt2 import GPT2, GPT2Config

    torch.manual_seed(0)
    return GPT2(GPT2Config(vocab_size=64, n_positions=16, n_layer=2, n_head=2, n_embd=32))


def test_offload_checkpoint_preserves_gradients():
    import copy

    from dlrover_wuqiong_amd.atorch.offload_checkpoint import OffloadActivations, apply_offload_checkpoint
    from dlrover_wuqiong_amd.models.gpt2 import Block

    m = _gpt2()
    ref = copy.deepcopy(m)
    ids = torch.randint(0, 64, (2, 16))
    ref(ids, ids).backward()
    assert apply_offload_checkpoint(m, (Block,), min_bytes=0) == 2
    m(ids, ids).backward()
    for (n, p), q in zip(m.named_parameters(), ref.parameters()):
        assert torch.allclose(p.grad, q.grad, atol=1e-6), n
    with OffloadActivations(min_bytes=0) as off:
        x = torch.randn(8, 8, requires_grad=True)
        (x @ x).sum().backward()
    assert off.offloaded_bytes > 0 and torch.allclose(x.grad, (torch.ones(8, 8) @ x.T + x.T @ torch.ones(8, 8)))


def test_numeric_checker_finds_divergent_module(tmp_path):
    from dlrover_wuqiong_amd.atorch.utils.numeric_checker import module_numeric_checker

    m = _gpt2()
    ids = torch.randint(0, 64, (2, 16))
    c = module_numeric_checker(m, "save", str(tmp_path))
    m(ids)
    c.detach()
    c2 = module_numeric_checker(m, "compare", str(tmp_path), rtol=1e-5, atol=1e-6)
    m(ids)
    assert c2.first_mismatch() is None and len(c2.report()) > 5
    c2.detach()
    with torch.no_grad():
        m.h[1].mlp.c_fc.weight.add_(0.1 * torch.randn_like(m.h[1].mlp.c_fc.weight))  # (a constant shift is cancelled by the LayerNorm)
    c3 = module_numeric_checker(m, "compare", str(tmp_path), rtol=1e-5, atol=1e-6)
    m(ids)
    bad = c3.first_mismatch()
    assert bad is not None and bad[0].startswith("h.1")


def test_loss_spike_record_and_decode(tmp_path):
    from dlrover_wuqiong_amd.atorch.utils.loss_spike import TokenLossSpike, losses_to_str

    data = tmp_path / "corpus"
    (tmp_path / "corpus.scatter" / "3.lazy").mkdir(parents=True)
    toks = np.arange(40, dtype=np.int32).reshape(5, 8)
    toks.tofile(tmp_path / "corpus.scatter" / "3.lazy" / "text")
    spikes = tmp_path / "spikes"
    spikes.mkdir()
    ls = TokenLossSpike(str(spikes), [("wiki", str(data))], each_sample_len=8, min_iter=10, min_loss=4.0)
    assert not ls.save_loss("r0.txt", 9.0, 5, losses_str="1,2", sample_infos_str="3-0-0-0-1,3-0-0-0-2")
    assert ls.save_loss("r0.txt", 9.0, 20, losses_str=losses_to_str([1.0, 7.5]),
                        sample_infos_str="3-0-0-0-1,3-0-0-0-4")

    class Tok:
        def decode(self, ids):
            return " ".join(map(str, ids))

    out = tmp_path / "decoded.txt"
    assert ls.decode_loss_spike(str(out), Tok()) == 1
    text = out.read_text()
    assert "wiki" in text and "32 33 34 35 36 37 38 39" in text  # sample 4 had the max loss


def test_throughput_timer_and_timers():
    from dlrover_wuqiong_amd.atorch.utils.timer import ThroughputTimer, Timers

    msgs = []
    t = ThroughputTimer(batch_size=8, start_step=1, steps_per_output=2, logging_fn=msgs.append)
    for _ in range(5):
        t.start()
        sum(range(20000))
        t.stop()
    assert t.avg_samples_per_sec() > 0 and msgs
    tm = Timers()
    tm.start("x")
    sum(range(10000))
    tm.stop("x")
    assert tm.elapsed("x") > 0


def test_meta_init_materialize_and_load(tmp_path):
    from safetensors.torch import save_file

    from dlrover_wuqiong_amd.atorch.utils.meta_init import (find_tied_parameters, init_empty_weights, is_meta,
                                                            load_state_dict_to_meta, materialize)

    class Tied(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.emb = torch.nn.Embedding(10, 4)
            self.head = torch.nn.Linear(4, 10, bias=False)
            self.head.weight = self.emb.weight

    with init_empty_weights():
        m = Tied()
    assert is_meta(m) and find_tied_parameters(m) == [["emb.weight", "head.weight"]]
    materialize(m, device="cpu")
    assert not is_meta(m) and m.head.weight is m.emb.weight and float(m.emb.weight.abs().sum()) > 0
    src = Tied()
    save_file({"emb.weight": src.emb.weight.detach().clone()}, str(tmp_path / "w.safetensors"))
    with init_empty_weights():
        m2 = Tied()
    load_state_dict_to_meta(m2, str(tmp_path / "w.safetensors"), device="cpu")
    assert torch.equal(m2.head.weight, src.emb.weight)
