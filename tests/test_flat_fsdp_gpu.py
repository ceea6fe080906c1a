"""Flat-unit FSDP on the GPU (world 1): a bf16 Llama with the fused HIP ops
trains through FlatFSDP + FusedAdamW exactly like the same model on
FlatParams (the parameters ARE the shard: same kernels, same update), and
the flat-shard flash checkpoint restores the shard + optimizer state in
place."""

import pytest
import torch

pytestmark = pytest.mark.gpu


def _model():
    from dlrover_wuqiong_amd.atorch.auto_accelerate import auto_accelerate
    from dlrover_wuqiong_amd.models.llama import Llama, LlamaConfig

    torch.manual_seed(0)
    cfg = LlamaConfig.named("llama-tiny")
    with torch.device("cuda"):
        m = Llama(cfg)
    ok, res, _ = auto_accelerate(m, load_strategy=["module_replace", "half"])
    assert ok
    return res.model, cfg


def _train(model, opt, zero, cfg, steps=3):
    g = torch.Generator().manual_seed(3)
    losses = []
    for _ in range(steps):
        x = torch.randint(0, cfg.vocab_size, (2, 129), generator=g).cuda()
        loss = model(x[:, :-1], x[:, 1:])
        loss.backward()
        opt.step()
        zero()
        losses.append(float(loss))
    torch.cuda.synchronize()
    return losses


def test_flat_fsdp_world1_matches_flat_params():
    from dlrover_wuqiong_amd.models.llama import LlamaDecoderLayer
    from dlrover_wuqiong_amd.optimizers.fused import FusedAdamW
    from dlrover_wuqiong_amd.parallel.flat import FlatParams
    from dlrover_wuqiong_amd.parallel.flat_fsdp import FlatFSDP

    m1, cfg = _model()
    flat = FlatParams(m1)
    o1 = FusedAdamW(flat, lr=1e-3, weight_decay=0.1)
    l1 = _train(m1, o1, flat.zero_grad, cfg)
    m2, _ = _model()
    fs = FlatFSDP(m2, wrap_cls=(LlamaDecoderLayer,))
    o2 = FusedAdamW(fs.shard_flat, lr=1e-3, weight_decay=0.1)
    l2 = _train(fs, o2, o2.zero_grad, cfg)
    assert l1 == pytest.approx(l2, rel=1e-3)
    p1 = dict(m1.named_parameters())
    for n, p in m2.named_parameters():
        torch.testing.assert_close(p.float(), p1[n].float(), rtol=2e-2, atol=2e-3, msg=n)


def test_flat_fsdp_flash_ckpt_in_place_gpu(tmp_path):
    import os

    from dlrover_wuqiong_amd.atorch import fsdp_flat_ckpt as ffc
    from dlrover_wuqiong_amd.flash_checkpoint.checkpointer import StorageType
    from dlrover_wuqiong_amd.models.llama import LlamaDecoderLayer
    from dlrover_wuqiong_amd.optimizers.fused import FusedAdamW
    from dlrover_wuqiong_amd.parallel.flat_fsdp import FlatFSDP

    os.environ.setdefault("DWAMD_SHM_PREFIX", f"ffg{os.getpid()}")
    m, cfg = _model()
    fs = FlatFSDP(m, wrap_cls=(LlamaDecoderLayer,))
    opt = FusedAdamW(fs.shard_flat, lr=1e-3, max_grad_norm=1.0)
    _train(fs, opt, opt.zero_grad, cfg, steps=2)
    root = str(tmp_path)
    try:
        assert ffc.save_checkpoint(2, fs, opt, os.path.join(root, "step-2"), storage_type=StorageType.MEMORY)
        ffc._engine(root).wait_for_memory_save()
        want = [t.clone() for t in (fs.shard_flat.data, opt.exp_avg, opt.exp_avg_sq, opt.master)]
        _train(fs, opt, opt.zero_grad, cfg, steps=1)
        assert ffc.load_checkpoint(fs, opt, os.path.join(root, "step-2")) == 2
        torch.cuda.synchronize()
        for a, b in zip((fs.shard_flat.data, opt.exp_avg, opt.exp_avg_sq, opt.master), want):
            assert torch.equal(a, b)
        assert opt.step_count == 2
    finally:
        ffc.close_engines()


def _two_rank_worker(rank, port, reshard, q):
    import os

    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE="2",
                      LOCAL_RANK="0", LOCAL_WORLD_SIZE="1")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=2)  # two ranks on ONE GPU: gloo over CUDA tensors
    try:
        from dlrover_wuqiong_amd.atorch.auto_accelerate import auto_accelerate
        from dlrover_wuqiong_amd.models.llama import Llama, LlamaConfig, LlamaDecoderLayer

        torch.manual_seed(0)
        cfg = LlamaConfig.named("llama-tiny")
        with torch.device("cuda"):
            m = Llama(cfg)
        ok, res, _ = auto_accelerate(m, torch.optim.AdamW, optim_args={"lr": 1e-3, "max_grad_norm": 1.0},
                                     load_strategy=["module_replace", "half",
                                                    ("flat_fsdp" if reshard else "flat_zero2",
                                                     {"wrap_cls": (LlamaDecoderLayer,)})])
        model, opt = res.model, res.optim
        assert model.world == 2 and model.reshard == reshard
        g = torch.Generator().manual_seed(3)
        losses = []
        for _ in range(3):
            x = torch.randint(0, cfg.vocab_size, (4, 129), generator=g).cuda().chunk(2)[rank]
            loss = model(x[:, :-1], x[:, 1:])
            loss.backward()
            opt.step()
            opt.zero_grad()
            t = loss.detach().float().cpu()
            dist.all_reduce(t)
            losses.append(float(t) / 2)
        released = all(u.released and u.grad_released for u in model.units if not u.is_root)
        sd = model.full_state_dict()
        q.put((rank, losses, released, {k: v.float().cpu().numpy() for k, v in sd.items()} if rank == 0 else None))
    except Exception as e:  # pragma: no cover
        import traceback

        traceback.print_exc()
        q.put((rank, repr(e), None, None))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("reshard", [False, True])
def test_flat_fsdp_two_ranks_on_one_gpu(reshard):
    """FlatFSDP at world 2 on the GPU paths (HIP fused ops writing gradients
    into released / re-taken CUDA buffers, async gathers + prefetch,
    reduce-scatters, the fused AdamW over the shard with the global-norm
    all-reduce): two gloo ranks share the card; equal (bf16 tolerance) to
    one process accumulating both halves of the batch."""
    import torch.multiprocessing as mp

    from conftest import free_port
    from dlrover_wuqiong_amd.models.llama import LlamaDecoderLayer
    from dlrover_wuqiong_amd.optimizers.fused import FusedAdamW
    from dlrover_wuqiong_amd.parallel.flat_fsdp import FlatFSDP

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_two_rank_worker, args=(r, port, reshard, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted((q.get(timeout=180) for _ in ps), key=lambda r: r[0])
    for p in ps:
        p.join(timeout=60)
    errs = [r[1] for r in res if isinstance(r[1], str)]
    assert not errs, errs
    losses, released, params = res[0][1], res[0][2], res[0][3]
    assert released == reshard
    # reference: world 1, both halves accumulated, gradient scaled by 1/2
    m, cfg = _model()
    fs = FlatFSDP(m, wrap_cls=(LlamaDecoderLayer,))
    opt = FusedAdamW(fs.shard_flat, lr=1e-3, max_grad_norm=1.0)
    opt.grad_scale = 0.5
    g = torch.Generator().manual_seed(3)
    ref = []
    for _ in range(3):
        xs = torch.randint(0, cfg.vocab_size, (4, 129), generator=g).cuda().chunk(2)
        tot = 0.0
        for x in xs:
            loss = fs(x[:, :-1], x[:, 1:])
            loss.backward()
            tot += float(loss.detach())
        opt.step()
        opt.zero_grad()
        ref.append(tot / 2)
    assert losses == pytest.approx(ref, rel=2e-2)
    for n, p in m.named_parameters():
        torch.testing.assert_close(torch.from_numpy(params[n]), p.detach().float().cpu(), rtol=5e-2, atol=5e-3,
                                   msg=n)
