"""Llama-3 8B (or GPT2-1.5B: ``--model gpt2-1.5b --seq 1024``) through ``auto_accelerate`` (fused-op module replacement, bf16
autocast, FSDP2 per decoder layer, activation checkpointing) with
``FsdpShardCheckpointer`` flash checkpoints (BASELINE.json config "Llama-3 8B
FSDP + ATorch auto_accelerate fused ops, async ckpt").

One process per GPU; launch with torch.distributed.run for N GPUs (on one GPU
FSDP holds the whole model: fp32 parameters + AdamW states, ~96 GB).  Random
weights, synthetic tokens.  Reports the step time, the memory-save pause
(DTensor shards + optimizer state -> HBM snapshot, async flush to shared
memory), and the in-place restore time, verified against the saved shards.
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--model", default="llama3-8b")
    p.add_argument("--seq", type=int, default=4096)
    p.add_argument("--micro-batch", type=int, default=1)
    p.add_argument("--steps", type=int, default=8)
    p.add_argument("--ckpt-interval", type=int, default=4)
    p.add_argument("--ckpt-dir", default="/tmp/dwamd_fsdp_ckpt")
    p.add_argument("--precision", choices=["amp", "half"], default="half",
                   help="amp: fp32 sharded params, FSDP2 casts to bf16 per gather; half: bf16 params + fp32 "
                        "masters inside the fused optimizer")
    p.add_argument("--act-ckpt", choices=["on", "off"], default="off",
                   help="activation checkpointing of the decoder layers (off: a 288 GB MI355X holds every "
                        "activation of Llama-3-8B at S=4096, so the forward is not recomputed)")
    p.add_argument("--reshard", choices=["on", "off"], default="off",
                   help="off: FSDP2 reshard_after_forward=False (auto_accelerate 'zero2'): the gathered bf16 "
                        "parameters stay resident from forward to backward (16 GB for 8B on a 288 GB card), "
                        "no second all-gather per layer")
    p.add_argument("--torch-optim", action="store_true", help="keep torch.optim.AdamW (no multi-tensor HIP kernel)")
    p.add_argument("--optim-in-backward", action="store_true",
                   help="each FSDP unit's AdamW update from its post-backward reduce-scatter on a side stream "
                        "(optimizers/in_backward.py)")
    p.add_argument("--no-ckpt", action="store_true", help="step time only (no flash checkpoints)")
    p.add_argument("--meta", action="store_true",
                   help="build the model on the meta device (with --flat: each rank materialises only its shard)")
    p.add_argument("--flat", action="store_true",
                   help="flat-unit FSDP (auto_accelerate flat_zero2 / flat_fsdp, parallel/flat_fsdp.py: in-place "
                        "collectives, fused optimizer over the rank shard) + flat-shard flash checkpoints")
    p.add_argument("--fp8", action="store_true", help="auto_accelerate 'fp8' on the decoder layers' projections")
    p.add_argument("--storage", action="store_true",
                   help="also persist and time the storage restore (fast O_DIRECT reader vs stock dist_cp.load)")
    a = p.parse_args()
    for k, v in dict(MASTER_ADDR="127.0.0.1", MASTER_PORT="29571", RANK="0", WORLD_SIZE="1", LOCAL_RANK="0",
                     LOCAL_WORLD_SIZE="1").items():
        os.environ.setdefault(k, v)
    os.environ.setdefault("DWAMD_SHM_PREFIX", f"fsdp{os.environ['MASTER_PORT']}")
    lr = int(os.environ["LOCAL_RANK"])
    cuda = torch.cuda.is_available()
    dev = torch.device("cuda", lr) if cuda else torch.device("cpu")
    if cuda:
        torch.cuda.set_device(lr)
        dist.init_process_group("nccl", device_id=dev)
    else:  # CPU rehearsal of the same flow (gloo)
        dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()

    from dlrover_wuqiong_amd.atorch.auto_accelerate import auto_accelerate
    from dlrover_wuqiong_amd.flash_checkpoint.checkpointer import StorageType
    from dlrover_wuqiong_amd.flash_checkpoint.fsdp import FsdpShardCheckpointer
    torch.manual_seed(0)
    if a.model.startswith("gpt2"):
        # the reference's FSDP row (GPT2-1.5B, BASELINE.md: 2.9 s save / 15.1 s load)
        from dlrover_wuqiong_amd.models.gpt2 import GPT2, Block, GPT2Config

        cfg = GPT2Config.named(a.model)
        cfg.n_positions = max(cfg.n_positions, a.seq)
        with torch.device(dev):
            model = GPT2(cfg)
        layer_cls = Block
    else:
        from dlrover_wuqiong_amd.models.llama import Llama, LlamaConfig, LlamaDecoderLayer

        cfg = LlamaConfig.named(a.model)
        t_build = time.perf_counter()
        with torch.device("meta" if a.meta else dev):
            model = Llama(cfg)
        layer_cls = LlamaDecoderLayer
    prec = ("amp_native", {"dtype": torch.bfloat16}) if a.precision == "amp" else "half"
    if a.flat and (a.precision != "half" or a.optim_in_backward or a.torch_optim):
        raise SystemExit("--flat: bf16 parameters (--precision half) and the fused flat optimizer only")
    shard = ("flat_fsdp" if a.reshard == "on" else "flat_zero2") if a.flat else (
        "fsdp" if a.reshard == "on" else "zero2")
    scfg = {"wrap_cls": (layer_cls,)} if a.flat else {"wrap_cls": (layer_cls,), "optim_in_backward": a.optim_in_backward}
    ok, res, strategy = auto_accelerate(
        model, torch.optim.AdamW, optim_args={"lr": 2e-5, "betas": (0.9, 0.95), "weight_decay": 0.1},
        load_strategy=["module_replace", prec] + ([("fp8", {"include": ("layers", "h.")})] if a.fp8 else []) + [
                       (shard, scfg)]
        + ([("checkpoint", {"wrap_cls": (layer_cls,)})] if a.act_ckpt == "on" else []),
        fused_optimizer=not a.torch_optim)
    assert ok, "auto_accelerate failed"
    model, opt = res.model, res.optim
    if cuda:
        torch.cuda.synchronize()
    build_s = time.perf_counter() - t_build if not a.model.startswith("gpt2") else None
    build_peak_gb = round(torch.cuda.max_memory_allocated() / 2**30, 1) if cuda else None
    g = torch.Generator().manual_seed(rank)
    data = torch.randint(0, cfg.vocab_size, (2, a.micro_batch, a.seq + 1), generator=g).to(dev)
    ck = None if a.flat else FsdpShardCheckpointer(a.ckpt_dir)

    def sync():
        # the training stream only: a device-wide synchronize would also wait
        # for the async D2H flush on the copier's side stream, which the
        # training loop never waits for
        if cuda:
            torch.cuda.current_stream().synchronize()

    def step(i):
        b = data[i % 2]
        loss = model(b[:, :-1], b[:, 1:])  # bf16 compute via FSDP2's MixedPrecisionPolicy
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
        return loss

    for i in range(2):  # warm-up (+ the optimizer states get created)
        step(i)
        print(f"warm-up step {i} done", file=sys.stderr, flush=True)
    sync()
    if a.no_ckpt:
        steps, losses = [], []
        for i in range(a.steps):
            t0 = time.perf_counter()
            losses.append(float(step(i).item()))
            sync()
            steps.append(time.perf_counter() - t0)
        med = sorted(steps)[len(steps) // 2]
        if rank == 0:
            print(json.dumps({"metric": "fsdp train step", "n_gpus": world, "model": a.model, "seq_len": a.seq,
                              "precision": a.precision + ("+fp8" if a.fp8 else ""), "optimizer": type(opt).__name__,
                              "optim_in_backward": getattr(opt, "_in_backward", None) is not None,
                              "act_ckpt": a.act_ckpt, "reshard_after_forward": a.reshard == "on",
                              "fsdp": "flat" if a.flat else "fsdp2", "meta_init": a.meta,
                              "build_s": round(build_s, 2) if build_s else None, "build_peak_gb": build_peak_gb,
                              "train_step_ms": round(1000 * med, 1),
                              "tokens_per_s": round(world * a.micro_batch * a.seq / med, 1),
                              "peak_mem_gb": round(torch.cuda.max_memory_allocated() / 2**30, 1) if cuda else None,
                              "step_ms": [round(1000 * x, 1) for x in steps], "losses": [round(x, 3) for x in losses]}))
        dist.destroy_process_group()
        return
    if a.flat:
        _flat_ckpt_run(a, model, opt, step, sync, rank, world, cuda, strategy)
        dist.destroy_process_group()
        return
    ts = time.perf_counter()
    ck.prepare(model, opt)  # one-time shm set-up (both slots pinned) in the background
    ck.save_checkpoint(0, model, opt, storage_type=StorageType.MEMORY)  # untimed
    sync()
    setup_s = time.perf_counter() - ts
    ck.wait_latest_checkpoint()
    if ck.engine._shm_prep is not None:
        ck.engine._shm_prep.result()  # steady state: a long job finishes this during its first steps
    setup_s = time.perf_counter() - ts
    print(f"setup save {setup_s:.2f} s", file=sys.stderr, flush=True)
    pauses, steps, losses, landed = [], [], [], []
    for i in range(a.steps):
        t0 = time.perf_counter()
        losses.append(float(step(i).item()))
        sync()
        steps.append(time.perf_counter() - t0)
        if i % a.ckpt_interval == 0:
            prof = None
            if os.environ.get("DWAMD_PROFILE_SAVE") == "1" and rank == 0:
                import cProfile

                prof = cProfile.Profile()
                prof.enable()
            t0 = time.perf_counter()
            ok = ck.save_checkpoint(i + 1, model, opt, storage_type=StorageType.MEMORY)
            sync()
            pauses.append(time.perf_counter() - t0)
            landed.append(bool(ok))
            if prof is not None:
                import pstats

                prof.disable()
                pstats.Stats(prof, stream=sys.stderr).sort_stats("cumulative").print_stats(30)
    last = a.steps
    ck.wait_latest_checkpoint()  # the final save must not be skipped as busy
    ck.save_checkpoint(last + 1, model, opt, storage_type=StorageType.MEMORY)  # final state, untimed
    ck.wait_latest_checkpoint()
    if cuda:
        torch.cuda.synchronize()
    want = {k: v.to_local().clone() for k, v in model.state_dict().items()}
    with torch.no_grad():
        for v in model.state_dict().values():
            v.to_local().zero_()
    copier = getattr(ck.engine, "_copier", None)
    if copier is not None:
        copier.pinned.release_all()
    sync()
    t0 = time.perf_counter()
    extra = ck.load_checkpoint(model, opt)
    if cuda:
        torch.cuda.synchronize()  # restore is complete only when every stream is
    load_s = time.perf_counter() - t0
    verified = extra.get("step") == last + 1 and all(
        torch.equal(v.to_local(), want[k]) for k, v in model.state_dict().items())
    nbytes = ck.engine._shm_handler.payload_size if ck.engine._shm_handler.shared_memory else 0
    storage = {}
    if a.storage:
        # node replaced: the persisted DCP checkpoint read back (page cache
        # dropped) -- this framework's O_DIRECT range reader into the live
        # shards vs torch's stock dist_cp.load (FileSystemReader)
        import glob as _glob

        from dlrover_wuqiong_amd.flash_checkpoint.fsdp import _set_model_optim_state, wait_for_persist
        from dlrover_wuqiong_amd.flash_checkpoint.storage_loader import drop_file_cache

        sstep = last + 2
        ck.save_checkpoint(sstep, model, opt, storage_type=StorageType.DISK)
        if rank == 0:
            wait_for_persist(a.ckpt_dir, sstep, timeout=600)
        dist.barrier()
        want = {k: v.to_local().clone() for k, v in model.state_dict().items()}
        path = os.path.join(a.ckpt_dir, str(sstep))
        for mode in ("fast", "dcp"):
            os.environ["DWAMD_FAST_STORAGE_LOAD"] = "1" if mode == "fast" else "0"
            with torch.no_grad():
                for v in model.state_dict().values():
                    v.to_local().zero_()
            for f in _glob.glob(os.path.join(path, "*.distcp")):
                drop_file_cache(f)
            sync()
            t0 = time.perf_counter()
            sd = ck._state(model, opt, None)
            got = ck.engine._load_from_storage_dcp(sd, path)
            _set_model_optim_state(model, opt, sd.pop("model"), sd.pop("optim", None), full=False)
            sync()
            sec = time.perf_counter() - t0
            ok = got == sstep and all(torch.equal(v.to_local(), want[k]) for k, v in model.state_dict().items())
            storage[mode] = {"sec": round(sec, 3), "verified": bool(ok),
                             "source": ck.engine.last_restore_source,
                             "stats": ck.engine.last_storage_load_stats}
        os.environ["DWAMD_FAST_STORAGE_LOAD"] = "1"
    if rank == 0:
        print(json.dumps({
            "metric": "fsdp flash ckpt pause s", "unit": "s",
            # saves skipped as busy (previous flush still running) are not pauses
            "value": round(sum(p for p, ok in zip(pauses, landed) if ok) / max(1, sum(landed)), 4),
            "higher_is_better": False, "n_gpus": world, "dtype": ("bf16 autocast, fp32 params" if a.precision == "amp" else "bf16 params, fp32 masters"),
            "optimizer": type(opt).__name__,
            "data": "synthetic tokens, random-init weights",
            "config": {"model": a.model, "seq_len": a.seq, "micro_batch": a.micro_batch,
                       "strategy": str(strategy)[:300]},
            "save_sec": [round(x, 4) for x in pauses], "setup_save_s": round(setup_s, 2),
            "saves_landed": landed, "pause_landed_mean_s": round(
                sum(p for p, ok in zip(pauses, landed) if ok) / max(1, sum(landed)), 4),
            "flush_gbps": round(sum(n for n, _ in ck.engine._copier.flush_stats) / max(1e-9, sum(
                t for _, t in ck.engine._copier.flush_stats)) / 1e9, 1) if getattr(ck.engine, "_copier", None) else None,
            "load_sec": round(load_s, 3), "load_verified": bool(verified), "ckpt_bytes_per_rank": nbytes,
            "load_sec_storage": storage.get("fast", {}).get("sec"),
            "load_sec_storage_stock_dcp": storage.get("dcp", {}).get("sec"), "storage_restores": storage,
            "reference_fsdp_gpt2_1.5b_ssd_read_s": 18.0,
            "train_step_ms": round(1000 * sorted(steps)[len(steps) // 2], 1),
            "tokens_per_s": round(world * a.micro_batch * a.seq / sorted(steps)[len(steps) // 2], 1),
            "losses": [round(x, 3) for x in losses]}))
    ck.close()
    dist.destroy_process_group()


def _flat_ckpt_run(a, model, opt, step, sync, rank, world, cuda, strategy):
    """Flash checkpoints of a FlatFSDP model in the flat-shard format
    (atorch/fsdp_flat_ckpt.py): the live shard + fused-optimizer state
    buffers are the state, restored in place from memory."""
    from dlrover_wuqiong_amd.atorch import fsdp_flat_ckpt as ffc
    from dlrover_wuqiong_amd.flash_checkpoint.checkpointer import StorageType

    eng = ffc._engine(a.ckpt_dir)

    def save(i):
        return ffc.save_checkpoint(i, model, opt, os.path.join(a.ckpt_dir, f"step-{i}"),
                                   storage_type=StorageType.MEMORY)

    ts = time.perf_counter()
    save(0)  # untimed: shm set-up
    sync()
    eng.wait_for_memory_save()
    setup_s = time.perf_counter() - ts
    pauses, steps, losses, landed = [], [], [], []
    for i in range(a.steps):
        t0 = time.perf_counter()
        losses.append(float(step(i).item()))
        sync()
        steps.append(time.perf_counter() - t0)
        if i % a.ckpt_interval == 0:
            t0 = time.perf_counter()
            ok = save(i + 1)
            sync()
            pauses.append(time.perf_counter() - t0)
            landed.append(bool(ok))
    last = a.steps + 1
    eng.wait_for_memory_save()
    save(last)
    eng.wait_for_memory_save()
    if cuda:
        torch.cuda.synchronize()
    live = (model.shard_flat.data, opt.exp_avg, opt.exp_avg_sq) + ((opt.master,) if opt.master is not None else ())

    def fingerprint(t):  # bit-exact sum of the raw words: no full-size clone next to a 100+ GB state
        w = t.view(torch.int16 if t.element_size() == 2 else torch.int32)
        return int(torch.sum(w, dtype=torch.int64)), int(torch.sum(w[1::7], dtype=torch.int64))

    want = [fingerprint(t) for t in live]
    with torch.no_grad():
        for t in live:
            t.zero_()
    sync()
    t0 = time.perf_counter()
    got = ffc.load_checkpoint(model, opt, os.path.join(a.ckpt_dir, f"step-{last}"))
    if cuda:
        torch.cuda.synchronize()
    load_s = time.perf_counter() - t0
    verified = got == last and [fingerprint(t) for t in live] == want
    med = sorted(steps)[len(steps) // 2]
    if rank == 0:
        ok_p = [p for p, ok in zip(pauses, landed) if ok]
        print(json.dumps({
            "metric": "fsdp flash ckpt pause s", "unit": "s", "value": round(sum(ok_p) / max(1, len(ok_p)), 4),
            "higher_is_better": False, "n_gpus": world, "dtype": "bf16 params, fp32 masters", "fsdp": "flat",
            "optimizer": type(opt).__name__, "data": "synthetic tokens, random-init weights",
            "config": {"model": a.model, "seq_len": a.seq, "micro_batch": a.micro_batch, "strategy": str(strategy)[:300]},
            "save_sec": [round(x, 4) for x in pauses], "setup_save_s": round(setup_s, 2), "saves_landed": landed,
            "load_sec": round(load_s, 3), "load_verified": bool(verified),
            "ckpt_bytes_per_rank": int(sum(t.numel() * t.element_size() for t in live)),
            "train_step_ms": round(1000 * med, 1), "tokens_per_s": round(world * a.micro_batch * a.seq / med, 1),
            "peak_mem_gb": round(torch.cuda.max_memory_allocated() / 2**30, 1) if cuda else None,
            "step_ms": [round(1000 * x, 1) for x in steps], "losses": [round(x, 3) for x in losses]}))
    ffc.close_engines()


if __name__ == "__main__":
    main()
