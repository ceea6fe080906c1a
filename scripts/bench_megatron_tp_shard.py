"""Flash-checkpoint pause / restore for ONE tensor-parallel rank of a
Megatron-LM model, in Megatron's checkpoint layout (BASELINE.json config
"Llama-3 70B Megatron-LM TP=8 checkpoint-format-compatible async save
(288 GB HBM sizing)").

The state is exactly what TP rank 0 of Llama-3 70B at TP=8 holds with the
non-distributed mixed-precision optimizer: Megatron-core parameter names and
per-rank shard shapes (QKV / FC1 column-split, proj / FC2 row-split,
vocab-split embedding and output layer), bf16 weights, and fp32 main
params + Adam exp_avg / exp_avg_sq per parameter -- ~8.8 B parameters,
~123 GB on the one GPU.  Between checkpoints the compute stream runs ~3 s of
bf16 GEMMs (stand-in for the training steps of one checkpoint interval: one
70B TP=8 step at 64K tokens is ~3.4 PFLOP per GPU) and nudges the state so
successive checkpoints differ.  The background flush of the previous
checkpoint (HBM staging -> pinned shared memory, ~2.2 s for 123 GB) runs
under that compute; a snapshot only waits for it when the interval is
shorter than the flush.

Measured: paused time of ``MegatronCheckpointer.save_checkpoint`` (memory
save; the agent-side persist to ``iter_XXXXXXX/mp_rank_00/model_optim_rng.pt``
is asynchronous) and the cold in-memory restore into the live GPU tensors,
verified by checksums.  Synthetic values; one rank of the TP group.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {
    "llama3-70b": dict(vocab=128256, hidden=8192, ffn=28672, layers=80, heads=64, kv_heads=8, head_dim=128),
    "llama3-8b": dict(vocab=128256, hidden=4096, ffn=14336, layers=32, heads=32, kv_heads=8, head_dim=128),
    "llama-tiny": dict(vocab=1024, hidden=256, ffn=688, layers=2, heads=8, kv_heads=8, head_dim=32),
    # the reference's Megatron-LM row (GPT-1.5B, BASELINE.md: 1.2 s save / 2.1 s load): learned positions,
    # LayerNorm / linear biases, plain GELU MLP, vocab padded to 50304
    "gpt2-1.5b": dict(vocab=50304, hidden=1600, ffn=6400, layers=48, heads=25, kv_heads=25, head_dim=64,
                      gated=False, bias=True, positions=1024),
}


def shard_param_shapes(m, tp):
    """Megatron-core GPTModel parameter names -> TP-rank shard shapes."""
    h, hd = m["hidden"], m["head_dim"]
    qkv = (m["heads"] + 2 * m["kv_heads"]) * hd // tp
    fc1 = (2 if m.get("gated", True) else 1) * m["ffn"] // tp
    bias = m.get("bias", False)
    out = {"embedding.word_embeddings.weight": (m["vocab"] // tp, h)}
    if m.get("positions"):
        out["embedding.position_embeddings.weight"] = (m["positions"], h)
    for i in range(m["layers"]):
        p = f"decoder.layers.{i}."
        out[p + "self_attention.linear_qkv.layer_norm_weight"] = (h,)
        if bias:
            out[p + "self_attention.linear_qkv.layer_norm_bias"] = (h,)
            out[p + "self_attention.linear_qkv.bias"] = (qkv,)
        out[p + "self_attention.linear_qkv.weight"] = (qkv, h)
        out[p + "self_attention.linear_proj.weight"] = (h, m["heads"] * hd // tp)
        if bias:
            out[p + "self_attention.linear_proj.bias"] = (h,)
        out[p + "mlp.linear_fc1.layer_norm_weight"] = (h,)
        if bias:
            out[p + "mlp.linear_fc1.layer_norm_bias"] = (h,)
            out[p + "mlp.linear_fc1.bias"] = (fc1,)
        out[p + "mlp.linear_fc1.weight"] = (fc1, h)
        out[p + "mlp.linear_fc2.weight"] = (h, m["ffn"] // tp)
        if bias:
            out[p + "mlp.linear_fc2.bias"] = (h,)
    out["decoder.final_layernorm.weight"] = (h,)
    if bias:
        out["decoder.final_layernorm.bias"] = (h,)
    out["output_layer.weight"] = (m["vocab"] // tp, h)
    return out


def build_state(shapes, device):
    model, main, exp_avg, exp_avg_sq = {}, [], {}, {}
    for i, (name, shp) in enumerate(shapes.items()):
        w = torch.empty(shp, dtype=torch.bfloat16, device=device).normal_(0, 0.02)
        model[name] = w
        main.append(w.float())
        exp_avg[i] = torch.empty(shp, dtype=torch.float32, device=device).normal_(0, 1e-3)
        exp_avg_sq[i] = torch.empty(shp, dtype=torch.float32, device=device).uniform_(0, 1e-6)
    optim = {
        "optimizer": {"state": {i: {"exp_avg": exp_avg[i], "exp_avg_sq": exp_avg_sq[i], "step": 0}
                                for i in exp_avg},
                      "param_groups": [{"lr": 1.5e-4, "betas": (0.9, 0.95), "eps": 1e-8, "weight_decay": 0.1,
                                        "params": list(exp_avg)}]},
        "fp32_from_fp16_params": [main],
    }
    return {"model": model, "optimizer": optim, "rng_state": [{"random_rng_state": 0}]}


def megatron_names_gpt2(n_layer: int):
    """This framework's GPT2 parameter names -> Megatron-core GPTModel names
    (same shapes at TP=1; tied embeddings = Megatron's default
    share_embeddings_and_output_weights, so no output_layer)."""
    out = {"wte.weight": "embedding.word_embeddings.weight", "wpe.weight": "embedding.position_embeddings.weight",
           "ln_f.weight": "decoder.final_layernorm.weight", "ln_f.bias": "decoder.final_layernorm.bias"}
    per = {"ln_1.weight": "self_attention.linear_qkv.layer_norm_weight",
           "ln_1.bias": "self_attention.linear_qkv.layer_norm_bias",
           "attn.c_attn.weight": "self_attention.linear_qkv.weight", "attn.c_attn.bias": "self_attention.linear_qkv.bias",
           "attn.c_proj.weight": "self_attention.linear_proj.weight", "attn.c_proj.bias": "self_attention.linear_proj.bias",
           "ln_2.weight": "mlp.linear_fc1.layer_norm_weight", "ln_2.bias": "mlp.linear_fc1.layer_norm_bias",
           "mlp.c_fc.weight": "mlp.linear_fc1.weight", "mlp.c_fc.bias": "mlp.linear_fc1.bias",
           "mlp.c_proj.weight": "mlp.linear_fc2.weight", "mlp.c_proj.bias": "mlp.linear_fc2.bias"}
    for i in range(n_layer):
        for k, v in per.items():
            out[f"h.{i}.{k}"] = f"decoder.layers.{i}.{v}"
    return out


def build_trained_gpt2(device, micro_batch: int, seq: int):
    """A real GPT2-1.5B training setup (bf16 params, fp32 masters + Adam in
    FusedAdamW's flat buffers) whose state dict in Megatron's layout is
    views into the live tensors: the saves checkpoint what training writes."""
    from dlrover_wuqiong_amd.models.gpt2 import GPT2, GPT2Config
    from dlrover_wuqiong_amd.optimizers.fused import FusedAdamW
    from dlrover_wuqiong_amd.parallel.flat import FlatParams

    cfg = GPT2Config.named("gpt2-1.5b")
    cfg.n_positions = max(cfg.n_positions, seq)
    torch.manual_seed(0)
    with torch.device(device):
        model = GPT2(cfg)
    model.to(torch.bfloat16)
    flat = FlatParams(model, dtype=torch.bfloat16, device=device)
    opt = FusedAdamW(flat, lr=1.5e-4, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1, max_grad_norm=1.0)
    names = megatron_names_gpt2(cfg.n_layer)
    pname = {id(p): n for n, p in model.named_parameters()}
    msd, main, exp_avg, exp_avg_sq = {}, [], {}, {}
    for i, (o, c) in enumerate(flat.offsets):
        p = flat.params[i]
        msd[names[pname[id(p)]]] = p.data
        main.append(opt.master[o:o + c].view(p.shape))
        exp_avg[i] = opt.exp_avg[o:o + c].view(p.shape)
        exp_avg_sq[i] = opt.exp_avg_sq[o:o + c].view(p.shape)
    g = opt.param_groups[0]
    optim = {"optimizer": {"state": {i: {"exp_avg": exp_avg[i], "exp_avg_sq": exp_avg_sq[i], "step": opt._step_t}
                                     for i in exp_avg},
                           "param_groups": [{"lr": g["lr"], "betas": g["betas"], "eps": g["eps"],
                                             "weight_decay": g["weight_decay"], "params": list(exp_avg)}]},
             "fp32_from_fp16_params": [main]}
    data = torch.randint(0, cfg.vocab_size, (2, micro_batch, seq + 1), device=device)

    def step(i):
        b = data[i % 2]
        loss = model(b[:, :-1], b[:, 1:])
        loss.backward()
        opt.step()
        flat.zero_grad()
        return loss

    return {"model": msd, "optimizer": optim, "rng_state": [{"random_rng_state": 0}]}, step, model.num_params()


def tensors(sd):
    if isinstance(sd, torch.Tensor):
        yield sd
    elif isinstance(sd, dict):
        for v in sd.values():
            yield from tensors(v)
    elif isinstance(sd, (list, tuple)):
        for v in sd:
            yield from tensors(v)


def checksum(sd):
    return float(sum(t.float().sum(dtype=torch.float64).item() for t in tensors(sd)))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--model", default="llama3-70b", choices=sorted(SHAPES))
    p.add_argument("--tp", type=int, default=8)
    p.add_argument("--saves", type=int, default=3)
    p.add_argument("--work-gemms", type=int, default=4000, help="bf16 8192^3 GEMMs between saves (~3.3 s)")
    p.add_argument("--train-steps", type=int, default=0,
                   help="gpt2-1.5b at TP=1: REAL training steps (B=8 x 1024) between saves instead of stand-in "
                        "GEMMs; the Megatron-layout state is views into the live model / optimizer")
    p.add_argument("--ckpt-dir", default="/tmp/dwamd_megatron_ckpt")
    args = p.parse_args()
    os.environ.setdefault("LOCAL_WORLD_SIZE", "1")
    os.environ.setdefault("DWAMD_SHM_PREFIX", f"mtp{os.getpid()}")
    from dlrover_wuqiong_amd.common.constants import CheckpointConstant
    from dlrover_wuqiong_amd.flash_checkpoint.checkpointer import StorageType
    from dlrover_wuqiong_amd.flash_checkpoint.megatron import MegatronCheckpointer, get_checkpoint_name

    cuda = torch.cuda.is_available()
    device = torch.device("cuda", 0) if cuda else torch.device("cpu")
    if cuda:
        torch.cuda.set_device(device)
        torch.cuda.set_stream(torch.cuda.Stream(device))
    m = SHAPES[args.model]
    shapes = shard_param_shapes(m, args.tp)
    nparams = sum(int(torch.Size(s).numel()) for s in shapes.values())
    t0 = time.perf_counter()
    real = args.train_steps > 0
    if real:
        assert args.model == "gpt2-1.5b" and args.tp == 1 and cuda, "real training: gpt2-1.5b, TP=1, on a GPU"
        sd, train_step, nparams = build_trained_gpt2(device, 8, 1024)
    else:
        sd = build_state(shapes, device)
    nbytes = sum(t.numel() * t.element_size() for t in tensors(sd))
    print(f"{args.model} TP={args.tp} rank-0 shard: {nparams / 1e9:.2f} B params, {len(shapes)} tensors, "
          f"{nbytes / 1e9:.1f} GB state, built in {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)

    n = 8192 if cuda else 256
    a = torch.randn(n, n, dtype=torch.bfloat16 if cuda else torch.float32, device=device)
    bmat = torch.randn_like(a)

    step_times = []
    n_trained = [0]

    def work():
        if real:
            for _ in range(args.train_steps):
                ts = time.perf_counter()
                train_step(n_trained[0])
                torch.cuda.current_stream().synchronize()
                step_times.append(time.perf_counter() - ts)
                n_trained[0] += 1
            return
        for _ in range(args.work_gemms):
            torch.mm(a, bmat)
        for t in list(tensors(sd["model"]))[:8]:  # the step changes the state
            t.add_(1e-3)

    ckpt = MegatronCheckpointer(args.ckpt_dir)
    it = 0

    def save():
        nonlocal it
        it += 1
        ts = time.perf_counter()
        ok = ckpt.save_checkpoint(it, sd, storage_type=StorageType.MEMORY)
        if cuda:
            torch.cuda.current_stream().synchronize()
        return time.perf_counter() - ts, ok

    # once per job: the first save creates and registers the shared-memory
    # segment, the second is the first write of the second in-memory slot
    setup, flush_s = [], 0.0
    for _ in range(2):
        setup.append(save()[0])
        tf = time.perf_counter()
        ckpt.wait_latest_checkpoint()
        flush_s = time.perf_counter() - tf
    print(f"setup saves {[round(x, 2) for x in setup]} s, flush {flush_s:.2f} s", file=sys.stderr, flush=True)
    pauses, work_s = [], []
    for _ in range(args.saves):
        tw = time.perf_counter()
        work()
        if cuda:
            torch.cuda.current_stream().synchronize()
        work_s.append(time.perf_counter() - tw)
        pause, ok = save()
        assert ok, "memory save refused"
        pauses.append(pause)
        print(f"save {it}: pause {pause * 1e3:.1f} ms after {work_s[-1]:.2f} s of compute", file=sys.stderr,
              flush=True)
    ckpt.wait_latest_checkpoint()
    if cuda:
        torch.cuda.synchronize()
    ref = checksum(sd)
    for t in tensors(sd):
        t.zero_()
    copier = getattr(ckpt.engine, "_copier", None)
    if copier is not None:
        copier.pinned.release_all()  # a restarted process has nothing pinned: cold restore
    if cuda:
        torch.cuda.synchronize()
    tl = time.perf_counter()
    target = {CheckpointConstant.MODEL_STATES_NAME: dict(sd, iteration=it, checkpoint_version=3.0)}
    step, _restored = ckpt.load_checkpoint(target=target)
    if cuda:
        torch.cuda.synchronize()
    load_s = time.perf_counter() - tl
    got = checksum(sd)
    verified = step == it and abs(got - ref) <= 1e-9 * max(1.0, abs(ref))
    ckpt.close()
    print(json.dumps({
        "metric": "megatron tp-shard flash ckpt pause s", "value": round(sum(pauses) / len(pauses), 4), "unit": "s",
        "higher_is_better": False, "dtype": "bf16 params + fp32 main/Adam",
        "data": ("synthetic tokens, random-init weights, trained between saves" if real else "synthetic values"),
        "train_step_ms": round(1000 * sorted(step_times)[len(step_times) // 2], 1) if step_times else None,
        "config": {"model": f"{args.model} (Megatron-core names)", "parallelism": f"tp{args.tp}: rank 0's shard "
                   "on one GPU", "layout": os.path.relpath(get_checkpoint_name(args.ckpt_dir, it), args.ckpt_dir)},
        "params": nparams, "ckpt_bytes": nbytes, "save_sec": [round(x, 4) for x in pauses],
        "save_sec_max": round(max(pauses), 4), "load_sec": round(load_s, 3), "load_step": step,
        "load_verified": bool(verified), "compute_between_saves_s": round(sum(work_s) / len(work_s), 2),
        "setup_saves_s": [round(x, 2) for x in setup], "flush_s": round(flush_s, 2),
        "shm_slots": 2}))


if __name__ == "__main__":
    main()
