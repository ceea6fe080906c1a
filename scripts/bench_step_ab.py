"""GPT2-1.5B training step A/B (1 GPU, B=8 x 1024, bf16, FusedAdamW with
clipping): one process per variant, K timed steps between device-wide syncs.

  python scripts/bench_step_ab.py --steps 10                     # overlap off / on
  python scripts/bench_step_ab.py --variant on --env DWAMD_NORM_BWD_PART_OFF=1
"""
import argparse
import json
import os
import subprocess
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _init_pg(kind):
    """A/B: a world-1 process group next to the training loop (none | nccl |
    nccl_lazy | nccl_destroy | gloo)."""
    if kind == "none":
        return
    import torch
    import torch.distributed as dist

    for k, v in dict(MASTER_ADDR="127.0.0.1", MASTER_PORT="29611", RANK="0", WORLD_SIZE="1").items():
        os.environ.setdefault(k, v)
    if kind == "gloo":
        dist.init_process_group("gloo")
        return
    dev = torch.device("cuda", 0)
    env0 = dict(os.environ)
    if kind == "nccl_lazy":
        dist.init_process_group("nccl")  # no communicator until a collective
        return
    dist.init_process_group("nccl", device_id=dev)
    t = torch.ones(1, device=dev)
    dist.all_reduce(t)
    torch.cuda.synchronize()
    changed = {k: (env0.get(k), v) for k, v in os.environ.items() if env0.get(k) != v}
    gone = [k for k in env0 if k not in os.environ]
    print(json.dumps({"env_changed_by_rccl_init": changed, "env_removed": gone}), flush=True)
    if kind == "nccl_destroy":
        dist.destroy_process_group()


def _flusher(dev, gb, dst_kind="pinned"):
    """A checkpoint-flush stand-in: D2H of ``gb`` GB on the flash-checkpoint
    copier's side stream, issued every other step.  dst_kind "pinned": torch
    pinned memory (hipHostMalloc); "shm": a /dev/shm file mapping registered
    with hipHostRegister and copied with the copier's own call (what a real
    flush writes)."""
    import ctypes
    import mmap

    import torch

    from dlrover_wuqiong_amd.flash_checkpoint.copier import PinnedRegistry, GpuCopier, _kern

    c = GpuCopier(dev)
    n = int(gb * 1e9) // 2
    src = torch.ones(n, dtype=torch.bfloat16, device=dev)
    s = c.side_stream
    if dst_kind == "shm":
        path = f"/dev/shm/dwamd_step_ab_{os.getpid()}"
        fd = os.open(path, os.O_CREAT | os.O_RDWR, 0o600)
        os.ftruncate(fd, 2 * n)
        mm = mmap.mmap(fd, 2 * n)
        os.close(fd)
        os.unlink(path)  # the mapping keeps the pages; nothing left behind
        addr = ctypes.addressof(ctypes.c_char.from_buffer(mm))
        reg = PinnedRegistry()
        assert reg.ensure(addr, 2 * n)
        segs = reg.split(addr, 2 * n)
        _flusher.keep = (mm, reg)

        def go():
            s.wait_stream(torch.cuda.current_stream(dev))
            sp = ctypes.c_void_p(s.cuda_stream)
            for a, cnt, pinned in segs:
                assert _kern().dw_memcpy_async(ctypes.c_void_p(a), ctypes.c_void_p(src.data_ptr() + (a - addr)), cnt,
                                               1 if pinned else 3, sp) == 0
        return go
    dst = torch.empty(n, dtype=torch.bfloat16, pin_memory=True)

    def go():
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            dst.copy_(src, non_blocking=True)
    return go


def run(variant, steps, model_name, pg="none", flush_gb=0.0, flusher_first=False, flush_dst="pinned",
        pg_late=False, sync_each=False):
    import torch

    from dlrover_wuqiong_amd.models.gpt2 import GPT2, GPT2Config
    from dlrover_wuqiong_amd.optimizers.fused import FusedAdamW
    from dlrover_wuqiong_amd.parallel.flat import FlatParams

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    flush = _flusher(dev, flush_gb, flush_dst) if flush_gb and flusher_first else None
    if not pg_late:
        _init_pg(pg)
    torch.manual_seed(0)
    cfg = GPT2Config.named(model_name)
    with torch.device(dev):
        model = GPT2(cfg)
    model.to(torch.bfloat16)
    flat = FlatParams(model, dtype=torch.bfloat16, device=dev, lazy_zero_grad=True)
    opt = FusedAdamW(flat, lr=1e-4, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1, max_grad_norm=1.0)
    if variant == "on":
        opt.overlap_with_forward(model)
    if pg_late:  # as in bench.py: the group after the model and optimizer exist
        _init_pg(pg)
    data = torch.randint(0, cfg.vocab_size, (8, 1025), device=dev)
    losses = []
    if flush is None and flush_gb:
        flush = _flusher(dev, flush_gb, flush_dst)
    it = [0]

    def step():
        it[0] += 1
        if flush is not None and it[0] % 2 == 0:
            flush()
        loss = model(data[:, :-1], data[:, 1:])
        loss.backward()
        opt.step()
        flat.zero_grad()
        losses.append(loss.detach())
        if sync_each:  # as bench.py: the host waits for the compute stream every step
            torch.cuda.current_stream().synchronize()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    import resource

    ru0 = resource.getrusage(resource.RUSAGE_SELF)
    c0 = time.thread_time()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    c1 = time.thread_time()  # main thread CPU time of issuing the steps
    torch.cuda.synchronize()
    ms = 1000 * (time.perf_counter() - t0) / steps
    ru1 = resource.getrusage(resource.RUSAGE_SELF)
    cpu_ms = 1000 * ((ru1.ru_utime - ru0.ru_utime) + (ru1.ru_stime - ru0.ru_stime)) / steps
    print(json.dumps({"variant": variant, "pg": pg, "flush_gb": flush_gb, "flusher_first": flusher_first, "flush_dst": flush_dst, "pg_late": pg_late, "sync_each": sync_each, "step_ms": round(ms, 2), "tok_s": round(8 * 1024 / ms * 1000),
                      "loss_last": round(float(losses[-1]), 4),
                      "main_thread_cpu_ms_per_step": round(1000 * (c1 - c0) / steps, 2),
                      "process_cpu_ms_per_step": round(cpu_ms, 2),
                      "env": {k: v for k, v in os.environ.items() if k.startswith(("DWAMD_", "TORCH_NCCL", "NCCL_",
                                                                                       "RCCL_", "HSA_", "GPU_", "HIP_"))}}), flush=True)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--model", default="gpt2-1.5b")
    p.add_argument("--variant", default="", help="off | on (one process); default: both")
    p.add_argument("--env", action="append", default=[], help="KEY=VAL for the child processes")
    p.add_argument("--pg", default="none", help="world-1 process group: none | nccl | nccl_lazy | nccl_destroy | gloo")
    p.add_argument("--flush-gb", type=float, default=0.0, help="D2H flush of this many GB every other step")
    p.add_argument("--flusher-first", action="store_true", help="create the flush stream before the process group")
    p.add_argument("--flush-dst", default="pinned", choices=["pinned", "shm"])
    p.add_argument("--pg-late", action="store_true", help="create the process group after the model / optimizer")
    p.add_argument("--sync-each", action="store_true", help="compute-stream synchronize after every step")
    a = p.parse_args()
    if a.variant:
        run(a.variant, a.steps, a.model, a.pg, a.flush_gb, a.flusher_first, a.flush_dst, a.pg_late, a.sync_each)
        return
    env = dict(os.environ)
    for kv in a.env:
        k, v = kv.split("=", 1)
        env[k] = v
    for v in ("off", "on"):
        rc = subprocess.call([sys.executable, __file__, "--steps", str(a.steps), "--model", a.model, "--variant", v],
                             env=env)
        if rc:
            sys.exit(rc)


if __name__ == "__main__":
    main()
