"""Node health / network check workload (runs as the worker processes of a
network-check round).

Parity: reference ``dlrover/trainer/torch/node_check/nvidia_gpu.py:23-49`` and
``node_check/utils.py`` (matmul + all_reduce/all_gather timing, elapsed time
written to ``/tmp/dlrover/network_check/{local_rank}.txt``, ``MOCK_ERR_RANK``
fault injection).  MI355X version: the compute probe is a bf16 GEMM that
runs on the MFMA matrix cores (a dead CU / throttled GPU shows up as a
straggler), the comm probe is a 64 MiB RCCL all-reduce over xGMI.
"""

import argparse
import os
import sys
import time

import torch
import torch.distributed as dist

from ..common.constants import ConfigPath, NodeEnv


def mock_error():
    r = os.getenv(NodeEnv.MOCK_ERR_RANK, "")
    if r != "" and int(r) == int(os.getenv("RANK", "-1")):
        raise RuntimeError(f"mock error on rank {r}")


def matmul_probe(device, n_iter=10) -> float:
    if device.type == "cuda":
        a = torch.randn(8192, 8192, device=device, dtype=torch.bfloat16)
        b = torch.randn(8192, 8192, device=device, dtype=torch.bfloat16)
    else:
        a = torch.randn(256, 256)
        b = torch.randn(256, 256)
    for _ in range(2):
        torch.matmul(a, b)
    if device.type == "cuda":
        torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n_iter):
        torch.matmul(a, b)
    if device.type == "cuda":
        torch.cuda.synchronize()
    return time.perf_counter() - t


def comm_probe(device, numel=1 << 24, warmup=5, iters=20, op="allreduce") -> float:
    if not dist.is_initialized() or dist.get_world_size() < 2:
        return 0.0
    x = torch.ones(numel if device.type == "cuda" else 1 << 16, dtype=torch.float32, device=device)
    outs = None
    if op == "allgather":
        outs = [torch.empty_like(x) for _ in range(dist.get_world_size())]

    def one():
        if op == "allgather":
            dist.all_gather(outs, x)
        else:
            dist.all_reduce(x)

    for _ in range(warmup):
        one()
    if device.type == "cuda":
        torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        one()
    if device.type == "cuda":
        torch.cuda.synchronize()
    return time.perf_counter() - t


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--comm-perf", action="store_true")
    p.add_argument("--out-dir", default=ConfigPath.NETWORK_CHECK_DATA_DIR)
    a = p.parse_args(argv)
    local_rank = int(os.getenv("LOCAL_RANK", "0"))
    cuda = torch.cuda.is_available()
    device = torch.device("cuda", local_rank) if cuda else torch.device("cpu")
    if cuda:
        torch.cuda.set_device(device)
    t0 = time.perf_counter()
    ok = True
    try:
        if int(os.getenv("WORLD_SIZE", "1")) > 1:
            dist.init_process_group("nccl" if cuda else "gloo")
        mock_error()
        mm = matmul_probe(device)
        cm = comm_probe(device)
        elapsed = time.perf_counter() - t0
    except Exception as e:
        print(f"node check failed: {e}", file=sys.stderr)
        ok = False
        elapsed = 3600.0
    os.makedirs(a.out_dir, exist_ok=True)
    with open(os.path.join(a.out_dir, f"{local_rank}.txt"), "w") as f:
        f.write(f"{elapsed:.6f}")
    if dist.is_initialized():
        dist.destroy_process_group()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
