"""Node health / network check workload (runs as the worker processes of a
network-check round or of the communication performance check).

Parity: reference ``dlrover/trainer/torch/node_check/nvidia_gpu.py:23-49`` and
``node_check/utils.py`` (matmul + all_reduce/all_gather timing, elapsed time
written to ``/tmp/dlrover/network_check/{local_rank}.txt``, ``MOCK_ERR_RANK``
fault injection, ``bm_allreduce`` / ``bm_allgather`` algorithm and bus
bandwidth :58-132).  MI355X version:

* the compute probe is a bf16 GEMM on the MFMA matrix cores (a dead CU / a
  throttled GPU shows up as a straggler);
* the health probe is a 64 MiB RCCL all-reduce over xGMI;
* only the probes are timed -- ``init_process_group`` (RCCL bootstrap,
  dominated by rendezvous jitter) is reported apart, so straggler detection
  compares GEMM and link speed, not bootstrap noise;
* ``--comm-perf``: all-reduce / all-gather / reduce-scatter sweeps over
  message sizes with algorithm and bus bandwidth (nccl-tests conventions),
  plus a pairwise link test -- every GPU pair of the node exchanges a buffer
  in both directions, n/2 disjoint pairs at a time (round-robin
  tournament).  xGMI is point-to-point (7 links per MI355X), so one degraded
  link shows up as one slow pair even when the ring collective's bandwidth
  only drops a little.
"""

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

from ..common.constants import ConfigPath, NodeEnv

GB = 1e9


def mock_error():
    r = os.getenv(NodeEnv.MOCK_ERR_RANK, "")
    if r != "" and int(r) == int(os.getenv("RANK", "-1")):
        raise RuntimeError(f"mock error on rank {r}")


def _sync(device):
    if device.type == "cuda":
        torch.cuda.synchronize(device)


def matmul_probe(device, n_iter=10) -> float:
    """Seconds for ``n_iter`` GEMMs (8192^3 bf16 on a GPU)."""
    if device.type == "cuda":
        a = torch.randn(8192, 8192, device=device, dtype=torch.bfloat16)
        b = torch.randn(8192, 8192, device=device, dtype=torch.bfloat16)
    else:
        a = torch.randn(256, 256)
        b = torch.randn(256, 256)
    for _ in range(2):
        torch.matmul(a, b)
    _sync(device)
    t = time.perf_counter()
    for _ in range(n_iter):
        torch.matmul(a, b)
    _sync(device)
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
    _sync(device)
    t = time.perf_counter()
    for _ in range(iters):
        one()
    _sync(device)
    return time.perf_counter() - t


def _time_per_iter(fn, device, warmup: int, iters: int) -> float:
    """Seconds per call: device events on a GPU (the reference's
    ``_execute_nccl_comm``), wall clock on the CPU."""
    for _ in range(warmup):
        fn()
    _sync(device)
    if device.type == "cuda":
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        e.synchronize()
        return s.elapsed_time(e) / 1000.0 / iters
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    return (time.perf_counter() - t) / iters


def collective_perf(device, sizes, warmup=5, iters=20):
    """Algorithm / bus bandwidth (GB/s, 1e9) per op and message size.

    nccl-tests conventions (``size`` = bytes of the largest buffer of the
    op): all-reduce busbw = algbw * 2(n-1)/n; all-gather and reduce-scatter
    busbw = algbw * (n-1)/n with size = the gathered / scattered total."""
    n = dist.get_world_size()
    out = []
    for nbytes in sizes:
        per = max(1, nbytes // (4 * n)) * n  # divisible by n (reduce-scatter / all-gather chunks)
        x = torch.ones(per, dtype=torch.float32, device=device)
        chunk = torch.empty(per // n, dtype=torch.float32, device=device)
        ops = {
            "allreduce": (lambda: dist.all_reduce(x), 2.0 * (n - 1) / n),
            "allgather": (lambda: dist.all_gather_into_tensor(x, chunk), (n - 1) / n),
            "reducescatter": (lambda: dist.reduce_scatter_tensor(chunk, x), (n - 1) / n),
        }
        for name, (fn, factor) in ops.items():
            sec = _time_per_iter(fn, device, warmup, iters)
            algbw = per * 4 / sec / GB
            out.append({"op": name, "bytes": per * 4, "us": round(sec * 1e6, 2), "algbw_gbps": round(algbw, 3),
                        "busbw_gbps": round(algbw * factor, 3)})
        del x, chunk
    return out


def _round_robin(n: int):
    """Rounds of disjoint pairs covering every pair once (circle method;
    with odd n one rank sits out each round)."""
    m = n + (n % 2)
    ids = list(range(m))
    rounds = []
    for _ in range(m - 1):
        pairs = [(ids[i], ids[m - 1 - i]) for i in range(m // 2)]
        rounds.append([(a, b) for a, b in pairs if a < n and b < n])
        ids = [ids[0]] + [ids[-1]] + ids[1:-1]
    return rounds


def link_perf(device, nbytes: int, warmup=2, iters=5):
    """Bidirectional exchange bandwidth of every pair of ranks: per round,
    n/2 disjoint pairs exchange ``nbytes`` each way at once.  Returns
    ``{peer: GB/s per direction}`` for this rank."""
    n, me = dist.get_world_size(), dist.get_rank()
    numel = max(1, nbytes // 4)
    send = torch.ones(numel, dtype=torch.float32, device=device)
    recv = torch.empty_like(send)
    res = {}
    for pairs in _round_robin(n):
        peer = next((b if a == me else a for a, b in pairs if me in (a, b)), None)
        dist.barrier()
        if peer is None:
            continue

        def xchg(peer=peer):
            ops = [dist.P2POp(dist.isend, send, peer), dist.P2POp(dist.irecv, recv, peer)]
            if me > peer:
                ops.reverse()
            for r in dist.batch_isend_irecv(ops):
                r.wait()

        sec = _time_per_iter(xchg, device, warmup, iters)
        res[peer] = round(numel * 4 / sec / GB, 3)
    dist.barrier()
    return res


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--comm-perf", action="store_true")
    p.add_argument("--out-dir", default=ConfigPath.NETWORK_CHECK_DATA_DIR)
    p.add_argument("--sizes-mb", default="", help="comm-perf message sizes (MiB, comma separated)")
    p.add_argument("--link-mb", type=float, default=0.0, help="pairwise link test buffer (MiB)")
    a = p.parse_args(argv)
    local_rank = int(os.getenv("LOCAL_RANK", "0"))
    cuda = torch.cuda.is_available()
    device = torch.device("cuda", local_rank) if cuda else torch.device("cpu")
    if cuda:
        torch.cuda.set_device(device)
    ok = True
    rep = {"local_rank": local_rank, "rank": int(os.getenv("RANK", "0")), "world": int(os.getenv("WORLD_SIZE", "1")),
           "device": str(device)}
    try:
        t_init = time.perf_counter()
        if rep["world"] > 1:
            dist.init_process_group("nccl" if cuda else "gloo",
                                    device_id=device if cuda else None)
            dist.barrier()  # every peer is up: the probes start together
        rep["init_sec"] = round(time.perf_counter() - t_init, 4)
        mock_error()
        t0 = time.perf_counter()
        mm = matmul_probe(device)
        cm = comm_probe(device)
        elapsed = time.perf_counter() - t0  # the probes only, not the RCCL bootstrap
        rep.update(matmul_sec=round(mm, 6), comm_sec=round(cm, 6), elapsed=round(elapsed, 6))
        if cuda:
            rep["matmul_tflops"] = round(10 * 2 * 8192 ** 3 / mm / 1e12, 1)
        if a.comm_perf and rep["world"] > 1:
            if a.sizes_mb:
                sizes = [int(float(x) * (1 << 20)) for x in a.sizes_mb.split(",") if x]
            else:
                sizes = [x << 20 for x in ((1, 16, 64, 256) if cuda else (1,))]
            rep["collectives"] = collective_perf(device, sizes, iters=20 if cuda else 3)
            link_bytes = int((a.link_mb or (256 if cuda else 1)) * (1 << 20))
            rep["links_gbps"] = link_perf(device, link_bytes, iters=5 if cuda else 2)
    except Exception as e:
        print(f"node check failed: {e}", file=sys.stderr)
        ok = False
        elapsed = 3600.0
        rep["error"] = str(e)
    rep["ok"] = ok
    os.makedirs(a.out_dir, exist_ok=True)
    with open(os.path.join(a.out_dir, f"{local_rank}.txt"), "w") as f:
        f.write(f"{elapsed:.6f}")
    with open(os.path.join(a.out_dir, f"{local_rank}.json"), "w") as f:
        json.dump(rep, f)
    if dist.is_initialized():
        dist.destroy_process_group()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
