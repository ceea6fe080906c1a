"""Does gloo run the tensor collectives FlatFSDP uses on CUDA tensors (two
ranks sharing one GPU)?"""
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def run(rank, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29681")
    dist.init_process_group("gloo", rank=rank, world_size=2)
    out = {}
    x = torch.full((4,), float(rank + 1), device="cuda")
    for name, fn in [("all_gather_into_tensor", lambda: dist.all_gather_into_tensor(torch.empty(8, device="cuda"), x)),
                     ("reduce_scatter_tensor", lambda: dist.reduce_scatter_tensor(torch.empty(2, device="cuda"), x)),
                     ("all_reduce", lambda: dist.all_reduce(x.clone())),
                     ("all_gather_into_tensor_async", lambda: dist.all_gather_into_tensor(
                         torch.empty(8, device="cuda"), x, async_op=True).wait())]:
        try:
            fn()
            torch.cuda.synchronize()
            out[name] = "ok"
        except Exception as e:
            out[name] = repr(e)[:120]
    q.put((rank, out))
    dist.destroy_process_group()


if __name__ == "__main__":
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=run, args=(r, q)) for r in range(2)]
    [p.start() for p in ps]
    print(sorted(q.get(timeout=120) for _ in ps))
    [p.join() for p in ps]
