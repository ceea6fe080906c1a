"""Tensor / sequence parallel layers vs. their single-device equivalents
(gloo, 2 ranks), vocab-parallel embedding + cross entropy, ATorch named
parallel groups (parity: ATorch tests/distributed_modules)."""

import os

import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn
import torch.nn.functional as F

from conftest import free_port


def test_pg_ranks_layout():
    from dlrover_wuqiong_amd.atorch.distributed import get_pg_ranks

    g = get_pg_ranks([("tensor", 4), ("pipeline", 2), ("data", 2)], list(range(16)))[0]
    assert g["tensor"][:2] == [[0, 1, 2, 3], [4, 5, 6, 7]]
    assert g["pipeline"][:2] == [[0, 4], [1, 5]]
    assert g["data"][:2] == [[0, 8], [1, 9]]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    try:
        from dlrover_wuqiong_amd.atorch import distributed as adist
        from dlrover_wuqiong_amd.parallel import tensor_parallel as tp

        adist.init_distributed("gloo")
        adist.create_parallel_group(([("tensor", world)], None))
        group = adist.parallel_group("tensor")
        assert adist.parallel_rank("tensor") == rank and adist.parallel_group_size("tensor") == world
        torch.manual_seed(0)
        fc1, fc2 = nn.Linear(16, 32), nn.Linear(32, 16)
        x = torch.randn(8, 4, 16, requires_grad=True)  # [S, B, H]
        ref = fc2(F.gelu(fc1(x)))
        ref.square().sum().backward()
        ok = True
        for sp in (False, True):
            c = tp.ColumnParallelLinear.from_linear(fc1, group, sequence_parallel=sp)
            r = tp.RowParallelLinear.from_linear(fc2, group, sequence_parallel=sp)
            xi = x.detach().clone().requires_grad_(True)
            inp = tp.scatter_to_sequence_parallel_region(xi, group) if sp else xi
            y = r(F.gelu(c(inp)))
            if sp:
                y = tp.gather_from_sequence_parallel_region(y, group, tensor_parallel_output_grad=False)
            y.square().sum().backward()
            per = 32 // world
            ok &= torch.allclose(y, ref, atol=1e-5)
            ok &= torch.allclose(xi.grad, x.grad, atol=1e-4)
            ok &= torch.allclose(c.weight.grad, fc1.weight.grad[rank * per:(rank + 1) * per], atol=1e-4)
            ok &= torch.allclose(r.weight.grad, fc2.weight.grad[:, rank * per:(rank + 1) * per], atol=1e-4)
            if sp:
                # row-parallel bias grad is partial under SP: reduce it
                tp.allreduce_sequence_parallel_grads(r, group)
            ok &= torch.allclose(r.bias.grad, fc2.bias.grad, atol=1e-4)
        # vocab-parallel embedding + cross entropy
        emb = nn.Embedding(50, 8)
        head = nn.Linear(8, 50, bias=False)
        ids = torch.randint(0, 50, (6, 5))
        tgt = torch.randint(0, 50, (6, 5))
        tgt[0, 0] = -100
        ref_logits = head(emb(ids))
        ref_loss = F.cross_entropy(ref_logits.view(-1, 50), tgt.view(-1), reduction="none", label_smoothing=0.1)
        ref_loss.sum().backward()
        vemb = tp.VocabParallelEmbedding.from_embedding(emb, group)
        vhead = tp.ColumnParallelLinear.from_linear(head, group)
        logits = vhead(vemb(ids))
        loss = tp.vocab_parallel_cross_entropy(logits, tgt, group, label_smoothing=0.1)
        ok &= torch.allclose(loss.view(-1), ref_loss, atol=1e-5)
        loss.sum().backward()
        per = 50 // world
        ok &= torch.allclose(vhead.weight.grad, head.weight.grad[rank * per:(rank + 1) * per], atol=1e-5)
        ok &= torch.allclose(vemb.weight.grad[:per], emb.weight.grad[rank * per:(rank + 1) * per], atol=1e-5)
        # Ulysses all-to-all round trip: [S/sp, B, H, D] -> [S, B, H/sp, D] -> back
        adist.create_sequence_parallel_group(world)
        t = torch.arange(2 * 3 * 4 * 2, dtype=torch.float32).view(2, 3, 4, 2) + 100 * rank
        a = adist.seq_all_to_all(t, scatter_idx=2, gather_idx=0)
        ok &= tuple(a.shape) == (2 * world, 3, 4 // world, 2)
        back = adist.seq_all_to_all(a, scatter_idx=0, gather_idx=2)
        ok &= torch.equal(back, t)
        q.put((rank, bool(ok)))
    except Exception as e:  # pragma: no cover
        import traceback

        traceback.print_exc()
        q.put((rank, repr(e)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_tensor_and_sequence_parallel_two_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=180) for _ in ps)
    for p in ps:
        p.join(timeout=30)
    assert res == [(0, True), (1, True)], res


def _overlap_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    try:
        from dlrover_wuqiong_amd.parallel import tensor_parallel as tp

        dist.init_process_group("gloo")
        group = dist.group.WORLD
        torch.manual_seed(1)
        fc = nn.Linear(16, 32)
        x = torch.randn(8, 4, 16)
        out = {}
        for sp in (False, True):
            grads = []
            for overlap in (False, True):
                c = tp.ColumnParallelLinear.from_linear(fc, group, sequence_parallel=sp)
                c.overlap_comm = overlap
                xi = (x.chunk(world, 0)[rank] if sp else x).clone().requires_grad_(True)
                y = c(xi)
                y.square().sum().backward()
                grads.append((y.detach(), xi.grad, c.weight.grad, c.bias.grad))
            out[sp] = all(torch.allclose(a, b, atol=1e-5) for a, b in zip(*grads))
        # order of events in the overlapped backward: the input-gradient
        # collective is issued BEFORE the weight-gradient GEMM and waited after
        log = []

        real_ar = dist.all_reduce

        def ar(t, *a, **k):
            log.append("all_reduce_async" if k.get("async_op") else "all_reduce")
            w = real_ar(t, *a, **k)
            if k.get("async_op"):
                class W:
                    def wait(self_):
                        log.append("wait")
                        return w.wait()
                return W()
            return w

        real_mm = torch.Tensor.matmul

        def mm(self_, other):
            log.append("matmul")
            return real_mm(self_, other)

        c = tp.ColumnParallelLinear.from_linear(fc, group)
        y = c(x.clone().requires_grad_(True))
        dist.all_reduce, torch.Tensor.matmul = ar, mm
        try:
            y.square().sum().backward()
        finally:
            dist.all_reduce, torch.Tensor.matmul = real_ar, real_mm
        q.put((rank, (out[False], out[True], log)))
    except Exception as e:  # pragma: no cover
        import traceback

        traceback.print_exc()
        q.put((rank, repr(e)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_column_parallel_comm_overlap_two_ranks():
    """The overlapped column-parallel Linear (ATorch
    LinearWithGradAccumulationAndAsyncCommunication) gives the gradients of
    the blocking form, with and without sequence parallelism, and issues
    the dX all-reduce before the dW GEMM, waiting only after it."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_overlap_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=180) for _ in ps)
    for p in ps:
        p.join(timeout=30)
    for _r, out in res:
        assert isinstance(out, tuple), res
        tp_ok, sp_ok, log = out
        assert tp_ok and sp_ok, out
        i = log.index("all_reduce_async")
        assert "matmul" in log[i + 1:log.index("wait")], log
