"""Multi-dimension parallel randomizer (reference randomizer_test.py): on 4
gloo ranks as tensor 2 x data 2, a stream requested "same across G" is
identical exactly for the ranks that differ only along G -- for torch ops
under fork() and for the (seed, offset) pairs of the counter-hash kernels."""

import os

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import free_port


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    from dlrover_wuqiong_amd.atorch import distributed as adist
    from dlrover_wuqiong_amd.parallel import randomizer as R

    try:
        adist.init_distributed("gloo")
        adist.create_parallel_group(([("tensor", 2), ("data", 2)], None))
        R.reset_randomizer()
        R.init_randomizer(1234)
        out = {}
        before = torch.get_rng_state()
        for key in [(), ("tensor",), ("data",), ("tensor", "data")]:
            with R.get_randomizer(*key).fork():
                out[key] = torch.rand(4).tolist()
            with R.get_randomizer(*key).fork():  # the stream advances
                out[key + ("next",)] = torch.rand(4).tolist()
            out[key + ("philox",)] = [R.get_randomizer(*key).philox(10), R.get_randomizer(*key).philox(10)]
        assert torch.equal(before, torch.get_rng_state())  # the default generator is untouched
        states = R.get_MDPRInstance().get_states()
        with R.get_randomizer("tensor").fork():
            a = torch.rand(3)
        R.get_MDPRInstance().set_states(states)
        with R.get_randomizer("tensor").fork():
            b = torch.rand(3)
        out["restored"] = torch.equal(a, b)
        q.put((rank, adist.parallel_rank("tensor"), adist.parallel_rank("data"), out))
    except Exception as e:  # pragma: no cover
        import traceback

        traceback.print_exc()
        q.put((rank, None, None, repr(e)))
    finally:
        adist.reset_distributed()


def test_four_rank_parallel_randomizer():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_worker, args=(r, 4, port, q)) for r in range(4)]
    for p in ps:
        p.start()
    res = sorted((q.get(timeout=120) for _ in ps), key=lambda x: x[0])
    for p in ps:
        p.join(timeout=60)
    assert all(isinstance(r[3], dict) for r in res), res
    by = {(t, d): o for _r, t, d, o in res}
    assert all(o["restored"] for o in by.values())
    for key, same_t, same_d in [((), False, False), (("tensor",), True, False), (("data",), False, True),
                                (("tensor", "data"), True, True)]:
        for k in (key, key + ("next",), key + ("philox",)):
            v = {td: by[td][k] for td in by}
            assert (v[(0, 0)] == v[(1, 0)]) == same_t, (k, v)
            assert (v[(0, 0)] == v[(0, 1)]) == same_d, (k, v)
            assert (v[(0, 0)] == v[(1, 1)]) == (same_t and same_d), (k, v)
        assert by[(0, 0)][key] != by[(0, 0)][key + ("next",)]
        (s1, o1), (s2, o2) = by[(0, 0)][key + ("philox",)]
        assert s1 == s2 and (o1, o2) == (0, 10)
    # different G never collide on one rank
    seeds = {by[(0, 0)][k + ("philox",)][0][0] for k in [(), ("tensor",), ("data",), ("tensor", "data")]}
    assert len(seeds) == 4


def test_rng_checkpoint_replays_forked_streams():
    """Dropout inside a forked randomizer stream / tracked state: the
    checkpointed recompute regenerates the forward's masks, so gradients
    equal the uncheckpointed ones (torch's checkpoint alone would draw new
    masks from the advanced streams)."""
    from dlrover_wuqiong_amd.parallel import randomizer as R

    R.reset_randomizer()
    R.init_randomizer(7, dims={"tensor": (2, 1), "data": (2, 0)})
    tr = R.get_cuda_rng_tracker()
    tr.reset()
    tr.add("model-parallel-rng", 99)
    lin = torch.nn.Linear(32, 32)

    def block(x):
        with R.get_randomizer("tensor").fork():
            x = torch.nn.functional.dropout(lin(x), 0.5)
        with tr.fork():
            x = torch.nn.functional.dropout(lin(x), 0.5)
        return x

    x = torch.randn(8, 32, requires_grad=True)
    s0 = R.get_MDPRInstance().get_states()
    t0 = tr.get_states()
    block(x).square().sum().backward()
    g_ref, gx_ref = lin.weight.grad.clone(), x.grad.clone()
    lin.weight.grad, x.grad = None, None
    R.get_MDPRInstance().set_states(s0)
    tr.set_states(t0)
    R.rng_checkpoint(block, x).square().sum().backward()
    assert torch.allclose(lin.weight.grad, g_ref) and torch.allclose(x.grad, gx_ref)
    R.reset_randomizer()
    tr.reset()
