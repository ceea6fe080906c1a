"""Acceleration engine: executor task flow, planner / SG algorithms, the
gRPC service, and a 2-rank gloo ``auto_accelerate(load_strategy="engine")``
end to end (reference test model: atorch/atorch/tests/auto_engine_test/ and
auto_accelerate tests)."""

import os
import threading

import torch
import torch.multiprocessing as mp
import torch.nn.functional as F

from conftest import free_port
from dlrover_wuqiong_amd.atorch.engine import (AccelerationEngine, EngineClient, Executor, StrategyStatus,
                                               TaskType)
from dlrover_wuqiong_amd.atorch.engine.task import decode, encode


def _analysis(params=1_000_000, world=2):
    return {"params": params, "trainable_params": params, "module_types": {"LayerNorm": 2},
            "block_classes": ["Block"], "has_module_for_replace": True, "tp_able": True, "num_heads": 4,
            "state_bytes": {"ddp": 18 * params, "zero1": int((6 + 12 / world) * params),
                            "zero2": int((2 + 16 / world) * params), "fsdp": int(18 / world * params)}}


def _fake_throughput(strategy):
    names = {x[0] for x in strategy}
    t = 100.0
    t += 50 if "amp_native" in names else 0
    t += 20 if "fsdp" in names else 0
    t -= 30 if "checkpoint" in names else 0
    t += 5 if "module_replace" in names else 0
    return t


def _drive(ex, world, analysis, fail=lambda s: False, max_rounds=5000):
    """Simulated processes polling the executor round-robin."""
    runs = {p: [] for p in range(world)}
    done = {}
    inflight = {}
    for _ in range(max_rounds):
        for p in range(world):
            if p in done:
                continue
            if p in inflight:
                t = inflight.pop(p)
                if t.task_type == TaskType.ANALYSE:
                    ex.report_task_result(t.task_id, p, True, analysis)
                elif t.task_type == TaskType.SETUP_PARALLEL_GROUP:
                    ex.report_task_result(t.task_id, p, True, None)
                elif t.task_type == TaskType.TUNE:
                    s = [(n, ([("tensor", 2), ("data", world // 2)], None) if n == "parallel_mode" else c, False)
                         for n, c, _ in t.info]
                    ex.report_task_result(t.task_id, p, True, s)
                elif t.task_type == TaskType.DRYRUN:
                    ok = not fail(t.info)
                    ex.report_task_result(t.task_id, p, ok, {"throughput": _fake_throughput(t.info)} if ok else None)
                continue
            t = ex.get_task(p)
            if t.task_type in (TaskType.FINISH, TaskType.FAIL):
                done[p] = t
                continue
            if t.task_type != TaskType.WAIT:
                runs[p].append(t.task_type)
                inflight[p] = t
        if len(done) == world:
            return done, runs
    raise AssertionError("executor did not finish")


def test_task_wire_roundtrip():
    s = [("parallel_mode", ([("data", 2)], None), False), ("amp_native", {"dtype": torch.bfloat16}, False)]
    back = decode(encode(s))
    assert back[0][1] == ([("data", 2)], None) and back[1][1]["dtype"] is torch.bfloat16


def test_executor_combination_picks_fastest():
    ctx = {"node_num": 1, "nproc_per_node": 2, "total_gpu": 2, "gpu_arch": "gfx950:sramecc+:xnack-"}
    ex = Executor(ctx, excluded_opts=["tensor_parallel", "zero1", "zero2"])
    done, runs = _drive(ex, 2, _analysis())
    fin = done[0]
    assert fin.task_type == TaskType.FINISH and done[1].info == fin.info
    names = {x[0] for x in fin.info}
    assert {"amp_native", "fsdp", "module_replace"} <= names and "checkpoint" not in names
    # ALL_PROCESS dry runs ran on both processes; the analysis ran once
    assert runs[0].count("DRYRUN") == runs[1].count("DRYRUN") > 1
    assert runs[0].count("ANALYSE") + runs[1].count("ANALYSE") == 1
    # one parallel mode for every candidate -> its group is set up once
    assert runs[0].count("SETUP_PARALLEL_GROUP") == 1
    assert all(i.status == StrategyStatus.SUCCEED for i in ex.strategies.infos.values())
    assert ex.can_be_terminated


def test_executor_prunes_by_memory_and_device():
    # 30B params: neither DDP nor ZeRO-1/2 state fits one 288 GB GPU at world 2
    ctx = {"node_num": 1, "nproc_per_node": 2, "total_gpu": 2, "gpu_arch": "gfx942"}
    ex = Executor(ctx, excluded_opts=["tensor_parallel"])
    assert not ex.lib.enabled("module_replace")  # gfx950 kernels only
    done, _ = _drive(ex, 2, _analysis(params=30_000_000_000))
    for info in ex.strategies.infos.values():
        assert "fsdp" in {x[0] for x in info.strategy}
    assert ex.strategies.baseline_id is None
    assert "fsdp" in {x[0] for x in done[0].info}


def test_executor_tensor_parallel_tune_and_failures():
    ctx = {"node_num": 1, "nproc_per_node": 2, "total_gpu": 2, "gpu_arch": "gfx950"}
    ex = Executor(ctx, included_opts=["tensor_parallel", "amp_native"])
    # every TP strategy's dry run fails (e.g. OOM): the search still finishes
    done, runs = _drive(ex, 2, _analysis(), fail=lambda s: any(x[0] == "tensor_parallel" for x in s))
    assert "TUNE" in runs[0] + runs[1]
    tp = [i for i in ex.strategies.infos.values() if any(x[0] == "tensor_parallel" for x in i.strategy)]
    assert tp and all(i.status == StrategyStatus.FAILED for i in tp)
    assert all(i.strategy[0][1] == ([("tensor", 2), ("data", 1)], None) for i in tp)
    assert [x[0] for x in done[0].info] == ["parallel_mode", "amp_native"]


def test_executor_all_fail_gives_fail_task():
    ex = Executor({"node_num": 1, "nproc_per_node": 1}, included_opts=["amp_native"])
    done, _ = _drive(ex, 1, _analysis(world=1), fail=lambda s: True)
    assert done[0].task_type == TaskType.FAIL


def test_executor_bayes_opt_large_space(monkeypatch):
    monkeypatch.setenv("DWAMD_ENGINE_MAX_EXHAUSTIVE", "2")
    monkeypatch.setenv("DWAMD_BO_MAX_ITER", "6")
    ctx = {"node_num": 1, "nproc_per_node": 4, "total_gpu": 4, "gpu_arch": "gfx950"}
    ex = Executor(ctx, excluded_opts=["tensor_parallel"])
    assert ex.planner.max_exhaustive == 2
    done, _ = _drive(ex, 4, _analysis(world=4))
    assert ex.algos == ["bo_sg"]
    n = len(ex.strategies)
    assert 2 <= n <= 1 + 6  # baseline + at most max_iter proposals
    best = max(_fake_throughput(i.strategy) for i in ex.strategies.infos.values())
    assert _fake_throughput(done[0].info) == best


def test_load_strategy_is_dry_run_then_finished():
    ex = Executor({"node_num": 1, "nproc_per_node": 2}, load_strategy=[("amp_native", None, False)])
    done, runs = _drive(ex, 2, _analysis())
    assert [x[0] for x in done[0].info] == ["amp_native"] and "ANALYSE" not in runs[0] + runs[1]


def test_engine_service_over_grpc():
    eng = AccelerationEngine({"node_num": 1, "nproc_per_node": 2}, included_opts=["amp_native"])
    port = eng.start_service(0)
    out = {}

    def proc(p):
        c = EngineClient("127.0.0.1", port, process_id=p)
        while True:
            t = c.get_task()
            if t.task_type in (TaskType.FINISH, TaskType.FAIL):
                out[p] = t
                break
            if t.task_type == TaskType.WAIT:
                continue
            res = _analysis() if t.task_type == TaskType.ANALYSE else \
                {"throughput": _fake_throughput(t.info)} if t.task_type == TaskType.DRYRUN else None
            c.report_task_result(t, True, res)
        c.close()

    th = [threading.Thread(target=proc, args=(p,)) for p in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(60)
    eng.tear_down(timeout=5)
    assert out[0].task_type == TaskType.FINISH and out[0].info == out[1].info
    assert out[0].info[1][0] == "amp_native" and out[0].info[1][1]["dtype"] is torch.bfloat16


# ------------------------------------------------------------ end to end
def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world), DWAMD_DRYRUN_WARMUP="1",
                      DWAMD_DRYRUN_STEPS="1")
    try:
        from test_auto_accelerate import DS, Toy, _train

        from dlrover_wuqiong_amd.atorch import distributed as adist
        from dlrover_wuqiong_amd.atorch.auto_accelerate import auto_accelerate

        class KwToy(Toy):
            def forward(self, ids, labels=None):
                return super().forward(ids)

        def loss(batch, out):
            return F.cross_entropy(out.reshape(-1, 64).float(), batch["labels"].reshape(-1))

        adist.init_distributed("gloo")
        torch.manual_seed(0)
        ok, res, strat = auto_accelerate(KwToy(), torch.optim.AdamW, dataset=DS(), loss_func=loss,
                                         optim_args={"lr": 1e-2}, dataloader_args={"batch_size": 8},
                                         model_input_format="unpack_dict", load_strategy="engine",
                                         included=["amp_native", "fsdp"])
        losses = _train(res, 8)
        q.put((rank, bool(ok and min(losses[-3:]) < losses[0]), strat.names()))
    except Exception as e:  # pragma: no cover
        import traceback

        traceback.print_exc()
        q.put((rank, repr(e), None))
    finally:
        adist.reset_distributed()


def test_two_rank_auto_accelerate_engine():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted((q.get(timeout=300) for _ in ps), key=lambda x: x[0])
    for p in ps:
        p.join(timeout=30)
    assert all(r[1] is True for r in res), res
    assert res[0][2] == res[1][2] and "parallel_mode" in res[0][2]


def test_reference_import_paths():
    from atorch.auto.engine.acceleration_engine import AccelerationEngine as A
    from atorch.auto.engine_client import EngineClient as C

    assert A is AccelerationEngine and C is EngineClient
