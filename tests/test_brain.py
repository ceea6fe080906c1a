"""Brain service (metrics store + resource optimisation) and GP Bayesian
optimisation.  Parity: reference dlrover/python/tests/test_hpsearch_bo.py
(Hartmann-6 BO loop improves on the cold-start candidates) and the Go
brain's optimizer tests (pkg/optimizer/implementation/optalgorithm/*_test.go)."""

import numpy as np


def _hartmann6(x):
    alpha = np.array([1.0, 1.2, 3.0, 3.2])
    A = np.array([[10, 3, 17, 3.5, 1.7, 8], [0.05, 10, 17, 0.1, 8, 14],
                  [3, 3.5, 1.7, 10, 17, 8], [17, 8, 0.05, 10, 0.1, 14]])
    P = 1e-4 * np.array([[1312, 1696, 5569, 124, 8283, 5886], [2329, 4135, 8307, 3736, 1004, 9991],
                         [2348, 1451, 3522, 2883, 3047, 6650], [4047, 8828, 8732, 5743, 1091, 381]])
    x = np.asarray(x)
    return -float(-(alpha * np.exp(-(A * (x - P) ** 2).sum(1))).sum())  # maximise -H


def test_bayesian_optimizer_improves_on_hartmann6():
    from dlrover_wuqiong_amd.brain.hpsearch import BayesianOptimizer

    bounds = [[0.0, 1.0]] * 6
    history = []
    rng = np.random.default_rng(0)
    cold = BayesianOptimizer(bounds, history, 3, seed=0).optimize()
    assert len(cold) == 3 and len(cold[0].parameters) == 6
    for c in cold:
        c.reward = _hartmann6(c.parameters)
    history.append(cold)
    best = [max(c.reward for c in cold)]
    for it in range(8):
        cands = BayesianOptimizer(bounds, history, 3, use_variance=bool(it % 2), seed=it).optimize()
        for c in cands:
            assert all(0.0 <= v <= 1.0 for v in c.parameters)
            c.reward = _hartmann6(c.parameters) + 0.01 * rng.standard_normal()
            c.variance = 1e-4
        history.append(cands)
        best.append(max(best[-1], max(c.reward for c in cands)))
    assert best[-1] > best[0] + 0.3, best  # optimum is 3.32


def test_brain_service_plans():
    from dlrover_wuqiong_amd.brain.client import BrainClient, BrainResourceOptimizer
    from dlrover_wuqiong_amd.brain.service import BrainService
    from dlrover_wuqiong_amd.common.node import JobResource

    svc = BrainService(0).start()
    try:
        addr = f"127.0.0.1:{svc.port}"
        old = BrainClient(addr, job_uuid="job-1", job_name="llama-pretrain")
        for cpu_used, mem in ((10.0, 30000), (12.0, 40000), (11.0, 38000)):
            assert old.report_resource_usage("worker", "w0", 32, cpu_used, 65536, mem)
        new = BrainClient(addr, job_uuid="job-2", job_name="llama-pretrain")
        assert new.available()
        plan = new.request_optimization("job_create_resource")
        assert plan["worker"]["memory_mb"] == 48000 and plan["worker"]["cpu"] == 14.4
        assert len(new.get_job_metrics(job_uuid="job-1")) == 3
        # OOM: memory x1.5
        new.report_oom("worker", 40000)
        jr = JobResource()
        jr.update_node_group_resource("worker", count=4, cpu=8, memory=40000)
        bro = BrainResourceOptimizer(new, jr, max_workers=16, node_unit=2)
        p = bro.get_oom_resource_plan()
        assert p.node_group_resources["worker"].node_resource.memory == 60000
        # speed curve: near-linear to 8 workers, flat beyond
        for n, s in ((2, 100.0), (4, 198.0), (8, 390.0), (12, 400.0)):
            new.report_speed(n, s)
        p = bro.get_job_resource_plan()
        assert p.node_group_resources["worker"].count == 8
        # initial plan via the optimizer (history from job-1)
        p = bro.init_job_resource()
        assert p.node_group_resources["worker"].node_resource.memory == 48000
        # hot PS
        new.report_resource_usage("ps", "ps-0", 8, 7.5, 16000, 8000)
        new.report_resource_usage("ps", "ps-1", 8, 2.0, 16000, 8000)
        hp = new.request_optimization("job_hot_ps")
        assert hp == {"ps_nodes": {"ps-0": {"cpu": 12.0}}}
    finally:
        svc.stop()
