"""Communication performance check (--comm-perf-test) on CPU/gloo: the
collective sweep + pairwise link test workload on 4 ranks, the agent-side
summary (degraded-link detection), and dwamd-run running it before training
(parity: reference training.py:1092-1109 comm_perf_check,
node_check/utils.py:58-132 bm_allreduce / bm_allgather)."""

import json
import os
import subprocess
import sys

from conftest import free_port

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXAMPLE = os.path.join(REPO, "examples", "elastic_train.py")


def test_round_robin_covers_every_pair_once():
    from dlrover_wuqiong_amd.trainer.node_check import _round_robin

    for n in (2, 3, 4, 7, 8):
        seen = [tuple(sorted(p)) for r in _round_robin(n) for p in r]
        assert sorted(seen) == sorted((a, b) for a in range(n) for b in range(a + 1, n))
        for r in _round_robin(n):  # disjoint within a round
            flat = [x for p in r for x in p]
            assert len(flat) == len(set(flat))


def test_workload_reports_bandwidths_and_links(tmp_path):
    port = free_port()
    procs = []
    for r in range(4):
        env = dict(os.environ, LOCAL_RANK=str(r), RANK=str(r), WORLD_SIZE="4", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), PYTHONPATH=REPO)
        procs.append(subprocess.Popen([sys.executable, "-m", "dlrover_wuqiong_amd.trainer.node_check", "--comm-perf",
                                       "--out-dir", str(tmp_path), "--sizes-mb", "0.25,1", "--link-mb", "0.5"],
                                      env=env))
    assert all(p.wait(timeout=240) == 0 for p in procs)
    reps = [json.loads((tmp_path / f"{r}.json").read_text()) for r in range(4)]
    for rep in reps:
        assert rep["ok"] and rep["init_sec"] >= 0 and rep["elapsed"] > 0
        ops = {(c["op"], c["bytes"]) for c in rep["collectives"]}
        assert {o for o, _b in ops} == {"allreduce", "allgather", "reducescatter"} and len(ops) == 6
        for c in rep["collectives"]:
            factor = 1.5 if c["op"] == "allreduce" else 0.75  # 2(n-1)/n, (n-1)/n at n=4
            assert c["busbw_gbps"] == round(c["algbw_gbps"] * factor, 3) or abs(
                c["busbw_gbps"] - c["algbw_gbps"] * factor) < 2e-3
        assert sorted(int(p) for p in rep["links_gbps"]) == [x for x in range(4) if x != rep["rank"]]
        assert all(v > 0 for v in rep["links_gbps"].values())
    from dlrover_wuqiong_amd.elastic_agent.node_check import summarize_comm_perf

    s = summarize_comm_perf(reps, 0.6)
    assert s["ok"] and len(s["links"]) == 6 and s["allreduce_busbw_gbps"] > 0


def test_summary_flags_a_degraded_link():
    from dlrover_wuqiong_amd.elastic_agent.node_check import summarize_comm_perf

    reps = []
    for r in range(4):
        links = {str(p): 50.0 for p in range(4) if p != r}
        reps.append({"ok": True, "rank": r, "local_rank": r, "world": 4, "links_gbps": links,
                     "collectives": [{"op": "allreduce", "bytes": 1 << 20, "algbw_gbps": 10, "busbw_gbps": 15}]})
    reps[1]["links_gbps"]["3"] = 20.0  # one direction of the 1<->3 link degraded
    s = summarize_comm_perf(reps, 0.6)
    assert s["slow_links"] == [[1, 3]] and s["link_median_gbps"] == 50.0
    assert s["allreduce_busbw_gbps"] == 15


def test_dwamd_run_comm_perf_test_then_train(tmp_path):
    out = tmp_path / "out.jsonl"
    env = dict(os.environ, PYTHONPATH=REPO, DWAMD_COMM_PERF_ARGS="--sizes-mb 0.25 --link-mb 0.25")
    p = subprocess.run([sys.executable, "-m", "dlrover_wuqiong_amd.trainer.run", "--nnodes", "1", "--nproc-per-node",
                        "2", "--comm-perf-test", EXAMPLE, "--steps", "3", "--out", str(out), "--ckpt-dir",
                        str(tmp_path / "ck")], env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    log = p.stdout + p.stderr
    assert "comm perf check: ok" in log and "busbw" in log
    rep = json.load(open("/tmp/dlrover/network_check/comm_perf_n0.json"))
    assert rep["world"] == 2 and rep["links"] and rep["slow_node"] is False
