"""Master-driven node relaunch on the local-process platform: the master
launches 2 node agents, one node is killed (SIGKILL on the whole node),
the watcher reports it, the job manager relaunches a replacement with the
same rank, the surviving node re-rendezvouses and training finishes from the
in-memory checkpoint (parity: reference dist_job_manager / pod scaler
relaunch tests)."""

import json
import os
import threading
import time

from conftest import free_port

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXAMPLE = os.path.join(REPO, "examples", "elastic_train.py")


def _wait(pred, timeout):
    deadline = time.time() + timeout
    while time.time() < deadline:
        if pred():
            return True
        time.sleep(0.1)
    return False


def test_master_relaunches_killed_node(tmp_path, monkeypatch):
    from dlrover_wuqiong_amd.common.node import JobResource
    from dlrover_wuqiong_amd.master.master import DistributedJobMaster
    from dlrover_wuqiong_amd.master.scaler import ProcessScaler, kill_process_tree

    monkeypatch.setenv("PYTHONPATH", REPO + os.pathsep + os.environ.get("PYTHONPATH", ""))
    out, prog = tmp_path / "out.jsonl", tmp_path / "progress"
    entry = [EXAMPLE, "--steps", "40", "--out", str(out), "--ckpt-dir", str(tmp_path / "ck"),
             "--step-sleep", "0.15", "--progress", str(prog)]
    jr = JobResource()
    jr.update_node_group_resource("worker", 2)
    m = DistributedJobMaster(jr, lambda addr: ProcessScaler("plat", addr, entry, 1, "2", str(tmp_path / "logs"),
                                                            agent_args=["--rdzv-conf", "lastcall_timeout=1"]),
                             port=free_port(), loop_interval=0.5, max_relaunch_count=2)
    result = {}
    try:
        m.prepare()
        t = threading.Thread(target=lambda: result.setdefault("rc", m.run()), daemon=True)
        t.start()
        assert _wait(lambda: prog.exists() and int(prog.read_text() or 0) >= 8, 120), "training did not start"
        victim = next(n for n in m.job_manager.nodes.values() if n.rank_index == 1)
        kill_process_tree(m.scaler.procs[victim.id].pid)
        t.join(timeout=240)
        assert not t.is_alive(), "job did not finish"
    finally:
        m.stop()
    assert result.get("rc") == 0, open(tmp_path / "logs" / "worker-0.log").read()[-3000:]
    ranks1 = [n for n in m.job_manager.nodes.values() if n.rank_index == 1]
    assert len(ranks1) == 2 and ranks1[-1].relaunch_count == 1  # replaced once
    res = [json.loads(x) for x in out.read_text().splitlines() if x.strip()]
    assert res[-1]["world"] == 2 and res[-1]["start_step"] >= 8  # resumed, not from scratch
