"""Worker-environment policies of the elastic agent (CPU)."""

from dlrover_wuqiong_amd.elastic_agent.agent import _hw_queues


def test_hw_queues_kept_by_default_raised_on_request(monkeypatch):
    monkeypatch.delenv("DWAMD_GPU_MAX_HW_QUEUES", raising=False)
    env = {"GPU_MAX_HW_QUEUES": "4"}
    _hw_queues(env)
    assert env["GPU_MAX_HW_QUEUES"] == "4"
    env = {}
    _hw_queues(env)
    assert "GPU_MAX_HW_QUEUES" not in env
    monkeypatch.setenv("DWAMD_GPU_MAX_HW_QUEUES", "0")
    env = {"GPU_MAX_HW_QUEUES": "4"}
    _hw_queues(env)
    assert env["GPU_MAX_HW_QUEUES"] == "4"
    monkeypatch.setenv("DWAMD_GPU_MAX_HW_QUEUES", "8")
    env = {"GPU_MAX_HW_QUEUES": "4"}
    _hw_queues(env)
    assert env["GPU_MAX_HW_QUEUES"] == "8"


def test_hw_queues_never_lowered_and_capped(monkeypatch):
    monkeypatch.setenv("DWAMD_GPU_MAX_HW_QUEUES", "8")
    env = {"GPU_MAX_HW_QUEUES": "16"}
    _hw_queues(env)
    assert env["GPU_MAX_HW_QUEUES"] == "16"
    monkeypatch.setenv("DWAMD_GPU_MAX_HW_QUEUES", "64")
    env = {"GPU_MAX_HW_QUEUES": "4"}
    _hw_queues(env)
    assert env["GPU_MAX_HW_QUEUES"] == "32"
    monkeypatch.setenv("DWAMD_GPU_MAX_HW_QUEUES", "0")  # off: the inherited value stays
    env = {"GPU_MAX_HW_QUEUES": "4"}
    _hw_queues(env)
    assert env["GPU_MAX_HW_QUEUES"] == "4"


def test_exit_watcher_wakes_on_a_killed_worker(monkeypatch):
    """A SIGKILLed worker wakes the agent's main loop within a few ms (the
    watcher reads /proc, it never reaps: the process stays a zombie until the
    main loop's poll)."""
    import signal
    import subprocess
    import threading
    import time
    from types import SimpleNamespace

    from dlrover_wuqiong_amd.elastic_agent.agent import ElasticTrainingAgent

    monkeypatch.setenv("DWAMD_EXIT_POLL_S", "0.002")
    p = subprocess.Popen(["sleep", "30"])
    fake = SimpleNamespace(workers=[SimpleNamespace(proc=p)], _stop_hb=threading.Event(), _exit_evt=threading.Event())
    t = threading.Thread(target=ElasticTrainingAgent._exit_watch_loop, args=(fake,), daemon=True)
    t.start()
    try:
        time.sleep(0.05)
        assert not fake._exit_evt.is_set()  # healthy worker: no wake-up
        t0 = time.perf_counter()
        p.send_signal(signal.SIGKILL)
        assert fake._exit_evt.wait(2.0)
        assert time.perf_counter() - t0 < 0.5
        assert p.returncode is None  # not reaped by the watcher
        fake._exit_evt.clear()
        time.sleep(0.02)
        assert not fake._exit_evt.is_set()  # one wake-up per failed process
    finally:
        fake._stop_hb.set()
        p.kill()
        p.wait()
        t.join(timeout=2)
