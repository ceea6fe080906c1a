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
