"""Ray platform against an in-process stand-in for the ``ray`` package (ray
is not installed here): actors run the node command as a child process, the
watcher turns exits / dead actors into node events.  Parity unpinned against
a real Ray cluster."""

import sys
import time
import types

import pytest


class _Ref:
    def __init__(self, fn):
        self.fn = fn


class _Handle:
    def __init__(self, obj):
        self._obj, self.dead = obj, False

    def __getattr__(self, name):
        meth = getattr(self._obj, name)
        handle = self

        class _M:
            @staticmethod
            def remote(*a, **kw):
                def run():
                    if handle.dead:
                        raise RuntimeError("actor died")
                    return meth(*a, **kw)
                return _Ref(run)
        return _M


def _fake_ray():
    ray = types.ModuleType("ray")
    ray.resources = []

    def remote(**opts):
        def deco(cls):
            class _Cls:
                @staticmethod
                def remote(*a, **kw):
                    ray.resources.append(opts)
                    return _Handle(cls(*a, **kw))
            return _Cls
        return deco

    def get(ref, timeout=None):
        return ref.fn()

    def kill(handle):
        handle._obj.stop()
        handle.dead = True

    ray.remote, ray.get, ray.kill = remote, get, kill
    return ray


@pytest.fixture()
def fake_ray(monkeypatch):
    ray = _fake_ray()
    monkeypatch.setitem(sys.modules, "ray", ray)
    return ray


def test_ray_scaler_and_watcher(fake_ray, monkeypatch):
    from dlrover_wuqiong_amd.common.constants import NodeExitReason, NodeStatus
    from dlrover_wuqiong_amd.common.node import Node
    from dlrover_wuqiong_amd.master.scaler import ScalePlan
    from dlrover_wuqiong_amd.platform.ray import RayScaler, RayWatcher

    sc = RayScaler("job", "10.0.0.1:5000", ["train.py", "--x"], gpus_per_node=8)
    cmd = sc._cmd(Node(id=3, rank_index=2))
    assert cmd[1:3] == ["-m", "dlrover_wuqiong_amd.trainer.run"] and "--node-rank" in cmd and cmd[-2:] == [
        "train.py", "--x"]
    assert cmd[cmd.index("--master-port") + 1] == "5000"
    codes = {0: "import sys; sys.exit(0)", 1: "import sys; sys.exit(3)", 2: "import time; time.sleep(30)"}
    monkeypatch.setattr(RayScaler, "_cmd", lambda self, node: [sys.executable, "-c", codes[node.id]])
    sc.scale(ScalePlan(launch_nodes=[Node(id=i, rank_index=i) for i in range(3)]))
    assert fake_ray.resources == [{"num_gpus": 8}] * 3
    w = RayWatcher(sc)
    deadline = time.time() + 20
    while time.time() < deadline:
        st = {n.id: n.status for n in w.list()}
        if st[0] != NodeStatus.RUNNING and st[1] != NodeStatus.RUNNING:
            break
        time.sleep(0.1)
    nodes = {n.id: n for n in w.list()}
    assert nodes[0].status == NodeStatus.SUCCEEDED and nodes[1].status == NodeStatus.FAILED
    assert nodes[1].exit_reason == NodeExitReason.FATAL_ERROR and nodes[2].status == NodeStatus.RUNNING
    evs = list(w.watch())
    assert len(evs) == 3 and not list(w.watch())  # only changes are reported
    # a dead actor (host lost) -> hardware error
    sc.actors[2].dead = True
    n2 = [n for n in w.list() if n.id == 2][0]
    assert n2.status == NodeStatus.FAILED and n2.exit_reason == NodeExitReason.HARDWARE_ERROR
    sc.scale(ScalePlan(remove_nodes=[Node(id=2)]))
    assert 2 not in sc.actors


def test_ray_missing_package_message(monkeypatch):
    monkeypatch.setitem(sys.modules, "ray", None)
    from dlrover_wuqiong_amd.platform.ray import RayScaler

    with pytest.raises(ImportError, match="'ray' package"):
        RayScaler("j", "h:1", ["t.py"])
