"""Ray platform: run every elastic-training node as a Ray actor.

``RayScaler`` (the master's ``Scaler``) starts one actor per node with the
requested GPUs; each actor launches the ``dwamd-run`` agent as a child
process on its host and reports its exit code.  ``RayWatcher`` polls the
actors and turns finished / dead ones into node events, so the job master's
relaunch logic is identical to the process and Kubernetes platforms.

``ray`` is not part of this image: importing this module works, creating a
``RayScaler`` raises an ImportError naming the missing dependency.

Parity: reference ``dlrover/python/scheduler/ray.py`` (RayClient /
actor-as-node), ``master/scaler/ray_scaler.py``, ``master/watcher/ray_watcher.py``
and ``client/platform/ray/ray_job_submitter.py``.
"""

import subprocess
import sys
from typing import Dict, Iterator, List, Optional

from ..common.constants import NodeEventType, NodeExitReason, NodeStatus
from ..common.log import logger
from ..common.node import Node
from ..master.scaler import ScalePlan, Scaler
from ..master.watcher import NodeEvent, NodeWatcher


def _ray():
    try:
        import ray  # noqa: F401
    except ImportError as e:
        raise ImportError("the Ray platform needs the 'ray' package, which is not installed") from e
    return ray


class _NodeRunner:
    """Body of the per-node actor: runs the agent command, returns its code."""

    def __init__(self, cmd: List[str], env: Dict[str, str]):
        import os

        self.proc = subprocess.Popen(cmd, env={**os.environ, **env})

    def poll(self) -> Optional[int]:
        return self.proc.poll()

    def stop(self):
        if self.proc.poll() is None:
            self.proc.terminate()


class RayScaler(Scaler):
    def __init__(self, job_name: str, master_addr: str, entry: List[str], gpus_per_node: int = 8,
                 agent_args: Optional[List[str]] = None):
        super().__init__(job_name)
        ray = _ray()
        self.master_addr, self.entry, self.gpus = master_addr, entry, gpus_per_node
        self.agent_args = agent_args or []
        self.actor_cls = ray.remote(num_gpus=gpus_per_node)(_NodeRunner)
        self.actors: Dict[int, object] = {}
        self.nodes: Dict[int, Node] = {}

    def _cmd(self, node: Node) -> List[str]:
        return [sys.executable, "-m", "dlrover_wuqiong_amd.trainer.run", "--nproc-per-node", str(self.gpus),
                "--node-rank", str(node.rank_index), "--master-addr", self.master_addr.rsplit(":", 1)[0],
                "--master-port", self.master_addr.rsplit(":", 1)[1], *self.agent_args, *self.entry]

    def scale(self, plan: ScalePlan):
        for node in plan.launch_nodes:
            env = {"NODE_ID": str(node.id), "DWAMD_JOB_NAME": self.job_name, "HSA_ENABLE_IPC_MODE_LEGACY": "0"}
            logger.info(f"ray: starting actor for node {node.id} (rank {node.rank_index})")
            self.actors[node.id] = self.actor_cls.remote(self._cmd(node), env)
            self.nodes[node.id] = node
        for node in plan.remove_nodes:
            a = self.actors.pop(node.id, None)
            if a is not None:
                _ray().kill(a)


class RayWatcher(NodeWatcher):
    def __init__(self, scaler: RayScaler):
        self.scaler = scaler
        self._reported: Dict[int, str] = {}

    def list(self) -> List[Node]:
        ray = _ray()
        out = []
        for nid, actor in list(self.scaler.actors.items()):
            node = self.scaler.nodes[nid]
            try:
                code = ray.get(actor.poll.remote(), timeout=10)
            except Exception:  # actor / host died
                node.status, node.exit_reason = NodeStatus.FAILED, NodeExitReason.HARDWARE_ERROR
                out.append(node)
                continue
            if code is None:
                node.status = NodeStatus.RUNNING
            else:
                node.status = NodeStatus.SUCCEEDED if code == 0 else NodeStatus.FAILED
                node.exit_reason = NodeExitReason.SUCCEEDED if code == 0 else NodeExitReason.FATAL_ERROR
            out.append(node)
        return out

    def watch(self) -> Iterator[NodeEvent]:
        for node in self.list():
            if self._reported.get(node.id) != node.status:
                self._reported[node.id] = node.status
                yield NodeEvent(NodeEventType.MODIFIED, node)
