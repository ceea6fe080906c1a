"""Scale plans and node scalers.

Parity: reference ``master/scaler/base_scaler.py`` (``ScalePlan``,
``Scaler``), ``scaler/pod_scaler.py`` / ``elasticjob_scaler.py`` (K8s) and
``ray_scaler.py``.  Kubernetes / Ray clients are not part of this image, so
the concrete back-end here is ``ProcessScaler``: every node is a local
``dwamd-run`` agent process (own session, own shm namespace), which is how a
multi-node MI355X job is rehearsed on one host and how the node-relaunch
path is tested end to end.  A K8s scaler implements the same two calls
(``scale(plan)`` creating / deleting pods of the ElasticJob).
"""

import os
import signal
import subprocess
import sys
import threading
from abc import ABC, abstractmethod
from dataclasses import dataclass, field
from typing import Dict, List, Optional

from ..common.log import logger
from ..common.node import Node, NodeGroupResource


@dataclass
class ScalePlan:
    node_group_resources: Dict[str, NodeGroupResource] = field(default_factory=dict)
    launch_nodes: List[Node] = field(default_factory=list)
    remove_nodes: List[Node] = field(default_factory=list)
    ps_addrs: List[str] = field(default_factory=list)

    def empty(self) -> bool:
        return not (self.node_group_resources or self.launch_nodes or self.remove_nodes)

    def merge(self, other: "ScalePlan"):
        if other is None:
            return
        self.node_group_resources.update(other.node_group_resources)
        self.launch_nodes.extend(other.launch_nodes)
        self.remove_nodes.extend(other.remove_nodes)
        self.ps_addrs.extend(a for a in other.ps_addrs if a not in self.ps_addrs)


class Scaler(ABC):
    def __init__(self, job_name: str):
        self.job_name = job_name

    def start(self):
        pass

    @abstractmethod
    def scale(self, plan: ScalePlan):
        ...


class ProcessScaler(Scaler):
    """Nodes as local ``dwamd-run`` process groups.

    ``entry``: training script + args; ``nproc_per_node``; ``nnodes`` as
    ``min:max``.  Each node gets ``DWAMD_SHM_PREFIX=<job>n<rank>`` so nodes do
    not share checkpoint memory (a relaunched node of the same rank finds
    its predecessor's shm, like a pod restarted on the same host).
    """

    def __init__(self, job_name: str, master_addr: str, entry: List[str], nproc_per_node: int = 1,
                 nnodes: str = "1", log_dir: str = "", extra_env: Optional[Dict[str, str]] = None,
                 agent_args: Optional[List[str]] = None):
        super().__init__(job_name)
        self.master_addr = master_addr
        self.entry = list(entry)
        self.nproc_per_node = nproc_per_node
        self.nnodes = nnodes
        self.log_dir = log_dir
        self.extra_env = dict(extra_env or {})
        self.agent_args = list(agent_args or [])
        self.procs: Dict[int, subprocess.Popen] = {}  # node id -> agent process
        self.nodes: Dict[int, Node] = {}
        self._lock = threading.Lock()

    def _cmd(self, node: Node) -> List[str]:
        host, port = self.master_addr.rsplit(":", 1)
        return ([sys.executable, "-m", "dlrover_wuqiong_amd.trainer.run", "--nnodes", self.nnodes,
                 "--nproc-per-node", str(self.nproc_per_node), "--node-rank", str(node.rank_index),
                 "--master-addr", host, "--master-port", port, "--rdzv-id", self.job_name]
                + self.agent_args + self.entry)

    def launch(self, node: Node):
        env = dict(os.environ)
        env.update(self.extra_env)
        env["DWAMD_SHM_PREFIX"] = f"{env.get('DWAMD_SHM_PREFIX', '')}{self.job_name}n{node.rank_index}"
        env["NODE_ID"] = str(node.id)
        env["DLROVER_MASTER_ADDR"] = self.master_addr
        env["DWAMD_EXIT_ON_NODE_ERROR"] = "1"  # the platform replaces nodes with hardware faults
        out = None
        if self.log_dir:
            os.makedirs(self.log_dir, exist_ok=True)
            out = open(os.path.join(self.log_dir, f"{node.name}.log"), "w")
        p = subprocess.Popen(self._cmd(node), env=env, stdout=out, stderr=subprocess.STDOUT if out else None,
                             start_new_session=True)
        if out is not None:
            out.close()
        with self._lock:
            self.procs[node.id] = p
            self.nodes[node.id] = node
        logger.info(f"launched {node.name} (rank {node.rank_index}) as pid {p.pid}")

    def remove(self, node: Node):
        with self._lock:
            p = self.procs.get(node.id)
        if p is not None and p.poll() is None:
            kill_process_tree(p.pid)

    def scale(self, plan: ScalePlan):
        for n in plan.remove_nodes:
            self.remove(n)
        for n in plan.launch_nodes:
            self.launch(n)

    def stop_all(self):
        with self._lock:
            procs = list(self.procs.values())
        for p in procs:
            if p.poll() is None:
                kill_process_tree(p.pid)


def kill_process_tree(pid: int, sig=signal.SIGKILL):
    """Kill an agent and every process below it (workers live in their own
    sessions, so a process-group kill alone would orphan them)."""
    try:
        import psutil

        root = psutil.Process(pid)
        procs = root.children(recursive=True) + [root]
    except Exception:
        procs = []
    if not procs:
        try:
            os.killpg(pid, sig)
        except (ProcessLookupError, PermissionError):
            pass
        return
    for p in procs:
        try:
            p.send_signal(sig)
        except Exception:
            pass
