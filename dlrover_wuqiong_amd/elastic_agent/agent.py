"""Per-node elastic training agent (runs inside ``dwamd-run``).

Responsibilities (parity: reference
``dlrover/python/elastic_agent/torch/training.py``: ``ElasticLaunchConfig``
:116-168, ``MasterRendezvousHandler`` :179-359, ``ElasticTrainingAgent``
:362-731, ``launch_agent`` :734-822, node check :864-1112):

* rendezvous through the job master (join, poll the completed world),
  global rank assignment (offset = sum of local world sizes of lower node
  ranks), MASTER_ADDR/PORT published by node 0 through the master KV store;
* spawn one process per GPU (plain ``subprocess``; this process never touches
  the GPU, so no fork/exec of a GPU-initialised process ever happens); a
  warm standby interpreter per local rank (``standby.py``) is kept ready so a
  restart skips interpreter start + ``import torch``;
* monitor loop: success -> exit barrier; failure -> report to master, persist
  the latest in-memory flash checkpoint ("save at breakpoint"), restart the
  worker group (re-rendezvous so the RCCL world is re-formed) while restarts
  remain; membership change (new/returning nodes waiting) -> restart without
  consuming a retry;
* host the asynchronous flash-checkpoint saver (shm -> storage) whose shm
  outlives the worker processes, so restarted workers restore from memory;
* heartbeats + resource reports; optional network check before training.
"""

import json
import os
import shutil
import signal
import socket
import subprocess
import sys
import tempfile
import threading
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

from ..common import env_utils
from ..common.constants import (Accelerators, JobConstant, NodeEnv, NodeStatus, RendezvousName,
                                TrainingExceptionLevel)
from ..common.log import logger
from ..common.rpc import find_free_port, find_free_port_in_range, find_free_port_in_set
from .master_client import MasterClient



def _hw_queues(env: Dict[str, str]):
    """Hardware queues per worker process.  HIP maps streams of one priority
    onto at most GPU_MAX_HW_QUEUES hardware queues (default 4) and shares
    them round-robin beyond that.  A worker here has more streams than that
    (compute, RCCL's own and torch's RCCL stream, the attention backward's
    dQ stream, the checkpoint snapshot / flush / restore streams); once RCCL
    has taken its queues, a later stream can land on the compute stream's
    queue, and a 20 GB checkpoint flush queued there stretched the next three
    GPT2-1.5B steps from 109 to ~155 ms (profiles/r5/flush_queue_sharing.md).
    The copier's flush stream is a normal-priority stream, which does not
    share that way at 4 queues (107.3 ms at 4 and 107.2 at 8).  An import
    standby creates its compute stream before RCCL's (its HBM reservation
    belongs to it, ``standby.py``) and therefore also creates the flush
    stream right after it; with the flush created later it shared the
    compute stream's queue (every step after a save +385 ms,
    ``profiles/r6/bench_1gpu_import_queue_sharing.json``).  At 8 queues the
    flush's blit kernels instead run beside every step (deep-standby steps
    after a save 110 -> 117-124 ms, goodput 93.5 -> 88.9 %,
    ``profiles/r6/bench_1gpu_8queues.json``), so the inherited value is kept
    by default.  DWAMD_GPU_MAX_HW_QUEUES=N raises it to N (at most 32)."""
    want = int(os.getenv("DWAMD_GPU_MAX_HW_QUEUES", "0") or 0)
    try:
        cur = int(env.get("GPU_MAX_HW_QUEUES", "4"))
    except ValueError:
        cur = 4
    if want > cur:
        env["GPU_MAX_HW_QUEUES"] = str(min(want, 32))

class RendezvousTimeoutError(RuntimeError):
    pass


class NodeCheckFailedError(RuntimeError):
    pass


@dataclass
class ElasticLaunchConfig:
    min_nodes: int = 1
    max_nodes: int = 1
    nproc_per_node: int = 1
    run_id: str = "dwamd"
    max_restarts: int = JobConstant.MAX_RESTART_DEFAULT
    monitor_interval: float = 0.1
    join_timeout: float = JobConstant.RDZV_JOIN_TIMEOUT_DEFAULT
    lastcall_timeout: float = 3.0
    pend_timeout: float = float("inf")
    node_unit: int = 1
    network_check: bool = False
    comm_perf_test: bool = False
    exclude_straggler: bool = False
    save_at_breakpoint: bool = True
    auto_config: bool = False
    auto_tunning: bool = False
    accelerator: str = Accelerators.AMD_GPU
    log_dir: str = ""
    redirects: bool = False
    node_rank: int = 0
    local_addr: str = ""
    heartbeat_interval: float = JobConstant.HEARTBEAT_INTERVAL
    exit_barrier_timeout: float = 300.0
    stop_timeout: float = 15.0
    extra_env: Dict[str, str] = field(default_factory=dict)
    # pre-started interpreters (torch imported) that become the next workers
    warm_standby: bool = field(default_factory=lambda: os.getenv("DWAMD_WARM_STANDBY", "1") == "1")
    standby_delay: float = field(default_factory=lambda: float(os.getenv("DWAMD_STANDBY_DELAY", "3")))
    # "import": standbys pre-import torch only (any script); "deep": standbys
    # run the script up to standby_point() (model on the GPU, kernels warm,
    # checkpoint shm pinned) -- see standby.py
    standby_mode: str = field(default_factory=lambda: os.getenv("DWAMD_STANDBY_MODE", "import"))
    # on a worker failure the surviving local workers are usually blocked in
    # a collective with the dead rank: give them this long after SIGTERM
    # before SIGKILL (the breakpoint checkpoint is persisted from shm by the
    # agent, not by the dying workers)
    failure_stop_timeout: float = field(default_factory=lambda: float(os.getenv("DWAMD_FAILURE_STOP_TIMEOUT", "2")))
    # JSONL timeline of agent events (failure detected, restart, ...) for
    # goodput accounting; "" = off
    event_log: str = field(default_factory=lambda: os.getenv("DWAMD_AGENT_EVENT_LOG", ""))
    # persist the breakpoint checkpoint while the new workers already start
    async_breakpoint_save: bool = True
    # exit (and let the platform relaunch the node) on GPU/driver fault signatures
    exit_on_node_error: bool = field(default_factory=lambda: os.getenv("DWAMD_EXIT_ON_NODE_ERROR", "0") == "1")
    # > 0: a worker whose heartbeat file (atorch.fault_tolerance.heartbeat) is
    # older than this is treated as hung and the worker group is relaunched
    hang_timeout: float = field(default_factory=lambda: float(os.getenv("DWAMD_HANG_TIMEOUT", "0")))

    def auto_configure_params(self):
        """nnodes from NODE_NUM, nproc from the visible GPUs, network check
        on for >= 4 nodes (reference training.py:140-168)."""
        n = int(os.getenv(NodeEnv.NODE_NUM, "0") or 0)
        if n > 0:
            self.min_nodes = self.max_nodes = n
        if self.accelerator == Accelerators.AMD_GPU:
            ng = _visible_gpu_count()
            if ng > 0:
                self.nproc_per_node = ng
        if self.max_nodes >= 4:
            self.network_check = True


def _visible_gpu_count() -> int:
    """Count GPUs without initialising HIP in this process (sysfs / env)."""
    vis = os.getenv("HIP_VISIBLE_DEVICES") or os.getenv("ROCR_VISIBLE_DEVICES") or os.getenv(
        "CUDA_VISIBLE_DEVICES")
    if vis:
        return len([v for v in vis.split(",") if v.strip() != ""])
    try:
        import glob

        n = 0
        for p in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/gpu_id"):
            with open(p) as f:
                if int(f.read().strip() or 0) != 0:
                    n += 1
        return n
    except Exception:
        return 0


@dataclass
class WorkerProcess:
    local_rank: int
    global_rank: int
    proc: subprocess.Popen
    log_path: str = ""


class RunResult:
    SUCCEEDED = "SUCCEEDED"
    FAILED = "FAILED"
    HEALTHY = "HEALTHY"

    def __init__(self, state: str, failures: Optional[Dict[int, dict]] = None):
        self.state = state
        self.failures = failures or {}


class MasterRendezvousHandler:
    """Join the master's rendezvous and wait for a world containing us."""

    def __init__(self, client: MasterClient, config: ElasticLaunchConfig, rdzv_name=RendezvousName.ELASTIC_TRAINING):
        self.client = client
        self.config = config
        self.name = rdzv_name
        self.node_rank = config.node_rank

    def next_rendezvous(self) -> Tuple[int, int, Dict[int, int]]:
        self.client.join_rendezvous(self.node_rank, self.config.nproc_per_node, self.name)
        start = time.time()
        # poll fast first (a single-node restart completes on the first polls),
        # then back off to the reference's 1 s interval
        delay = 0.02
        cap = JobConstant.RDZV_POLL_INTERVAL if self.config.lastcall_timeout > 1 else 0.1
        while True:
            rnd, group, world = self.client.get_comm_world(self.name, self.node_rank)
            if world and self.node_rank in world:
                return rnd, group, world
            if world and self.node_rank not in world and time.time() - start > self.config.pend_timeout:
                raise RendezvousTimeoutError("node not admitted into the world")
            if time.time() - start > self.config.join_timeout:
                raise RendezvousTimeoutError(f"rendezvous {self.name} timed out after {self.config.join_timeout}s")
            time.sleep(delay)
            delay = min(cap, delay * 2)

    def num_nodes_waiting(self) -> int:
        return self.client.num_nodes_waiting(self.name)


class ElasticTrainingAgent:
    def __init__(self, config: ElasticLaunchConfig, entrypoint: str, args: List[str], client: MasterClient,
                 is_module: bool = False):
        self.config = config
        self.entrypoint = entrypoint
        self.args = list(args)
        self.is_module = is_module
        self.client = client
        self.rdzv = MasterRendezvousHandler(client, config)
        self.workers: List[WorkerProcess] = []
        self.restart_count = 0
        self.remaining_restarts = config.max_restarts
        self.round = 0
        self.world: Dict[int, int] = {}
        self.group_rank = 0
        self.master_addr = ""
        self.master_port = 0
        self._stop_hb = threading.Event()
        self._exit_evt = threading.Event()  # set by the exit watcher: a worker is failing
        self._hostname = config.local_addr or _local_ip()
        self.events: List[Tuple[float, str]] = []  # (time, what) for goodput accounting
        self._standby: Dict[int, subprocess.Popen] = {}
        self._workers_started_at = 0.0
        self._bp_thread: Optional[threading.Thread] = None
        self._reapers: List[threading.Thread] = []
        # worker <-> agent control files (heartbeats, relaunch requests)
        self.ctl_dir = os.path.join(tempfile.gettempdir(), "dwamd_ctl",
                                    f"{config.run_id}_n{config.node_rank}_{os.getpid()}")
        os.makedirs(self.ctl_dir, exist_ok=True)

    def _event(self, what: str, **kw):
        t = time.time()
        self.events.append((t, what))
        if self.config.event_log:
            try:
                with open(self.config.event_log, "a") as f:
                    f.write(json.dumps(dict({"t": t, "event": what, "restart": self.restart_count}, **kw)) + "\n")
            except OSError:
                pass

    # ------------------------------------------------------------ ranks
    @staticmethod
    def assign_ranks(node_rank: int, world: Dict[int, int]) -> Tuple[int, int, List[int]]:
        """(group_rank, world_size, global ranks of this node's workers)."""
        nodes = sorted(world)
        group_rank = nodes.index(node_rank)
        offset = sum(world[n] for n in nodes[:group_rank])
        return group_rank, sum(world.values()), list(range(offset, offset + world[node_rank]))

    def _store_key(self, what: str) -> str:
        return f"{self.config.run_id}/round{self.round}/{what}"

    def _free_port(self) -> int:
        hp = os.getenv("HOST_PORTS", "")
        if hp:
            try:
                return find_free_port_in_set([int(p) for p in hp.split(",") if p])
            except RuntimeError:
                pass
        try:
            return find_free_port_in_range(20000, 30000)
        except RuntimeError:
            return find_free_port()

    def _rendezvous(self):
        t0 = time.time()
        self.round, _group, self.world = self.rdzv.next_rendezvous()
        self.group_rank, world_size, ranks = self.assign_ranks(self.config.node_rank, self.world)
        if self.group_rank == 0:
            self.master_addr = self._hostname
            self.master_port = self._free_port()
            self.client.kv_store_set(self._store_key("master"), f"{self.master_addr}:{self.master_port}".encode())
        else:
            deadline = time.time() + self.config.join_timeout
            while True:
                v = self.client.kv_store_get(self._store_key("master"))
                if v:
                    a, p = v.decode().rsplit(":", 1)
                    self.master_addr, self.master_port = a, int(p)
                    break
                if time.time() > deadline:
                    raise RendezvousTimeoutError("no MASTER_ADDR published")
                time.sleep(0.05)
        self._event("rendezvous", seconds=round(time.time() - t0, 4), round=self.round)
        logger.info(f"rendezvous round {self.round} ({time.time() - t0:.2f}s): world={self.world} "
                    f"group_rank={self.group_rank} ranks={ranks} master={self.master_addr}:{self.master_port}")
        return ranks, world_size

    # ----------------------------------------------------------- workers
    def _worker_env(self, local_rank: int, global_rank: int, world_size: int) -> Dict[str, str]:
        env = dict(os.environ)
        env.update(self.config.extra_env)
        env.update({
            "LOCAL_RANK": str(local_rank),
            "RANK": str(global_rank),
            "GROUP_RANK": str(self.group_rank),
            "ROLE_RANK": str(global_rank),
            "ROLE_NAME": "dlrover-trainer",
            "LOCAL_WORLD_SIZE": str(self.config.nproc_per_node),
            "WORLD_SIZE": str(world_size),
            "GROUP_WORLD_SIZE": str(len(self.world)),
            "ROLE_WORLD_SIZE": str(world_size),
            "MASTER_ADDR": self.master_addr,
            "MASTER_PORT": str(self.master_port),
            "TORCHELASTIC_RESTART_COUNT": str(self.restart_count),
            "TORCHELASTIC_MAX_RESTARTS": str(self.config.max_restarts),
            "TORCHELASTIC_RUN_ID": self.config.run_id,
            "TORCHELASTIC_USE_AGENT_STORE": "False",
            NodeEnv.NODE_RANK: str(self.config.node_rank),
            NodeEnv.DLROVER_MASTER_ADDR: self.client.master_addr,
            "HSA_ENABLE_IPC_MODE_LEGACY": os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"),
            "DWAMD_AGENT_CTL_DIR": self.ctl_dir,
            "DWAMD_STANDBY_MODE": self.config.standby_mode,  # the HBM-budget preflight sizes for it
        })
        env.setdefault("OMP_NUM_THREADS", "1")
        # RCCL watchdog: a collective past DWAMD_COLLECTIVE_TIMEOUT_S tears the
        # process down (the agent then restarts the group) instead of hanging
        env.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "3")
        _hw_queues(env)
        return env

    def _clear_ctl(self):
        for f in os.listdir(self.ctl_dir):
            try:
                os.unlink(os.path.join(self.ctl_dir, f))
            except OSError:
                pass

    def _ctl_failures(self) -> Dict[int, dict]:
        """Relaunch requests and stale heartbeats from the control dir."""
        out = {}
        now = time.time()
        try:
            entries = list(os.scandir(self.ctl_dir))
        except OSError:
            return out
        by_lr = {w.local_rank: w for w in self.workers}
        for e in entries:
            kind, _, lr = e.name.partition(".")
            if not lr.isdigit() or int(lr) not in by_lr:
                continue
            w = by_lr[int(lr)]
            if kind == "relaunch":
                try:
                    with open(e.path) as f:
                        reason = f.read()
                except OSError:
                    reason = "relaunch requested"
                out[w.global_rank] = {"local_rank": w.local_rank, "exitcode": -1, "message": reason,
                                      "timestamp": int(now)}
            elif kind == "hb" and self.config.hang_timeout > 0:
                try:
                    age = now - e.stat().st_mtime
                except OSError:
                    continue
                if age > self.config.hang_timeout:
                    out[w.global_rank] = {"local_rank": w.local_rank, "exitcode": -1,
                                          "message": f"hang: no heartbeat for {age:.0f}s", "timestamp": int(now)}
        return out

    def _start_workers(self):
        ranks, world_size = self._rendezvous()
        adopt = self._can_adopt_pg(ranks, world_size)
        self._clear_ctl()
        self.workers = []
        warm = 0
        for lr, gr in enumerate(ranks):
            env = self._worker_env(lr, gr, world_size)
            log_path = ""
            if self.config.log_dir:
                os.makedirs(self.config.log_dir, exist_ok=True)
                log_path = os.path.join(self.config.log_dir,
                                        f"{self.config.run_id}_r{self.restart_count}_rank{gr}.log")
            p = self._activate_standby(lr, env, log_path, adopt)
            if p is None and adopt:
                # a standby of the pre-formed set vanished: the ones already
                # activated wait in a group that can never complete -- stop
                # them and start the whole local group without adoption
                logger.warning("pre-formed group incomplete at activation: forming the world cold")
                self._stop_workers(timeout=0)
                self._discard_standbys()
                self._clear_ctl()
                self._start_group_cold(ranks, world_size)
                return
            if p is None:
                p = self._cold_start(env, log_path)
            else:
                warm += 1
            self.workers.append(WorkerProcess(lr, gr, p, log_path))
        self._workers_started_at = time.time()
        self._preform_sent = False
        self._event("workers_started", warm=warm, n=len(self.workers), pg_adopted=adopt)
        logger.info(f"started {len(self.workers)} workers (restart {self.restart_count}, "
                    f"{warm} from warm standby{', pre-formed process group adopted' if adopt else ''})")

    def _start_group_cold(self, ranks: List[int], world_size: int):
        self.workers = []
        for lr, gr in enumerate(ranks):
            env = self._worker_env(lr, gr, world_size)
            log_path = ""
            if self.config.log_dir:
                log_path = os.path.join(self.config.log_dir,
                                        f"{self.config.run_id}_r{self.restart_count}_rank{gr}.log")
            self.workers.append(WorkerProcess(lr, gr, self._cold_start(env, log_path), log_path))
        self._workers_started_at = time.time()
        self._preform_sent = False
        self._event("workers_started", warm=0, n=len(self.workers), pg_adopted=False)

    # --------------------------------------- pre-formed process groups
    def _preform_wanted(self) -> bool:
        """Pre-form the standbys' communicator only when the world is this
        node alone (the next world is then, barring a membership change,
        exactly the standby set) -- see pg_preform.py."""
        return (self.config.warm_standby and os.getenv("DWAMD_STANDBY_PREFORM", "1") == "1"
                and len(self.world) == 1 and self.config.nproc_per_node >= 1)

    def _pg_store_addr(self) -> str:
        """The agent hosts the TCPStore the standbys rendezvous on (it never
        touches the GPU; the store outlives every worker generation)."""
        if getattr(self, "_pg_store", None) is None:
            import datetime

            import torch.distributed as dist

            port = self._free_port()
            self._pg_store = dist.TCPStore("127.0.0.1", port, is_master=True, wait_for_workers=False,
                                           timeout=datetime.timedelta(seconds=300))
            self._pg_store_port = port
        return f"127.0.0.1:{self._pg_store_port}"

    def _standbys_parked(self) -> bool:
        from .standby import READY_PREFIX

        if len(self._standby) < self.config.nproc_per_node:
            return False
        return all(p.poll() is None and os.path.exists(os.path.join(self.ctl_dir, READY_PREFIX + str(lr)))
                   for lr, p in self._standby.items())

    def _maybe_preform(self):
        if getattr(self, "_preform_sent", False) or not self._preform_wanted() or not self._standbys_parked():
            return
        self._preform_sent = True
        self._preform_gen = getattr(self, "_preform_gen", 0) + 1
        spec = {"store": self._pg_store_addr(), "prefix": f"{self.config.run_id}/standby_pg/{self._preform_gen}/",
                "world": self.config.nproc_per_node, "backend": os.getenv("DWAMD_STANDBY_PG_BACKEND", "auto"),
                "timeout": float(os.getenv("DWAMD_STANDBY_PG_TIMEOUT", "30"))}
        self._preform_prefix = spec["prefix"]
        for lr, p in self._standby.items():
            try:
                p.stdin.write(json.dumps({"preform": spec}) + "\n")
                p.stdin.flush()
            except (BrokenPipeError, OSError):
                pass
        self._event("standby_pg_preform", world=spec["world"], gen=self._preform_gen)

    def _can_adopt_pg(self, ranks: List[int], world_size: int) -> bool:
        """Adopt the standbys' pre-formed group iff the new world is exactly
        this node's local ranks 0..n-1 and every standby reported the group
        of the current generation formed."""
        from .pg_preform import PG_MARK_PREFIX

        prefix = getattr(self, "_preform_prefix", None)
        n = self.config.nproc_per_node
        if prefix is None or world_size != n or ranks != list(range(n)) or len(self._standby) != n:
            return False
        for lr, p in self._standby.items():
            if p.poll() is not None:
                return False
            try:
                with open(os.path.join(self.ctl_dir, PG_MARK_PREFIX + str(lr))) as f:
                    if f.read().split()[0] != prefix:
                        return False
            except (OSError, IndexError):
                return False
        return True

    def _cold_start(self, env: Dict[str, str], log_path: str) -> subprocess.Popen:
        cmd = [sys.executable, "-u"] + (["-m", self.entrypoint] if self.is_module else [self.entrypoint]) + self.args
        out, err = None, None
        if log_path:
            out = open(log_path, "w")
            err = subprocess.STDOUT
        p = subprocess.Popen(cmd, env=env, stdout=out, stderr=err, start_new_session=True)
        if out is not None:
            out.close()
        return p

    # ------------------------------------------------------ warm standby
    def _standby_env(self, local_rank: int) -> Dict[str, str]:
        env = dict(os.environ)
        env.update(self.config.extra_env)
        env.setdefault("OMP_NUM_THREADS", "1")
        env["DWAMD_AGENT_CTL_DIR"] = self.ctl_dir
        env["DWAMD_STANDBY_LOCAL_RANK"] = str(local_rank)
        _hw_queues(env)
        if self.config.standby_mode == "deep":
            from .standby import STANDBY_ENV

            # provisional worker environment: the device is known, the world
            # is not (RANK / WORLD_SIZE / MASTER_* arrive at activation)
            for k in ("RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "GROUP_RANK", "ROLE_RANK"):
                env.pop(k, None)
            env.update({
                "LOCAL_RANK": str(local_rank),
                "LOCAL_WORLD_SIZE": str(self.config.nproc_per_node),
                "ROLE_NAME": "dlrover-trainer",
                "TORCHELASTIC_RESTART_COUNT": str(self.restart_count + 1),
                "TORCHELASTIC_RUN_ID": self.config.run_id,
                NodeEnv.NODE_RANK: str(self.config.node_rank),
                "HSA_ENABLE_IPC_MODE_LEGACY": os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"),
                "DWAMD_AGENT_CTL_DIR": self.ctl_dir,
                STANDBY_ENV: "1",
            })
        return env

    def _standbys_useful(self) -> bool:
        """A standby only ever becomes a worker at a restart: with the restart
        budget spent on a fixed single-node job (no membership restarts
        either) it would only compete with the live, just-recovered workers
        -- its interpreter start, HIP context, HBM reservation (the driver
        clears fresh VRAM) and shm pinning ran into their restore and first
        checkpoint flushes (0.3-2.7 s save stalls, profiles/r4 bench runs)."""
        return self.remaining_restarts > 0 or self.config.max_nodes > 1

    def _spawn_standbys(self):
        """Start one standby process per local rank for the next (re)start."""
        if not self.config.warm_standby:
            return
        if not self._standbys_useful():
            if not getattr(self, "_standby_skip_logged", False):
                self._standby_skip_logged = True
                self._event("standby_skipped", reason="no restarts left")
            return
        deep = self.config.standby_mode == "deep"
        for lr in range(self.config.nproc_per_node):
            p = self._standby.get(lr)
            if p is not None and p.poll() is None:
                continue
            env = self._standby_env(lr)
            if deep:
                from .standby import SPEC_ENV

                log = ""
                if self.config.log_dir:
                    os.makedirs(self.config.log_dir, exist_ok=True)
                    log = os.path.join(self.config.log_dir, f"{self.config.run_id}_standby{self.restart_count + 1}"
                                                            f"_local{lr}.log")
                env[SPEC_ENV] = json.dumps({"entry": self.entrypoint, "args": self.args, "module": self.is_module,
                                            "cwd": os.getcwd(), "log": log})
            self._standby[lr] = subprocess.Popen(
                [sys.executable, "-u", "-m", "dlrover_wuqiong_amd.elastic_agent.standby"], env=env,
                stdin=subprocess.PIPE, start_new_session=True, text=True)
        self._event("standby_spawned", mode=self.config.standby_mode)

    def standbys_ready(self) -> bool:
        """All local standbys alive (and, in deep mode, parked in standby_point)."""
        if not self.config.warm_standby or len(self._standby) < self.config.nproc_per_node:
            return False
        for lr, p in self._standby.items():
            if p.poll() is not None:
                return False
            if self.config.standby_mode == "deep":
                from .standby import READY_PREFIX

                if not os.path.exists(os.path.join(self.ctl_dir, READY_PREFIX + str(lr))):
                    return False
        return True

    def _activate_standby(self, local_rank: int, env: Dict[str, str], log_path: str, adopt_pg: bool = False):
        p = self._standby.pop(local_rank, None)
        if p is None:
            return None
        if p.poll() is not None:
            return None
        cmd = {"env": env, "entry": self.entrypoint, "args": self.args, "module": self.is_module,
               "log": log_path, "cwd": os.getcwd(), "adopt_pg": adopt_pg}
        try:
            p.stdin.write(json.dumps(cmd) + "\n")
            p.stdin.close()
        except (BrokenPipeError, OSError):
            return None
        return p

    def _discard_standbys(self):
        for p in self._standby.values():
            try:
                if p.poll() is None:
                    p.stdin.close()  # the standby exits on EOF
                    p.wait(timeout=5)
            except Exception:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except (ProcessLookupError, PermissionError):
                    pass
        self._standby = {}

    def _job_pids(self) -> List[int]:
        pids = [w.proc.pid for w in self.workers if w.proc.poll() is None]
        return pids + [p.pid for p in self._standby.values() if p.poll() is None]

    def _sample_gpu_pdevs(self):
        """Remember which GPUs (PCI addresses) this node's workers / standbys
        hold open, and the largest worker's VRAM: the teardown-overlap
        decision looks at those GPUs and asks for room for one more worker."""
        from .monitor import ResourceMonitor

        workers = {w.proc.pid for w in self.workers if w.proc.poll() is None}
        found, vram = ResourceMonitor.process_gpu_usage(self._job_pids())
        if found:
            self._gpu_pdevs = found
        wv = [v for p, v in vram.items() if p in workers]
        if wv:
            self._worker_vram = max(wv)

    def _teardown_overlap_ok(self) -> bool:
        """May new workers start while the old ones are still exiting (the
        driver frees their HBM only at the end of the teardown)?  Yes when
        every GPU this job uses (its processes' DRM fds; all GPUs of the host
        if unknown) has free HBM for another worker of the last sampled size
        (+ DWAMD_OVERLAP_TEARDOWN_MARGIN_GB, default 8) -- the replacement
        may need all of it even when its standby pre-reserved part; with no
        size known, when the GPU is at most DWAMD_OVERLAP_TEARDOWN_MAX_USED
        (default 0.5) full.  amdgpu sysfs / fdinfo only (the agent never
        initialises HIP); no readable GPU -> wait."""
        from .monitor import ResourceMonitor

        pdevs = getattr(self, "_gpu_pdevs", None)
        stats = ResourceMonitor.gpu_stats(pdevs)
        need = getattr(self, "_worker_vram", 0)
        if need > 0:
            # the replacement is the standby: what it already holds in its
            # allocator cache (standby_warm marker = bytes reserved after the
            # warm-profile replay) it does not allocate again
            need = max(0, need - self._standby_reserved())
            need_mb = (need >> 20) + int(float(os.getenv("DWAMD_OVERLAP_TEARDOWN_MARGIN_GB", "8")) * 1024)
            ok = bool(stats) and all(g.total_memory_mb - g.used_memory_mb >= need_mb for g in stats)
            rule = f"free >= {need_mb / 1024:.1f} GiB"
        else:
            frac = float(os.getenv("DWAMD_OVERLAP_TEARDOWN_MAX_USED", "0.5"))
            ok = bool(stats) and all(g.used_memory_mb <= frac * g.total_memory_mb for g in stats)
            rule = f"used <= {frac}"
        logger.info(f"teardown overlap {'on' if ok else 'off'} ({rule}): GPUs {sorted(pdevs) if pdevs else 'all'} "
                    f"free GiB {[round((g.total_memory_mb - g.used_memory_mb) / 1024, 1) for g in stats]}")
        return ok

    def _standby_reserved(self) -> int:
        """Smallest HBM reservation among this node's waiting standbys (0 if
        any has not reported one): standby.py writes it into its
        ``standby_warm.<local rank>`` marker once the warm profile ran."""
        from .standby import WARM_PREFIX

        standby = getattr(self, "_standby", None)
        if not standby:
            return 0
        vals = []
        for lr in standby:
            try:
                with open(os.path.join(self.ctl_dir, WARM_PREFIX + str(lr))) as f:
                    vals.append(max(0, int(f.read().strip() or 0)))
            except (OSError, ValueError):
                return 0
        return min(vals) if vals else 0

    def _stop_workers(self, timeout: Optional[float] = None, wait: bool = True):
        """SIGTERM every live worker group, SIGKILL after ``timeout``.
        ``wait=False``: return at once and reap in the background (the next
        workers may start while the old processes are still being torn down
        -- their GPU memory is released by the driver at exit)."""
        timeout = self.config.stop_timeout if timeout is None else timeout
        workers, self.workers = self.workers, []
        for w in workers:
            if w.proc.poll() is None:
                try:
                    os.killpg(w.proc.pid, signal.SIGTERM if timeout > 0 else signal.SIGKILL)
                except ProcessLookupError:
                    pass

        def reap():
            deadline = time.time() + timeout
            for w in workers:
                while w.proc.poll() is None and time.time() < deadline:
                    time.sleep(0.02)
                if w.proc.poll() is None:
                    try:
                        os.killpg(w.proc.pid, signal.SIGKILL)
                    except ProcessLookupError:
                        pass
                    w.proc.wait()

        if wait:
            reap()
        else:
            t = threading.Thread(target=reap, daemon=True, name="dwamd-reap")
            t.start()
            self._reapers.append(t)

    def _exit_watch_loop(self):
        """Failure detection off the monitor period: every DWAMD_EXIT_POLL_S
        (5 ms) read each worker's /proc stat and wake the main loop as soon as
        one is inside do_exit with a failure status (``_exiting_code``) --
        the 100 ms monitor sleep otherwise adds ~50 ms to every recovery.
        Reads only, never reaps (the main loop's ``poll`` does)."""
        interval = float(os.getenv("DWAMD_EXIT_POLL_S", "0.005"))
        signaled = set()  # Popen objects (by identity: pids get reused across restarts)
        while not self._stop_hb.wait(interval):
            for w in list(self.workers):
                p = w.proc
                if p in signaled:
                    continue
                if p.returncode not in (None, 0) or _exiting_code(p.pid) is not None:
                    signaled.add(p)
                    self._exit_evt.set()

    def _monitor_workers(self) -> RunResult:
        codes = [(w, w.proc.poll()) for w in self.workers]
        # a SIGKILLed / crashing worker is reaped only after its address space
        # (tens of GB of pinned host + GPU mappings) is torn down, ~0.7 s on
        # MI355X; the kernel publishes the exit code before that teardown
        codes = [(w, c if c is not None else _exiting_code(w.proc.pid)) for w, c in codes]
        failed = {w.global_rank: self._failure(w, c) for w, c in codes if c not in (None, 0)}
        if failed:
            return RunResult(RunResult.FAILED, failed)
        if all(c == 0 for _w, c in codes):
            return RunResult(RunResult.SUCCEEDED)
        hung = self._ctl_failures()
        if hung:
            logger.error(f"relaunch requested / hang detected: { {r: f['message'] for r, f in hung.items()} }")
            return RunResult(RunResult.FAILED, hung)
        return RunResult(RunResult.HEALTHY)

    def _failure(self, w: WorkerProcess, code: int) -> dict:
        msg = ""
        if w.log_path and os.path.exists(w.log_path):
            try:
                with open(w.log_path, errors="replace") as f:
                    msg = f.read()[-2000:]
            except OSError:
                pass
        return {"local_rank": w.local_rank, "exitcode": code, "message": msg,
                "timestamp": int(time.time())}

    # ----------------------------------------------------- checkpointing
    def _saver(self):
        from .ckpt_saver import AsyncCheckpointSaver

        return AsyncCheckpointSaver.get_ckpt_saver()

    def _save_ckpt_to_storage(self):
        """Persist the latest in-memory checkpoint after a failure.  The shm
        outlives the workers and a save always writes the *other* slot, so
        this runs concurrently with the restart (the new workers restore from
        the same memory while it is written to storage)."""
        if not self.config.save_at_breakpoint:
            return
        saver = self._saver()
        if saver is None:
            return
        client = self.client if len(self.world) > 1 else None

        def run():
            try:
                saver.save_shm_to_storage(60, client)
            except Exception as e:
                logger.warning(f"breakpoint save failed: {e}")

        if self._bp_thread is not None and self._bp_thread.is_alive():
            self._bp_thread.join()
        if self.config.async_breakpoint_save:
            self._bp_thread = threading.Thread(target=run, daemon=True, name="dwamd-breakpoint-save")
            self._bp_thread.start()
        else:
            run()

    # --------------------------------------------------------- main loop
    def _heartbeat_loop(self):
        from .monitor import ResourceMonitor

        rm = ResourceMonitor()
        while not self._stop_hb.wait(self.config.heartbeat_interval):
            try:
                self.client.report_heart_beat()
                cpu, mem = rm.sample()
                self.client.report_used_resource(mem, cpu, rm.gpu_stats())
            except Exception as e:
                logger.debug(f"heartbeat failed: {e}")

    def run(self) -> int:
        from .ckpt_saver import AsyncCheckpointSaver

        AsyncCheckpointSaver.start_async_saving_ckpt()
        self.client.report_rdzv_params(self.config.min_nodes, self.config.max_nodes, self.config.lastcall_timeout,
                                       self.config.node_unit, int(self.config.join_timeout))
        hb = threading.Thread(target=self._heartbeat_loop, daemon=True, name="dwamd-heartbeat")
        hb.start()
        if float(os.getenv("DWAMD_EXIT_POLL_S", "0.005")) > 0:
            threading.Thread(target=self._exit_watch_loop, daemon=True, name="dwamd-exit-watch").start()
        if self.config.log_dir:
            from .diagnosis import DiagnosisMonitor

            DiagnosisMonitor(self.client, self.config.log_dir).start()
        try:
            if self.config.network_check:
                from .node_check import run_network_check

                ok = run_network_check(self.config, self.client)
                if not ok:
                    raise NodeCheckFailedError(f"node {self.config.node_rank} failed the network check")
            if self.config.comm_perf_test:
                from .node_check import run_comm_perf_check

                ok, rep = run_comm_perf_check(self.config, self.client)
                self._event("comm_perf", ok=ok, allreduce_busbw_gbps=rep.get("allreduce_busbw_gbps"),
                            slow_links=rep.get("slow_links"), slow_node=rep.get("slow_node"))
                if not ok:
                    raise NodeCheckFailedError(f"node {self.config.node_rank} failed the comm perf check")
            self._start_workers()
            AsyncCheckpointSaver.register_signal_handler()
            self._install_signal_handlers()
            return self._invoke_run()
        finally:
            self._stop_hb.set()
            self._discard_standbys()
            for t in self._reapers:
                t.join(timeout=30)
            if self._bp_thread is not None:
                self._bp_thread.join(timeout=600)

    def _invoke_run(self) -> int:
        last_membership_check = 0.0
        while True:
            # woken early by the exit watcher; cleared before the check, so a
            # failure that lands during it wakes the next wait at once
            if self._exit_evt.wait(self.config.monitor_interval):
                self._exit_evt.clear()
            if (self.config.warm_standby and not self._standby
                    and time.time() - self._workers_started_at > self.config.standby_delay):
                self._spawn_standbys()
            if self._standby:
                self._maybe_preform()
            res = self._monitor_workers()
            now = time.time()
            if now - getattr(self, "_pdev_sampled_at", 0.0) > 5.0 and res.state == RunResult.HEALTHY:
                self._pdev_sampled_at = now
                self._sample_gpu_pdevs()
            if res.state == RunResult.SUCCEEDED:
                self._event("succeeded")
                self._discard_standbys()
                if self._bp_thread is not None:
                    self._bp_thread.join(timeout=600)
                self._exit_barrier()
                self._wait_async_saver()
                self._cleanup_shm()
                try:  # the master may already be going away (its host node finished first)
                    self.client.report_node_event(NodeStatus.SUCCEEDED, "")
                    self.client.kv_store_add(f"{self.config.run_id}/exit_done", 1)
                except Exception as e:
                    logger.warning(f"final success report not delivered: {e}")
                return 0
            if res.state == RunResult.FAILED:
                self._event("failure_detected", ranks={str(r): f["exitcode"] for r, f in res.failures.items()})
                logger.error(f"worker failure: { {r: (f['exitcode']) for r, f in res.failures.items()} }")
                from .diagnosis import classify_failure

                level = max((classify_failure(f.get("message", "")) for f in res.failures.values()),
                            key=lambda lv: lv == TrainingExceptionLevel.NODE_ERROR)
                # deep standbys already hold their memory; import-mode
                # replacements allocate theirs, so they start before the failed
                # processes are torn down (~1-1.5 s for tens of GB of mappings)
                # only when every GPU has room for a second copy
                self._stop_workers(timeout=self.config.failure_stop_timeout,
                                   wait=self.config.standby_mode != "deep" and not self._teardown_overlap_ok())
                self._event("workers_stopped")
                if level == TrainingExceptionLevel.NODE_ERROR and self.config.exit_on_node_error:
                    # hardware signature: let the platform replace this node
                    logger.error("GPU/driver fault signature in the worker log: exiting for node relaunch")
                    try:
                        self.client.report_failures(json.dumps(res.failures), self.restart_count, level)
                    except Exception:
                        pass
                    self._save_ckpt_to_storage()
                    self._discard_standbys()
                    if self._bp_thread is not None:
                        self._bp_thread.join(timeout=600)
                    self.client.report_node_event(NodeStatus.FAILED, "node error")
                    return 2
                restart = self.remaining_restarts > 0
                if restart:
                    # restart first: reporting and the breakpoint persist are
                    # off the recovery critical path
                    self.remaining_restarts -= 1
                    self._restart_workers()
                try:
                    self.client.report_failures(json.dumps(res.failures), self.restart_count - int(restart), level)
                except Exception:
                    pass
                self._save_ckpt_to_storage()
                if restart:
                    continue
                self._discard_standbys()
                self.client.report_node_event(NodeStatus.FAILED, "max restarts reached")
                return 1
            # healthy: check membership change (rate limited)
            now = time.time()
            if now - last_membership_check > 2.0:
                last_membership_check = now
                if self.rdzv.num_nodes_waiting() > 0:
                    logger.info("new/returning nodes are waiting: restart the worker group")
                    self._stop_workers()
                    self._save_ckpt_to_storage()
                    self._restart_workers(count=False)

    def _install_signal_handlers(self):
        """SIGTERM/SIGINT: stop the worker processes first (they run in their
        own sessions), then the saver's handler persists shm and exits."""
        for sig in (signal.SIGTERM, signal.SIGINT):
            prev = signal.getsignal(sig)

            def handler(signum, frame, prev=prev):
                self._stop_workers(timeout=5)
                if callable(prev):
                    prev(signum, frame)
                raise SystemExit(128 + signum)

            signal.signal(sig, handler)

    def _restart_workers(self, count: bool = True):
        from .ckpt_saver import AsyncCheckpointSaver

        if count:
            self.restart_count += 1
        AsyncCheckpointSaver.reset()
        self._start_workers()

    def _exit_barrier(self):
        key = f"{self.config.run_id}/exit_barrier"
        try:
            n = self.client.kv_store_add(key, 1)
            deadline = time.time() + self.config.exit_barrier_timeout
            while n < len(self.world) and time.time() < deadline:
                time.sleep(0.2)
                n = int(self.client.kv_store_add(key, 0))
        except Exception:
            pass

    def _wait_async_saver(self):
        saver = self._saver()
        if saver is None:
            return
        t0 = time.time()
        while saver.wait_saving_checkpoint() and time.time() - t0 < 600:
            time.sleep(0.2)

    def _cleanup_shm(self):
        """The job finished: release the node's checkpoint memory."""
        import glob

        from ..common.multi_process import shm_name

        ns = shm_name("", "").rstrip("_")
        saver = self._saver()
        if saver is not None:
            saver.close()
        for f in glob.glob(f"/dev/shm/{ns}*"):
            try:
                os.remove(f)
            except OSError:
                pass


_PF_EXITING = 0x4


def _exiting_code(pid: int) -> Optional[int]:
    """Exit status of a process that is already inside ``do_exit`` but not
    yet reaped (``Popen.returncode`` convention: -signal or exit code), or
    None while it runs.  Reads ``/proc/<pid>/stat``: ``flags`` (field 9)
    carries PF_EXITING, ``exit_code`` (field 52, Linux >= 3.5) the wait
    status.  A clean exit (0) is left to ``poll()``: success needs the real
    reap, only failures are worth acting on early."""
    try:
        with open(f"/proc/{pid}/stat", "rb") as f:
            raw = f.read()
    except OSError:
        return None
    fields = raw[raw.rfind(b")") + 2:].split()
    if len(fields) < 50:
        return None
    try:
        flags = int(fields[6])
        status = int(fields[49])
    except ValueError:
        return None
    if not flags & _PF_EXITING or status == 0:
        return None
    sig = status & 0x7F
    return -sig if sig else (status >> 8) & 0xFF


def _local_ip() -> str:
    try:
        s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        s.connect(("10.255.255.255", 1))
        ip = s.getsockname()[0]
        s.close()
        return ip
    except OSError:
        return "127.0.0.1"


def launch_agent(config: ElasticLaunchConfig, entrypoint: str, args: List[str], master_addr: str,
                 is_module: bool = False) -> int:
    global LAST_WORLD_NODES
    client = MasterClient(master_addr, node_id=config.node_rank)
    agent = ElasticTrainingAgent(config, entrypoint, args, client, is_module=is_module)
    try:
        return agent.run()
    finally:
        # the launcher hosting the master keeps it up until every node of the
        # FINAL world reported (an elastic job may have grown past min_nodes)
        LAST_WORLD_NODES = len(agent.world)
        agent._stop_workers(timeout=5)
        shutil.rmtree(agent.ctl_dir, ignore_errors=True)


LAST_WORLD_NODES = 0


def wait_nodes_done(master_addr: str, run_id: str, nnodes: int, timeout: float = 15.0) -> bool:
    """Used by the launcher that hosts the local master: keep the master up
    until every node reported its final state (or ``timeout``)."""
    client = MasterClient(master_addr, node_id=-1)
    deadline = time.time() + timeout
    while time.time() < deadline:
        try:
            if client.kv_store_add(f"{run_id}/exit_done", 0) >= nnodes:
                return True
        except Exception:
            return False
        time.sleep(0.1)
    return False
