"""``dwamd-run``: elastic launcher, a superset of ``torchrun``.

Parity: reference ``dlrover/trainer/torch/elastic_run.py`` (``parse_args``
:125-186 with ``--network-check``, ``--comm-perf-test``, ``--node_unit``,
``--auto_config``, ``--auto_tunning``, ``--exclude-straggler``,
``--save_at_breakpoint``, ``--accelerator``; ``_launch_dlrover_local_master``
:237; ``_check_dlrover_master_available`` :269; ``run`` :342; console entry
``dlrover-run`` -> ``main``).

Usage::

    dwamd-run --nnodes=1 --nproc-per-node=8 train.py --args ...
    dwamd-run --nnodes=2:4 --nproc-per-node=8 --master-addr=host0 \
              --master-port=29400 --network-check train.py

Node 0 hosts the job master on ``--master-addr:--master-port`` unless
``DLROVER_MASTER_ADDR`` points at an existing master (K8s deployments).
"""

import argparse
import os
import subprocess
import sys
import time
import uuid
from typing import List, Optional, Tuple

from ..common.constants import Accelerators, NodeEnv
from ..common.log import logger
from ..common.rpc import addr_connected, find_free_port


def _bool(v) -> bool:
    return str(v).lower() in ("1", "true", "yes", "y", "on")


def parse_args(argv=None):
    p = argparse.ArgumentParser("dwamd-run", description="elastic training launcher (torchrun superset)")
    p.add_argument("--nnodes", default="1", help="N or MIN:MAX")
    p.add_argument("--nproc-per-node", "--nproc_per_node", default="1")
    p.add_argument("--node-rank", "--node_rank", type=int, default=int(os.getenv("NODE_RANK", "0") or 0))
    p.add_argument("--master-addr", "--master_addr", default="127.0.0.1")
    p.add_argument("--master-port", "--master_port", type=int, default=0)
    p.add_argument("--max-restarts", "--max_restarts", type=int, default=3)
    p.add_argument("--monitor-interval", "--monitor_interval", type=float, default=0.1)
    p.add_argument("--rdzv-backend", "--rdzv_backend", default="dlrover-master")
    p.add_argument("--rdzv-endpoint", "--rdzv_endpoint", default="")
    p.add_argument("--rdzv-id", "--rdzv_id", default="")
    p.add_argument("--rdzv-conf", "--rdzv_conf", default="")
    p.add_argument("--standalone", action="store_true")
    p.add_argument("--local-addr", "--local_addr", default="")
    p.add_argument("--log-dir", "--log_dir", default="")
    p.add_argument("--redirects", default="")
    p.add_argument("-m", "--module", action="store_true")
    p.add_argument("--no-python", "--no_python", action="store_true")
    # DLRover extensions
    p.add_argument("--network-check", "--network_check", action="store_true")
    p.add_argument("--comm-perf-test", "--comm_perf_test", action="store_true")
    p.add_argument("--node_unit", "--node-unit", type=int, default=1)
    p.add_argument("--auto_config", "--auto-config", action="store_true")
    p.add_argument("--auto_tunning", "--auto-tunning", action="store_true")
    p.add_argument("--exclude-straggler", "--exclude_straggler", action="store_true")
    p.add_argument("--save_at_breakpoint", "--save-at-breakpoint", type=_bool, default=True)
    p.add_argument("--relaunch-on-hang", "--relaunch_on_hanging", type=float, default=0.0, metavar="SECONDS",
                   help="relaunch the worker group when a worker heartbeat is older than SECONDS")
    p.add_argument("--standby-mode", "--standby_mode", choices=["import", "deep", "off"],
                   default=os.getenv("DWAMD_STANDBY_MODE", "import"),
                   help="warm standby per local rank: 'import' pre-imports torch (any script); 'deep' runs the "
                        "script up to trainer.elastic.standby_point() (model on GPU, kernels warm, ckpt shm pinned)")
    p.add_argument("--standby-delay", "--standby_delay", type=float,
                   default=float(os.getenv("DWAMD_STANDBY_DELAY", "3")),
                   help="seconds after (re)starting the workers before the next standbys are spawned")
    p.add_argument("--event-log", "--event_log", default=os.getenv("DWAMD_AGENT_EVENT_LOG", ""),
                   help="append the agent's timeline (failures, restarts, rendezvous) as JSON lines")
    p.add_argument("--xpu-timer", "--xpu_timer", action="store_true",
                   help="install the xpu_timer (GEMM/collective timing + hang detection) in every worker")
    p.add_argument("--accelerator", default=Accelerators.AMD_GPU,
                   choices=[Accelerators.AMD_GPU, Accelerators.NVIDIA_GPU, Accelerators.ASCEND_NPU,
                            Accelerators.CPU])
    p.add_argument("training_script")
    p.add_argument("training_script_args", nargs=argparse.REMAINDER)
    return p.parse_args(argv)


def _parse_nnodes(s: str) -> Tuple[int, int]:
    if ":" in s:
        a, b = s.split(":")
        return int(a), int(b)
    return int(s), int(s)


def _parse_rdzv_conf(s: str) -> dict:
    out = {}
    for kv in filter(None, s.split(",")):
        k, _, v = kv.partition("=")
        out[k.strip()] = v.strip()
    return out


def launch_local_master(port: int, node_num: int) -> subprocess.Popen:
    cmd = [sys.executable, "-m", "dlrover_wuqiong_amd.master.master", "--port", str(port),
           "--node_num", str(node_num), "--loop_interval", "5"]
    p = subprocess.Popen(cmd, start_new_session=True)
    addr = f"127.0.0.1:{port}"
    deadline = time.time() + 60
    while time.time() < deadline:
        if addr_connected(addr, 0.5):
            return p
        if p.poll() is not None:
            raise RuntimeError("local master exited during start-up")
        time.sleep(0.1)
    raise TimeoutError("local master did not come up")


def build_config(a) -> "ElasticLaunchConfig":
    from ..elastic_agent.agent import ElasticLaunchConfig

    mn, mx = _parse_nnodes(a.nnodes)
    nproc = a.nproc_per_node
    conf = _parse_rdzv_conf(a.rdzv_conf)
    cfg = ElasticLaunchConfig(min_nodes=mn, max_nodes=mx, nproc_per_node=1, run_id=a.rdzv_id or "dwamd",
                              max_restarts=a.max_restarts, monitor_interval=a.monitor_interval,
                              node_unit=a.node_unit, network_check=a.network_check,
                              comm_perf_test=a.comm_perf_test, exclude_straggler=a.exclude_straggler,
                              save_at_breakpoint=a.save_at_breakpoint, auto_config=a.auto_config,
                              auto_tunning=a.auto_tunning, accelerator=a.accelerator, log_dir=a.log_dir,
                              node_rank=a.node_rank, local_addr=a.local_addr)
    cfg.warm_standby = a.standby_mode != "off"
    if a.standby_mode != "off":
        cfg.standby_mode = a.standby_mode
    cfg.standby_delay = a.standby_delay
    cfg.event_log = a.event_log
    if a.relaunch_on_hang > 0:
        cfg.hang_timeout = a.relaunch_on_hang
    if a.xpu_timer:
        cfg.extra_env["DWAMD_XPU_TIMER"] = "1"
    if "join_timeout" in conf:
        cfg.join_timeout = float(conf["join_timeout"])
    if "lastcall_timeout" in conf:
        cfg.lastcall_timeout = float(conf["lastcall_timeout"])
    if "pend_timeout" in conf:
        cfg.pend_timeout = float(conf["pend_timeout"])
    if nproc in ("auto", "gpu"):
        from ..elastic_agent.agent import _visible_gpu_count

        cfg.nproc_per_node = max(1, _visible_gpu_count())
    elif nproc == "cpu":
        cfg.nproc_per_node = os.cpu_count() or 1
    else:
        cfg.nproc_per_node = int(nproc)
    if cfg.auto_config:
        cfg.auto_configure_params()
    return cfg


def run(a) -> int:
    from ..elastic_agent.agent import launch_agent

    cfg = build_config(a)
    master_addr = os.getenv(NodeEnv.DLROVER_MASTER_ADDR, "")
    master_proc: Optional[subprocess.Popen] = None
    if not master_addr and a.master_port and a.node_rank == 0 and not a.standalone:
        # a job master is already serving there (e.g. started by the platform)
        from ..common.rpc import addr_connected

        if addr_connected(f"{a.master_addr}:{a.master_port}"):
            master_addr = f"{a.master_addr}:{a.master_port}"
            os.environ[NodeEnv.DLROVER_MASTER_ADDR] = master_addr
    if not master_addr:
        port = a.master_port or find_free_port()
        if a.node_rank == 0 or a.standalone:
            master_proc = launch_local_master(port, cfg.max_nodes)
            master_addr = f"127.0.0.1:{port}" if a.standalone or a.master_addr in ("", "127.0.0.1",
                                                                                   "localhost") else f"{a.master_addr}:{port}"
        else:
            master_addr = f"{a.master_addr}:{port}"
        os.environ[NodeEnv.DLROVER_MASTER_ADDR] = master_addr
    if not cfg.run_id or cfg.run_id == "dwamd":
        cfg.run_id = os.getenv(NodeEnv.JOB_NAME, "") or f"dwamd-{uuid.uuid5(uuid.NAMESPACE_DNS, master_addr).hex[:8]}"
    os.environ.setdefault(NodeEnv.TORCHELASTIC_RUN_ID, cfg.run_id)
    logger.info(f"dwamd-run: master={master_addr} nodes={cfg.min_nodes}:{cfg.max_nodes} nproc={cfg.nproc_per_node} "
                f"node_rank={cfg.node_rank}")
    rc = 1
    try:
        rc = launch_agent(cfg, a.training_script, a.training_script_args, master_addr, is_module=a.module)
        return rc
    finally:
        if master_proc is not None:
            if rc == 0 and cfg.max_nodes > 1:
                from ..elastic_agent import agent as _agent

                _agent.wait_nodes_done(master_addr, cfg.run_id, max(cfg.min_nodes, _agent.LAST_WORLD_NODES))
            master_proc.terminate()
            try:
                master_proc.wait(timeout=10)
            except subprocess.TimeoutExpired:
                master_proc.kill()


def main(argv=None) -> int:
    import faulthandler
    import signal

    faulthandler.register(signal.SIGUSR2, all_threads=True)  # `kill -USR2 <agent pid>` dumps every stack
    a = parse_args(argv)
    return run(a)


if __name__ == "__main__":
    sys.exit(main())
