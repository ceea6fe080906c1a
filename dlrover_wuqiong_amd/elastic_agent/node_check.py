"""Agent side of the network / node health check.

Two rounds on the master's network-check rendezvous (parity: reference
``NodeCheckElasticAgent`` training.py:864-1013, ``run_network_check``
:1112): every round the node runs the check workload
(``trainer/node_check.py``) with the other node(s) of its group, reports
success + elapsed time, and after the rounds asks the master which nodes are
faulty (failed both rounds) or stragglers (> 2x median time).
"""

import os
import shutil
import subprocess
import sys
import time
from typing import Tuple

from ..common.constants import ConfigPath, NodeStatus, RendezvousName
from ..common.log import logger
from .master_client import MasterClient


def _run_check_round(config, client: MasterClient, round_idx: int) -> Tuple[bool, float]:
    from .agent import ElasticTrainingAgent, MasterRendezvousHandler

    rdzv = MasterRendezvousHandler(client, config, RendezvousName.NETWORK_CHECK)
    rnd, group, world = rdzv.next_rendezvous()
    group_rank, world_size, ranks = ElasticTrainingAgent.assign_ranks(config.node_rank, world)
    key = f"{config.run_id}/netcheck/{rnd}/{group}/master"
    if group_rank == 0:
        from ..common.rpc import find_free_port

        addr = config.local_addr or "127.0.0.1"
        client.kv_store_set(key, f"{addr}:{find_free_port()}".encode())
    deadline = time.time() + 120
    v = b""
    while not v and time.time() < deadline:
        v = client.kv_store_get(key)
        time.sleep(0.05)
    maddr, mport = v.decode().rsplit(":", 1)
    out_dir = os.path.join(ConfigPath.NETWORK_CHECK_DATA_DIR, f"n{config.node_rank}")
    shutil.rmtree(out_dir, ignore_errors=True)
    procs = []
    for lr, gr in enumerate(ranks):
        env = dict(os.environ)
        env.update({"LOCAL_RANK": str(lr), "RANK": str(gr), "WORLD_SIZE": str(world_size),
                    "LOCAL_WORLD_SIZE": str(config.nproc_per_node), "MASTER_ADDR": maddr, "MASTER_PORT": mport,
                    "GROUP_RANK": str(group_rank)})
        procs.append(subprocess.Popen([sys.executable, "-m", "dlrover_wuqiong_amd.trainer.node_check",
                                       "--out-dir", out_dir], env=env))
    ok = all(p.wait(timeout=600) == 0 for p in procs)
    elapsed = 0.0
    for lr in range(len(ranks)):
        try:
            with open(os.path.join(out_dir, f"{lr}.txt")) as f:
                elapsed = max(elapsed, float(f.read().strip()))
        except (OSError, ValueError):
            ok = False
    client.report_network_check_status(config.node_rank, NodeStatus.SUCCEEDED if ok else NodeStatus.FAILED,
                                       elapsed)
    logger.info(f"network check round {round_idx}: ok={ok} elapsed={elapsed:.3f}s group={list(world)}")
    return ok, elapsed


def _wait_result(client: MasterClient, fn, timeout=300):
    deadline = time.time() + timeout
    while True:
        nodes, reason = fn()
        if reason != "Waiting node" or time.time() > deadline:
            return nodes, reason
        time.sleep(0.5)


def run_network_check(config, client: MasterClient) -> bool:
    """True if this node is healthy (and, with ``exclude_straggler``, not a
    straggler)."""
    for i in range(2):
        _run_check_round(config, client, i)
        faults, reason = _wait_result(client, lambda: tuple(client.network_check_success()[1:]))
        if not faults:
            break
    faults, _ = _wait_result(client, lambda: tuple(client.network_check_success()[1:]))
    if config.node_rank in faults:
        logger.error(f"node {config.node_rank} is faulty (network check)")
        return False
    if config.exclude_straggler:
        stragglers, _ = _wait_result(client, client.check_straggler)
        if config.node_rank in stragglers:
            logger.error(f"node {config.node_rank} is a straggler and is excluded")
            return False
    return True
