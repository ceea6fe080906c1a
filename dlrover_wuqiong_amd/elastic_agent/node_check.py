"""Agent side of the network / node health check.

Two rounds on the master's network-check rendezvous (parity: reference
``NodeCheckElasticAgent`` training.py:864-1013, ``run_network_check``
:1112): every round the node runs the check workload
(``trainer/node_check.py``) with the other node(s) of its group, reports
success + elapsed time, and after the rounds asks the master which nodes are
faulty (failed both rounds) or stragglers (> 2x median time).
"""

import json
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


def _median(xs):
    xs = sorted(xs)
    n = len(xs)
    return 0.0 if n == 0 else (xs[n // 2] if n % 2 else 0.5 * (xs[n // 2 - 1] + xs[n // 2]))


def summarize_comm_perf(reports, threshold: float):
    """Node summary from the local ranks' reports: the collectives as rank 0
    measured them (every rank times the same collective), the pairwise link
    matrix and the links slower than ``threshold`` x the median link."""
    reports = sorted(reports, key=lambda r: r.get("local_rank", 0))
    ok = bool(reports) and all(r.get("ok") for r in reports)
    out = {"ok": ok, "world": reports[0].get("world") if reports else 0,
           "init_sec_max": max((r.get("init_sec", 0.0) for r in reports), default=None),
           "matmul_tflops": [r.get("matmul_tflops") for r in reports],
           "collectives": reports[0].get("collectives", []) if reports else []}
    links = {}
    for r in reports:
        for peer, bw in (r.get("links_gbps") or {}).items():
            a, b = sorted((r["rank"], int(peer)))
            links[(a, b)] = min(bw, links.get((a, b), bw))  # a pair is as fast as its slower direction
    med = _median(list(links.values()))
    out["links"] = [{"pair": [a, b], "gbps": bw} for (a, b), bw in sorted(links.items())]
    out["link_median_gbps"] = round(med, 3) if links else None
    out["slow_links"] = [[a, b] for (a, b), bw in sorted(links.items()) if med > 0 and bw < threshold * med]
    big = [c for c in out["collectives"] if c["op"] == "allreduce"]
    out["allreduce_busbw_gbps"] = max((c["bytes"], c["busbw_gbps"]) for c in big)[1] if big else None
    return out


def run_comm_perf_check(config, client: MasterClient, timeout: float = 600.0) -> Tuple[bool, dict]:
    """Communication performance check after a passing health check
    (reference ``comm_perf_check``, training.py:1092-1109,1135-1136;
    ``bm_allreduce`` / ``bm_allgather``, node_check/utils.py:58-132).

    Every node runs the collectives sweep + pairwise link test over its own
    GPUs (xGMI), writes ``comm_perf_n<node>.json`` under the network-check
    dir and publishes its all-reduce bus bandwidth in the master KV store.  A
    node below ``DWAMD_COMM_PERF_THRESHOLD`` (default 0.6) x the median of
    the nodes that reported, or with a link below that fraction of its
    node's median link, is flagged: excluded with ``--exclude-straggler``,
    logged otherwise.  Returns (ok, report)."""
    from ..common.rpc import find_free_port

    threshold = float(os.getenv("DWAMD_COMM_PERF_THRESHOLD", "0.6"))
    out_dir = os.path.join(ConfigPath.NETWORK_CHECK_DATA_DIR, f"perf_n{config.node_rank}")
    shutil.rmtree(out_dir, ignore_errors=True)
    port = str(find_free_port())
    n = config.nproc_per_node
    procs = []
    for lr in range(n):
        env = dict(os.environ)
        env.update({"LOCAL_RANK": str(lr), "RANK": str(lr), "WORLD_SIZE": str(n), "LOCAL_WORLD_SIZE": str(n),
                    "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": port, "GROUP_RANK": "0"})
        procs.append(subprocess.Popen([sys.executable, "-m", "dlrover_wuqiong_amd.trainer.node_check", "--comm-perf",
                                       "--out-dir", out_dir] + os.getenv("DWAMD_COMM_PERF_ARGS", "").split(), env=env))
    ok = True
    for pr in procs:
        try:
            ok = pr.wait(timeout=timeout) == 0 and ok
        except subprocess.TimeoutExpired:
            pr.kill()
            ok = False
    reports = []
    for lr in range(n):
        try:
            with open(os.path.join(out_dir, f"{lr}.json")) as f:
                reports.append(json.load(f))
        except (OSError, ValueError):
            ok = False
    rep = summarize_comm_perf(reports, threshold)
    rep["ok"] = rep["ok"] and ok
    rep["node_rank"] = config.node_rank
    mine = rep.get("allreduce_busbw_gbps") or 0.0
    # cross-node comparison through the master KV store
    key = f"{config.run_id}/comm_perf"
    try:
        client.kv_store_set(f"{key}/{config.node_rank}", json.dumps(mine).encode())
        client.kv_store_add(f"{key}/count", 1)
        deadline = time.time() + 60
        while int(client.kv_store_add(f"{key}/count", 0)) < config.min_nodes and time.time() < deadline:
            time.sleep(0.2)
        peers = {}
        for node in range(max(config.max_nodes, config.node_rank + 1)):
            v = client.kv_store_get(f"{key}/{node}")
            if v:
                peers[node] = float(json.loads(v.decode()))
        med = _median([v for v in peers.values() if v > 0])
        rep["node_busbw_gbps"] = peers
        rep["node_median_busbw_gbps"] = med
        rep["slow_node"] = bool(med > 0 and 0 < mine < threshold * med)
    except Exception as e:  # the check never blocks training on a master hiccup
        logger.warning(f"comm perf: cross-node comparison skipped: {e}")
        rep["slow_node"] = False
    os.makedirs(ConfigPath.NETWORK_CHECK_DATA_DIR, exist_ok=True)
    path = os.path.join(ConfigPath.NETWORK_CHECK_DATA_DIR, f"comm_perf_n{config.node_rank}.json")
    with open(path, "w") as f:
        json.dump(rep, f, indent=1)
    for c in rep["collectives"]:
        logger.info(f"comm perf {c['op']:>13} {c['bytes'] / 2**20:8.1f} MiB: algbw {c['algbw_gbps']:8.2f} GB/s "
                    f"busbw {c['busbw_gbps']:8.2f} GB/s")
    if rep["slow_links"]:
        logger.warning(f"comm perf: slow links (< {threshold} x median {rep['link_median_gbps']} GB/s): "
                       f"{rep['slow_links']}")
    if rep["slow_node"]:
        logger.warning(f"comm perf: node {config.node_rank} all-reduce busbw {mine} GB/s < {threshold} x node median "
                       f"{rep['node_median_busbw_gbps']}")
    healthy = rep["ok"] and not ((rep["slow_node"] or rep["slow_links"]) and config.exclude_straggler)
    logger.info(f"comm perf check: {'ok' if healthy else 'FAILED'} -> {path}")
    return healthy, rep
