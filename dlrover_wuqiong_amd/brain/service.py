"""Brain: job-metrics store + resource-optimisation service.

The reference runs this as a Go gRPC service backed by MySQL
(``dlrover/go/brain``: ``pkg/server/server.go`` persist_metrics /
get_job_metrics / optimize, ``pkg/datastore``, and the resource-plan
algorithms under ``pkg/optimizer/implementation/optalgorithm``).  Here it is
a Python service on the framework's JSON-over-gRPC transport
(``common/rpc.py``) with an SQLite datastore (stdlib, file or in-memory), so
a job master on any node can report metrics and ask for plans.

Optimisation algorithms (``opt_type``):

* ``job_create_resource``  initial worker resources of a new job from the
  history of jobs with the same name: memory = max observed x (1 + margin),
  CPU = p90 utilised cores x (1 + margin); defaults when there is no history.
* ``job_oom_resource``     a worker OOMed: memory x factor (capped).
* ``job_running_workers``  AllReduce worker count from the measured speed
  records (throughput at each worker count): scale to the largest count whose
  marginal per-worker efficiency stays above ``min_efficiency``; cap at
  ``max_workers`` and round down to ``node_unit``.
* ``job_hot_ps``           PS nodes whose CPU utilisation exceeds the
  threshold get ``factor`` x CPU (the PS path of the reference).

Parity: reference ``dlrover/proto/brain.proto`` (``persist_metrics``,
``get_job_metrics``, ``optimize``) and ``dlrover/python/brain/client.py``.
"""

import json
import sqlite3
import threading
import time
from typing import Any, Dict, List, Optional

from ..common.log import logger
from ..common.rpc import RpcServer

MB = 1


class BrainDatastore:
    def __init__(self, path: str = ":memory:"):
        self._db = sqlite3.connect(path, check_same_thread=False)
        self._lock = threading.Lock()
        with self._lock:
            self._db.execute("CREATE TABLE IF NOT EXISTS job_metrics (job_uuid TEXT, job_name TEXT, user TEXT, "
                             "metrics_type TEXT, payload TEXT, ts REAL)")
            self._db.execute("CREATE INDEX IF NOT EXISTS idx_uuid ON job_metrics(job_uuid)")
            self._db.execute("CREATE INDEX IF NOT EXISTS idx_name ON job_metrics(job_name)")
            self._db.commit()

    def persist(self, m: Dict[str, Any]):
        with self._lock:
            self._db.execute("INSERT INTO job_metrics VALUES (?, ?, ?, ?, ?, ?)",
                             (m["job_uuid"], m.get("job_name", ""), m.get("user", ""), m["metrics_type"],
                              json.dumps(m.get("metrics", {})), m.get("ts", time.time())))
            self._db.commit()

    def query(self, job_uuid: Optional[str] = None, job_name: Optional[str] = None,
              metrics_type: Optional[str] = None) -> List[Dict[str, Any]]:
        q, args = "SELECT job_uuid, job_name, user, metrics_type, payload, ts FROM job_metrics WHERE 1=1", []
        if job_uuid is not None:
            q += " AND job_uuid = ?"
            args.append(job_uuid)
        if job_name is not None:
            q += " AND job_name = ?"
            args.append(job_name)
        if metrics_type is not None:
            q += " AND metrics_type = ?"
            args.append(metrics_type)
        q += " ORDER BY ts"
        with self._lock:
            rows = self._db.execute(q, args).fetchall()
        return [{"job_uuid": r[0], "job_name": r[1], "user": r[2], "metrics_type": r[3],
                 "metrics": json.loads(r[4]), "ts": r[5]} for r in rows]


class MetricsType:
    JOB_META = "job_meta"
    RESOURCE_USAGE = "resource_usage"       # {"node_type", "cpu_used", "memory_used_mb", "cpu", "memory_mb"}
    SPEED = "training_speed"                # {"worker_num", "speed"}  (samples or steps / s)
    OOM = "oom"                             # {"node_type", "memory_mb"}
    HYPER_PARAMS = "training_hyper_params"  # {"batch_size", "epoch", "max_steps"}
    WORKFLOW = "workflow_feature"


class BrainOptimizer:
    def __init__(self, store: BrainDatastore, margin: float = 0.2, oom_factor: float = 1.5,
                 max_memory_mb: int = 2 << 20, default_cpu: float = 8.0, default_memory_mb: int = 65536):
        self.store = store
        self.margin, self.oom_factor = margin, oom_factor
        self.max_memory_mb = max_memory_mb
        self.default_cpu, self.default_memory_mb = default_cpu, default_memory_mb

    def _job_name(self, job_uuid: str) -> str:
        rows = self.store.query(job_uuid=job_uuid)
        return rows[0]["job_name"] if rows else ""

    def optimize(self, req: Dict[str, Any]) -> Dict[str, Any]:
        t = req.get("opt_type")
        fn = getattr(self, f"_opt_{t}", None)
        if fn is None:
            raise ValueError(f"unknown optimisation type {t}")
        return fn(req)

    def _opt_job_create_resource(self, req):
        name = req.get("job_name") or self._job_name(req.get("job_uuid", ""))
        usage = [r["metrics"] for r in self.store.query(job_name=name, metrics_type=MetricsType.RESOURCE_USAGE)
                 if r["metrics"].get("node_type", "worker") == "worker" and r["job_uuid"] != req.get("job_uuid")]
        if not usage:
            return {"worker": {"cpu": self.default_cpu, "memory_mb": self.default_memory_mb}, "source": "default"}
        mem = max(u.get("memory_used_mb", 0) for u in usage)
        cpus = sorted(u.get("cpu_used", 0.0) for u in usage)
        p90 = cpus[min(len(cpus) - 1, int(0.9 * len(cpus)))]
        return {"worker": {"cpu": round(max(1.0, p90 * (1 + self.margin)), 2),
                           "memory_mb": int(min(self.max_memory_mb, mem * (1 + self.margin)))},
                "source": f"history({len(usage)} records)"}

    def _opt_job_oom_resource(self, req):
        ooms = [r["metrics"] for r in self.store.query(job_uuid=req["job_uuid"], metrics_type=MetricsType.OOM)]
        if not ooms:
            return {}
        last = ooms[-1]
        mem = int(min(self.max_memory_mb, last.get("memory_mb", self.default_memory_mb) * self.oom_factor))
        return {last.get("node_type", "worker"): {"memory_mb": mem}}

    def _opt_job_running_workers(self, req):
        min_eff = float(req.get("min_efficiency", 0.7))
        max_w = int(req.get("max_workers", 0)) or 1 << 30
        unit = max(1, int(req.get("node_unit", 1)))
        recs = [r["metrics"] for r in self.store.query(job_uuid=req["job_uuid"], metrics_type=MetricsType.SPEED)]
        by_n: Dict[int, List[float]] = {}
        for r in recs:
            by_n.setdefault(int(r["worker_num"]), []).append(float(r["speed"]))
        if not by_n:
            return {}
        pts = sorted((n, sorted(v)[len(v) // 2]) for n, v in by_n.items())  # median speed per count
        cur_n = int(req.get("current_workers", pts[-1][0]))
        best = pts[0][0]
        for (n0, s0), (n1, s1) in zip(pts, pts[1:]):
            per0 = s0 / n0
            marginal = (s1 - s0) / max(1, n1 - n0)
            if marginal >= min_eff * per0:
                best = n1
            else:
                break
        if best == pts[-1][0] and best >= cur_n:
            # still scaling well at the largest measured count: try one more unit
            best = best + unit
        target = min(max_w, best) // unit * unit
        return {"worker": {"count": max(unit, target)}, "curve": pts}

    def _opt_job_hot_ps(self, req):
        thr = float(req.get("cpu_threshold", 0.8))
        factor = float(req.get("factor", 1.5))
        latest: Dict[str, Dict] = {}
        for r in self.store.query(job_uuid=req["job_uuid"], metrics_type=MetricsType.RESOURCE_USAGE):
            m = r["metrics"]
            if m.get("node_type") == "ps":
                latest[m.get("node_name", "ps")] = m
        plan = {}
        for name, m in latest.items():
            if m.get("cpu", 0) > 0 and m.get("cpu_used", 0) / m["cpu"] > thr:
                plan[name] = {"cpu": round(m["cpu"] * factor, 2)}
        return {"ps_nodes": plan} if plan else {}


class BrainService:
    """``report``: persist metrics.  ``get``: {"method": "get_job_metrics" |
    "optimize", ...}."""

    def __init__(self, port: int = 0, db_path: str = ":memory:"):
        self.store = BrainDatastore(db_path)
        self.optimizer = BrainOptimizer(self.store)
        self.server = RpcServer(port, self._report, self._get, max_workers=16)
        self.port = self.server.port

    def _report(self, data: bytes) -> bytes:
        try:
            m = json.loads(data)
            for item in (m if isinstance(m, list) else [m]):
                self.store.persist(item)
            return json.dumps({"success": True}).encode()
        except Exception as e:
            logger.warning(f"brain: bad metrics report: {e}")
            return json.dumps({"success": False, "reason": str(e)}).encode()

    def _get(self, data: bytes) -> bytes:
        try:
            req = json.loads(data)
            method = req.get("method")
            if method == "get_job_metrics":
                res = self.store.query(job_uuid=req.get("job_uuid"), metrics_type=req.get("metrics_type"))
            elif method == "optimize":
                res = self.optimizer.optimize(req)
            else:
                raise ValueError(f"unknown method {method}")
            return json.dumps({"success": True, "result": res}).encode()
        except Exception as e:
            return json.dumps({"success": False, "reason": str(e)}).encode()

    def start(self):
        self.server.start()
        return self

    def stop(self):
        self.server.stop()


def main(argv=None):
    import argparse

    p = argparse.ArgumentParser("dwamd-brain")
    p.add_argument("--port", type=int, default=50001)
    p.add_argument("--db", default="brain.sqlite")
    a = p.parse_args(argv)
    svc = BrainService(a.port, a.db).start()
    logger.info(f"brain service on :{svc.port} (db {a.db})")
    try:
        while True:
            time.sleep(3600)
    except KeyboardInterrupt:
        svc.stop()


if __name__ == "__main__":
    main()
