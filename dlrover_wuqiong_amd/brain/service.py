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
* ``job_ps_create_resource``  PS count / CPU / memory of a new PS job from its
  name's history (count = max seen, CPU p90, memory max, x (1 + margin)).
* ``job_ps_cold_create_resource``  no history for the name: the nearest job
  of the same user by parameter count (JOB_META), scaled by the size ratio;
  defaults when nothing is comparable.
* ``job_ps_init_adjust_resource``  early in a run PS memory grows with the
  embedding tables: a least-squares line over (step, memory) extrapolated to
  ``max_steps`` sizes each PS; CPU from its utilisation.
* ``job_ps_resource_util``  over-provisioned PS (utilisation below ``low``)
  shrink to used x (1 + margin), never below ``min_cpu``.
* ``job_ps_oom_resource`` / ``job_worker_create_oom_resource``  OOM at run /
  at creation: memory x factor of the largest OOMed size (creation OOMs use
  the job-name history so a re-submitted job starts big enough).
* ``job_gpu_host_memory``  host memory per GPU node for flash checkpointing:
  model/optimizer state per node x shm slots (2) + pinned staging + the
  agent's headroom, from the JOB_META ``ckpt_bytes_per_node``.

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


    # ------------------------------------------------------------- PS jobs
    def _usage(self, req, node_type: str, name: Optional[str] = None):
        q = self.store.query(job_uuid=req.get("job_uuid") if name is None else None, job_name=name,
                             metrics_type=MetricsType.RESOURCE_USAGE)
        return [r for r in q if r["metrics"].get("node_type") == node_type]

    def _opt_job_ps_create_resource(self, req):
        name = req.get("job_name") or self._job_name(req.get("job_uuid", ""))
        rows = [r for r in self._usage(req, "ps", name) if r["job_uuid"] != req.get("job_uuid")]
        if not rows:
            return self._opt_job_ps_cold_create_resource(req)
        per_job: Dict[str, set] = {}
        for r in rows:
            per_job.setdefault(r["job_uuid"], set()).add(r["metrics"].get("node_name", "ps"))
        count = max(len(v) for v in per_job.values())
        mem = max(r["metrics"].get("memory_used_mb", 0) for r in rows)
        cpus = sorted(r["metrics"].get("cpu_used", 0.0) for r in rows)
        p90 = cpus[min(len(cpus) - 1, int(0.9 * len(cpus)))]
        return {"ps": {"count": count, "cpu": round(max(1.0, p90 * (1 + self.margin)), 2),
                       "memory_mb": int(min(self.max_memory_mb, mem * (1 + self.margin)))},
                "source": f"history({len(per_job)} jobs)"}

    def _opt_job_ps_cold_create_resource(self, req):
        params = float(req.get("model_params", 0))
        user = req.get("user")
        metas = [r for r in self.store.query(metrics_type=MetricsType.JOB_META)
                 if r["job_uuid"] != req.get("job_uuid") and (user is None or r["user"] == user)]
        best = None
        for m in metas:
            p = float(m["metrics"].get("model_params", 0))
            if p > 0 and params > 0:
                d = abs(p - params) / max(p, params)
                if best is None or d < best[0]:
                    best = (d, m, p)
        if best is not None and best[0] <= 0.5:
            _d, m, p = best
            ref = self._opt_job_ps_create_resource({"job_uuid": "", "job_name": m["job_name"]})
            if ref.get("source", "").startswith("history"):
                ratio = params / p
                ps = dict(ref["ps"])
                ps["memory_mb"] = int(min(self.max_memory_mb, ps["memory_mb"] * ratio))
                ps["count"] = max(1, int(round(ps["count"] * max(1.0, ratio))))
                return {"ps": ps, "source": f"similar({m['job_name']}, ratio {ratio:.2f})"}
        return {"ps": {"count": int(req.get("default_ps", 1)), "cpu": self.default_cpu,
                       "memory_mb": self.default_memory_mb}, "source": "default"}

    def _opt_job_ps_init_adjust_resource(self, req):
        max_steps = float(req.get("max_steps", 0))
        out = {}
        by_ps: Dict[str, List[Dict]] = {}
        for r in self._usage(req, "ps"):
            by_ps.setdefault(r["metrics"].get("node_name", "ps"), []).append(r["metrics"])
        for name, ms in by_ps.items():
            pts = [(float(m["step"]), float(m.get("memory_used_mb", 0))) for m in ms if "step" in m]
            plan = {}
            if len(pts) >= 2 and max_steps > 0:
                n = len(pts)
                mx = sum(p[0] for p in pts) / n
                my = sum(p[1] for p in pts) / n
                sxx = sum((p[0] - mx) ** 2 for p in pts)
                slope = sum((p[0] - mx) * (p[1] - my) for p in pts) / sxx if sxx > 0 else 0.0
                final = my + max(0.0, slope) * (max_steps - mx)
                plan["memory_mb"] = int(min(self.max_memory_mb, max(pts[-1][1], final) * (1 + self.margin)))
            last = ms[-1]
            if last.get("cpu", 0) > 0:
                plan["cpu"] = round(max(1.0, last.get("cpu_used", 0.0) * (1 + self.margin)), 2)
            if plan:
                out[name] = plan
        return {"ps_nodes": out} if out else {}

    def _opt_job_ps_resource_util(self, req):
        low = float(req.get("low_threshold", 0.3))
        min_cpu = float(req.get("min_cpu", 1.0))
        latest: Dict[str, Dict] = {}
        for r in self._usage(req, "ps"):
            latest[r["metrics"].get("node_name", "ps")] = r["metrics"]
        plan = {}
        for name, m in latest.items():
            cpu, used = float(m.get("cpu", 0)), float(m.get("cpu_used", 0))
            if cpu > 0 and used / cpu < low:
                plan[name] = {"cpu": round(max(min_cpu, used * (1 + self.margin)), 2)}
        return {"ps_nodes": plan} if plan else {}

    def _opt_job_ps_oom_resource(self, req):
        ooms = [r["metrics"] for r in self.store.query(job_uuid=req["job_uuid"], metrics_type=MetricsType.OOM)
                if r["metrics"].get("node_type") == "ps"]
        if not ooms:
            return {}
        mem = max(o.get("memory_mb", self.default_memory_mb) for o in ooms)
        return {"ps": {"memory_mb": int(min(self.max_memory_mb, mem * self.oom_factor))}}

    def _opt_job_worker_create_oom_resource(self, req):
        name = req.get("job_name") or self._job_name(req.get("job_uuid", ""))
        ooms = [r["metrics"] for r in self.store.query(job_name=name, metrics_type=MetricsType.OOM)
                if r["metrics"].get("node_type", "worker") == "worker"]
        base = self._opt_job_create_resource(req)["worker"]
        if not ooms:
            return {"worker": base}
        mem = max(o.get("memory_mb", 0) for o in ooms) * self.oom_factor
        return {"worker": {"cpu": base["cpu"], "memory_mb": int(min(self.max_memory_mb, max(mem,
                                                                                           base["memory_mb"])))}}

    # ------------------------------------------------------- GPU host memory
    def _opt_job_gpu_host_memory(self, req):
        metas = [r["metrics"] for r in self.store.query(job_uuid=req["job_uuid"], metrics_type=MetricsType.JOB_META)]
        ckpt = int(req.get("ckpt_bytes_per_node", 0)) or max((int(m.get("ckpt_bytes_per_node", 0)) for m in metas),
                                                              default=0)
        if ckpt <= 0:
            return {}
        slots = int(req.get("shm_slots", 2))
        staging = int(req.get("pinned_staging_bytes", 0))
        headroom = int(req.get("headroom_mb", 64 << 10))
        mb = (ckpt * slots + staging) // (1 << 20) + headroom
        return {"worker": {"memory_mb": int(min(self.max_memory_mb, mb))},
                "detail": {"ckpt_mb": ckpt >> 20, "slots": slots, "headroom_mb": headroom}}


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
