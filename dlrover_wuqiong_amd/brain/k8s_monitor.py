"""Brain cluster side: a Kubernetes monitor that records every ElasticJob
and its nodes (pods) cluster-wide into the Brain datastore, so the
optimizer plans from what actually ran -- including jobs whose master never
reported (crashed, or never started) and OOM kills seen only by the kubelet.

* ``ClusterRecorder`` adds the reference's ``job`` / ``job_node`` tables next
  to the metrics table of ``BrainDatastore`` (same SQLite file): job (uid,
  name, scenario, created / started / finished, status) and job_node (uid,
  name, job uid / name, type, timestamps, resource, status, exit reason);
* ``K8sMonitor`` lists + watches ElasticJob custom resources and the pods
  labelled with an elastic job, and turns the events into recorder upserts;
  a pod terminated with ``OOMKilled`` also persists an ``oom`` metric for the
  job name, which ``job_worker_create_oom_resource`` /
  ``job_ps_oom_resource`` consume (the re-submitted job starts big enough).

Parity: reference ``dlrover/go/brain/cmd/k8smonitor/main.go``,
``pkg/platform/k8s/implementation/watchhandler/elasticjob_handler.go`` /
``elasticjob_node_handler.go`` and ``pkg/datastore/recorder/mysql``
(``job_recorder.go``, ``job_node_recorder.go``); SQLite instead of MySQL,
the framework's stdlib K8s REST client instead of client-go.
"""

import json
import threading
import time
from typing import Any, Dict, List, Optional

from ..common.log import logger
from .service import BrainDatastore, MetricsType

JOB_LABEL = "elasticjob-name"
TYPE_LABEL = "replica-type"


def _ts(s: Optional[str]) -> Optional[float]:
    if not s:
        return None
    try:
        return time.mktime(time.strptime(s.replace("Z", ""), "%Y-%m-%dT%H:%M:%S")) - time.timezone
    except ValueError:
        return None


class ClusterRecorder:
    """job / job_node tables (reference job_recorder.go / job_node_recorder.go)."""

    def __init__(self, store: BrainDatastore):
        self.store = store
        db = store._db
        with store._lock:
            db.execute("CREATE TABLE IF NOT EXISTS job (uid TEXT PRIMARY KEY, name TEXT, scenario TEXT, "
                       "created_at REAL, started_at REAL, finished_at REAL, status TEXT)")
            db.execute("CREATE TABLE IF NOT EXISTS job_node (uid TEXT PRIMARY KEY, name TEXT, job_uuid TEXT, "
                       "job_name TEXT, type TEXT, created_at REAL, started_at REAL, finished_at REAL, "
                       "resource TEXT, status TEXT, exit_reason TEXT, customized_data TEXT)")
            db.execute("CREATE INDEX IF NOT EXISTS idx_node_job ON job_node(job_name)")
            db.commit()

    def upsert_job(self, uid: str, name: str, scenario: str = "", created_at=None, started_at=None,
                   finished_at=None, status: str = ""):
        with self.store._lock:
            self.store._db.execute(
                "INSERT INTO job VALUES (?, ?, ?, ?, ?, ?, ?) ON CONFLICT(uid) DO UPDATE SET name=excluded.name, "
                "scenario=COALESCE(NULLIF(excluded.scenario, ''), job.scenario), "
                "created_at=COALESCE(job.created_at, excluded.created_at), "
                "started_at=COALESCE(job.started_at, excluded.started_at), "
                "finished_at=COALESCE(excluded.finished_at, job.finished_at), "
                "status=COALESCE(NULLIF(excluded.status, ''), job.status)",
                (uid, name, scenario, created_at, started_at, finished_at, status))
            self.store._db.commit()

    def upsert_node(self, uid: str, name: str, job_uuid: str, job_name: str, node_type: str, created_at=None,
                    started_at=None, finished_at=None, resource: Optional[Dict] = None, status: str = "",
                    exit_reason: str = "", customized: Optional[Dict] = None):
        with self.store._lock:
            self.store._db.execute(
                "INSERT INTO job_node VALUES (?, ?, ?, ?, ?, ?, ?, ?, ?, ?, ?, ?) ON CONFLICT(uid) DO UPDATE SET "
                "status=COALESCE(NULLIF(excluded.status, ''), job_node.status), "
                "started_at=COALESCE(job_node.started_at, excluded.started_at), "
                "finished_at=COALESCE(excluded.finished_at, job_node.finished_at), "
                "exit_reason=COALESCE(NULLIF(excluded.exit_reason, ''), job_node.exit_reason), "
                "resource=COALESCE(excluded.resource, job_node.resource)",
                (uid, name, job_uuid, job_name, node_type, created_at, started_at, finished_at,
                 json.dumps(resource) if resource else None, status, exit_reason,
                 json.dumps(customized or {})))
            self.store._db.commit()

    def jobs(self, name: Optional[str] = None) -> List[Dict[str, Any]]:
        q, a = "SELECT uid, name, scenario, created_at, started_at, finished_at, status FROM job", []
        if name is not None:
            q, a = q + " WHERE name = ?", [name]
        with self.store._lock:
            rows = self.store._db.execute(q, a).fetchall()
        keys = ("uid", "name", "scenario", "created_at", "started_at", "finished_at", "status")
        return [dict(zip(keys, r)) for r in rows]

    def nodes(self, job_name: Optional[str] = None) -> List[Dict[str, Any]]:
        q, a = ("SELECT uid, name, job_uuid, job_name, type, created_at, started_at, finished_at, resource, status, "
                "exit_reason FROM job_node"), []
        if job_name is not None:
            q, a = q + " WHERE job_name = ?", [job_name]
        with self.store._lock:
            rows = self.store._db.execute(q, a).fetchall()
        keys = ("uid", "name", "job_uuid", "job_name", "type", "created_at", "started_at", "finished_at",
                "resource", "status", "exit_reason")
        out = []
        for r in rows:
            d = dict(zip(keys, r))
            d["resource"] = json.loads(d["resource"]) if d["resource"] else {}
            out.append(d)
        return out


def _mem_mb(v: str) -> int:
    v = str(v)
    for suf, mul in (("Ti", 1 << 20), ("Gi", 1 << 10), ("Mi", 1), ("Ki", 1.0 / 1024), ("T", 1e12 / 2 ** 20),
                     ("G", 1e9 / 2 ** 20), ("M", 1e6 / 2 ** 20), ("K", 1e3 / 2 ** 20)):
        if v.endswith(suf):
            return int(float(v[: -len(suf)]) * mul)
    try:
        return int(float(v) / (1 << 20))
    except ValueError:
        return 0


def _cpu(v) -> float:
    v = str(v)
    return float(v[:-1]) / 1000.0 if v.endswith("m") else float(v or 0)


class K8sMonitor:
    """Watch ElasticJobs + their pods and record them (one per cluster)."""

    def __init__(self, client, store: BrainDatastore, job_plural: str = "elasticjobs"):
        self.client = client
        self.store = store
        self.recorder = ClusterRecorder(store)
        self.job_plural = job_plural
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self._job_uid: Dict[str, str] = {}
        self._oom_seen = set()

    # ------------------------------------------------------------- handlers
    def on_job(self, obj: Dict, deleted: bool = False):
        md = obj.get("metadata", {})
        name = md.get("name", "")
        uid = md.get("uid") or name
        self._job_uid[name] = uid
        st = obj.get("status", {}) or {}
        phase = st.get("phase", "") or ("Deleted" if deleted else "")
        finished = _ts(st.get("completionTime")) or (time.time() if deleted or phase in ("Succeeded", "Failed")
                                                     else None)
        self.recorder.upsert_job(uid, name, scenario=(md.get("labels") or {}).get("scenario", ""),
                                 created_at=_ts(md.get("creationTimestamp")), started_at=_ts(st.get("startTime")),
                                 finished_at=finished, status=phase)

    def on_pod(self, pod: Dict, deleted: bool = False):
        md = pod.get("metadata", {})
        labels = md.get("labels") or {}
        job = labels.get(JOB_LABEL)
        if not job:
            return
        name = md.get("name", "")
        uid = md.get("uid") or name
        st = pod.get("status", {}) or {}
        phase = st.get("phase", "") or ("Deleted" if deleted else "")
        reason = ""
        for cs in st.get("containerStatuses", []) or []:
            term = (cs.get("state") or {}).get("terminated") or (cs.get("lastState") or {}).get("terminated")
            if term:
                reason = term.get("reason", "") or reason
        req: Dict[str, Any] = {}
        for c in (pod.get("spec", {}) or {}).get("containers", []) or []:
            r = ((c.get("resources") or {}).get("requests") or {})
            if "cpu" in r:
                req["cpu"] = req.get("cpu", 0.0) + _cpu(r["cpu"])
            if "memory" in r:
                req["memory_mb"] = req.get("memory_mb", 0) + _mem_mb(r["memory"])
            for k, v in r.items():
                if k.endswith("gpu"):
                    req["gpu"] = req.get("gpu", 0) + int(v)
        node_type = labels.get(TYPE_LABEL, "worker")
        finished = time.time() if (deleted or phase in ("Succeeded", "Failed")) else None
        self.recorder.upsert_node(uid, name, self._job_uid.get(job, job), job, node_type,
                                  created_at=_ts(md.get("creationTimestamp")), started_at=_ts(st.get("startTime")),
                                  finished_at=finished, resource=req or None, status=phase, exit_reason=reason)
        if reason == "OOMKilled" and uid not in self._oom_seen:
            self._oom_seen.add(uid)
            self.store.persist({"job_uuid": self._job_uid.get(job, job), "job_name": job,
                                "metrics_type": MetricsType.OOM,
                                "metrics": {"node_type": node_type, "memory_mb": req.get("memory_mb", 0)}})
            logger.info(f"brain k8s monitor: {name} of {job} OOMKilled at {req.get('memory_mb', 0)} MB")

    # ----------------------------------------------------------------- loop
    def sync_once(self):
        """List everything (the informer resync of the reference)."""
        for j in self.client.list_custom(self.job_plural):
            self.on_job(j)
        for p in self.client.list_pods():
            self.on_pod(p)  # pods without the elastic-job label are ignored

    def watch_pods_once(self, timeout_s: int = 30):
        for ev in self.client.watch_pods("", timeout_s=timeout_s):
            obj = ev.get("object") or {}
            if obj.get("kind", "Pod") not in ("Pod", None) and "spec" not in obj:
                continue
            self.on_pod(obj, deleted=ev.get("type") == "DELETED")

    def run(self, interval: float = 10.0):
        while not self._stop.is_set():
            try:
                self.sync_once()
                self.watch_pods_once(timeout_s=int(interval))
            except Exception as e:  # keep monitoring through API-server hiccups
                logger.warning(f"brain k8s monitor: {e}")
            self._stop.wait(interval)

    def start(self, interval: float = 10.0):
        self._thread = threading.Thread(target=self.run, args=(interval,), daemon=True, name="dwamd-brain-k8s")
        self._thread.start()
        return self

    def stop(self):
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=30)


def main(argv=None):
    import argparse

    from ..platform.k8s import K8sClient

    p = argparse.ArgumentParser("dwamd-brain-k8s-monitor")
    p.add_argument("--namespace", default="default")
    p.add_argument("--db", default="/tmp/dwamd_brain.sqlite")
    p.add_argument("--interval", type=float, default=10.0)
    a = p.parse_args(argv)
    mon = K8sMonitor(K8sClient(a.namespace), BrainDatastore(a.db))
    mon.run(a.interval)


if __name__ == "__main__":
    main()
