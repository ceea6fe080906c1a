"""Kubernetes platform layer: REST client, pod scaler / watcher for the job
master, and the ElasticJob operator (reconciler) -- in Python, on the plain
Kubernetes REST API (``requests``), no client library or Go toolchain.

* ``K8sClient``: in-cluster config (service-account token + CA) or an
  explicit ``base_url``; pods, services, nodes (cordon), custom objects
  (``ElasticJob`` / ``ScalePlan`` of ``elastic.iml.github.io/v1alpha1``) and
  watch streams (``?watch=true`` JSON lines).
* ``PodScaler``: the master's ``Scaler`` -- creates worker pods named
  ``{job}-worker-{id}`` from the job's replica template (``amd.com/gpu``
  resources, ``dwamd-run`` command, ``DWAMD_*`` env incl. the master address
  and node rank) and deletes removed ones.
* ``PodWatcher``: ``NodeWatcher`` mapping pod phases / container exit codes
  (OOMKilled, 137 ...) to ``Node`` status and exit reasons.
* ``ElasticJobOperator``: reconcile loop -- for every ElasticJob without a
  master, create the master pod + service (``python -m
  dlrover_wuqiong_amd.master.master --platform k8s``); mirror the master
  pod phase into ``status.phase``; apply ``ScalePlan`` objects (manual or
  Brain-generated) to the job's replica counts and mark them consumed.

Parity: reference ``dlrover/python/scheduler/kubernetes.py`` (``k8sClient``
:121-572), ``master/scaler/pod_scaler.py`` / ``elasticjob_scaler.py``,
``master/watcher/k8s_watcher.py`` (``PodWatcher`` :194,
``K8sScalePlanWatcher`` :267) and the Go operator
``go/operator/pkg/controllers/{elasticjob,scaleplan}_controller.go``.
"""

import json
import os
import threading
import time
from typing import Dict, Iterator, List, Optional

from ..common.constants import NodeEventType, NodeExitReason, NodeStatus, NodeType
from ..common.log import logger
from ..common.node import Node, NodeResource
from ..master.scaler import ScalePlan, Scaler
from ..master.watcher import NodeEvent, NodeWatcher

GROUP, VERSION = "elastic.iml.github.io", "v1alpha1"
SA_DIR = "/var/run/secrets/kubernetes.io/serviceaccount"
JOB_LABEL, TYPE_LABEL, ID_LABEL, RANK_LABEL = ("elasticjob.dlrover/name", "elasticjob.dlrover/replica-type",
                                              "elasticjob.dlrover/replica-id", "elasticjob.dlrover/rank-index")


class K8sClient:
    def __init__(self, namespace: str = "default", base_url: Optional[str] = None, token: Optional[str] = None,
                 verify=None, timeout: float = 10.0):
        import requests

        self.ns = namespace
        if base_url is None:
            host, port = os.environ.get("KUBERNETES_SERVICE_HOST"), os.environ.get("KUBERNETES_SERVICE_PORT", "443")
            if not host:
                raise RuntimeError("not in a cluster and no base_url given")
            base_url = f"https://{host}:{port}"
            if token is None and os.path.exists(f"{SA_DIR}/token"):
                token = open(f"{SA_DIR}/token").read().strip()
            if verify is None and os.path.exists(f"{SA_DIR}/ca.crt"):
                verify = f"{SA_DIR}/ca.crt"
        self.base = base_url.rstrip("/")
        self.s = requests.Session()
        if token:
            self.s.headers["Authorization"] = f"Bearer {token}"
        self.s.verify = True if verify is None else verify
        self.timeout = timeout

    # -- generic
    def _req(self, method: str, path: str, body=None, params=None, content_type="application/json"):
        r = self.s.request(method, self.base + path, data=json.dumps(body) if body is not None else None,
                           params=params, headers={"Content-Type": content_type}, timeout=self.timeout)
        if r.status_code == 404:
            return None
        if r.status_code >= 400:
            raise RuntimeError(f"k8s {method} {path}: {r.status_code} {r.text[:300]}")
        return r.json() if r.content else {}

    def _core(self, kind: str, name: str = "") -> str:
        return f"/api/v1/namespaces/{self.ns}/{kind}" + (f"/{name}" if name else "")

    def _custom(self, plural: str, name: str = "") -> str:
        return f"/apis/{GROUP}/{VERSION}/namespaces/{self.ns}/{plural}" + (f"/{name}" if name else "")

    # -- pods / services / nodes
    def create_pod(self, pod: Dict):
        return self._req("POST", self._core("pods"), pod)

    def get_pod(self, name: str):
        return self._req("GET", self._core("pods", name))

    def delete_pod(self, name: str):
        return self._req("DELETE", self._core("pods", name))

    def list_pods(self, label_selector: str = "") -> List[Dict]:
        res = self._req("GET", self._core("pods"), params={"labelSelector": label_selector} if label_selector else None)
        return (res or {}).get("items", [])

    def watch_pods(self, label_selector: str = "", resource_version: str = "", timeout_s: int = 60) -> Iterator[Dict]:
        params = {"watch": "true", "timeoutSeconds": str(timeout_s)}
        if label_selector:
            params["labelSelector"] = label_selector
        if resource_version:
            params["resourceVersion"] = resource_version
        with self.s.get(self.base + self._core("pods"), params=params, stream=True, timeout=timeout_s + 5) as r:
            for line in r.iter_lines():
                if line:
                    yield json.loads(line)

    def create_service(self, svc: Dict):
        return self._req("POST", self._core("services"), svc)

    def get_service(self, name: str):
        return self._req("GET", self._core("services", name))

    def cordon_node(self, node_name: str):
        return self._req("PATCH", f"/api/v1/nodes/{node_name}", {"spec": {"unschedulable": True}},
                         content_type="application/merge-patch+json")

    # -- custom objects
    def list_custom(self, plural: str) -> List[Dict]:
        return (self._req("GET", self._custom(plural)) or {}).get("items", [])

    def get_custom(self, plural: str, name: str):
        return self._req("GET", self._custom(plural, name))

    def create_custom(self, plural: str, body: Dict):
        return self._req("POST", self._custom(plural), body)

    def patch_custom(self, plural: str, name: str, patch: Dict):
        return self._req("PATCH", self._custom(plural, name), patch, content_type="application/merge-patch+json")

    def patch_custom_status(self, plural: str, name: str, status: Dict):
        return self._req("PATCH", self._custom(plural, name) + "/status", {"status": status},
                         content_type="application/merge-patch+json")


# ----------------------------------------------------------------------------- pods <-> nodes

_PHASE = {"Pending": NodeStatus.PENDING, "Running": NodeStatus.RUNNING, "Succeeded": NodeStatus.SUCCEEDED,
          "Failed": NodeStatus.FAILED, "Unknown": NodeStatus.UNKNOWN}


def pod_name(job: str, node_type: str, node_id: int) -> str:
    return f"{job}-{node_type}-{node_id}"


def pod_to_node(pod: Dict) -> Node:
    meta, status = pod.get("metadata", {}), pod.get("status", {})
    labels = meta.get("labels", {})
    node = Node(type=labels.get(TYPE_LABEL, NodeType.WORKER), id=int(labels.get(ID_LABEL, 0)),
                rank_index=int(labels.get(RANK_LABEL, labels.get(ID_LABEL, 0))), name=meta.get("name", ""))
    node.status = _PHASE.get(status.get("phase", "Unknown"), NodeStatus.UNKNOWN)
    if meta.get("deletionTimestamp"):
        node.status = NodeStatus.DELETED
    node.host_addr = status.get("podIP", "")
    for cs in status.get("containerStatuses", []) or []:
        term = (cs.get("state", {}) or {}).get("terminated") or (cs.get("lastState", {}) or {}).get("terminated")
        if term:
            reason, code = term.get("reason", ""), int(term.get("exitCode", 0))
            if reason == "OOMKilled":
                node.exit_reason = NodeExitReason.OOM
            elif code == 0:
                node.exit_reason = NodeExitReason.SUCCEEDED
            elif code in (137, 143):
                node.exit_reason = NodeExitReason.KILLED
            elif code in (201, 202):  # reserved: hardware fault detected by the agent
                node.exit_reason = NodeExitReason.HARDWARE_ERROR
            else:
                node.exit_reason = NodeExitReason.FATAL_ERROR
    return node


class PodScaler(Scaler):
    def __init__(self, job_name: str, client: K8sClient, image: str, master_addr: str, command: List[str],
                 gpus_per_node: int = 8, env: Optional[Dict[str, str]] = None, namespace_labels=None):
        super().__init__(job_name)
        self.client, self.image, self.master_addr = client, image, master_addr
        self.command, self.gpus = command, gpus_per_node
        self.env = dict(env or {})

    def pod_spec(self, node: Node) -> Dict:
        res: NodeResource = node.config_resource
        limits = {"amd.com/gpu": str(res.gpu_num or self.gpus)}
        if res.cpu:
            limits["cpu"] = str(res.cpu)
        if res.memory:
            limits["memory"] = f"{res.memory}Mi"
        env = {"DWAMD_MASTER_ADDR": self.master_addr, "NODE_RANK": str(node.rank_index), "NODE_ID": str(node.id),
               "DWAMD_JOB_NAME": self.job_name, "HSA_ENABLE_IPC_MODE_LEGACY": "0", **self.env}
        return {
            "apiVersion": "v1", "kind": "Pod",
            "metadata": {"name": pod_name(self.job_name, node.type, node.id),
                         "labels": {JOB_LABEL: self.job_name, TYPE_LABEL: node.type, ID_LABEL: str(node.id),
                                    RANK_LABEL: str(node.rank_index)}},
            "spec": {"restartPolicy": "Never",
                     "containers": [{"name": "main", "image": self.image, "command": self.command,
                                     "env": [{"name": k, "value": v} for k, v in env.items()],
                                     "resources": {"limits": limits, "requests": dict(limits)},
                                     "volumeMounts": [{"name": "dshm", "mountPath": "/dev/shm"}]}],
                     # flash checkpoints live in /dev/shm: size it for the node's host memory
                     "volumes": [{"name": "dshm", "emptyDir": {"medium": "Memory"}}]},
        }

    def scale(self, plan: ScalePlan):
        for node in plan.launch_nodes:
            logger.info(f"k8s: creating pod for {node.type}-{node.id} (rank {node.rank_index})")
            self.client.create_pod(self.pod_spec(node))
        for node in plan.remove_nodes:
            logger.info(f"k8s: deleting pod {pod_name(self.job_name, node.type, node.id)}")
            self.client.delete_pod(pod_name(self.job_name, node.type, node.id))


class PodWatcher(NodeWatcher):
    def __init__(self, job_name: str, client: K8sClient):
        self.job_name, self.client = job_name, client
        self.selector = f"{JOB_LABEL}={job_name}"

    def list(self) -> List[Node]:
        return [pod_to_node(p) for p in self.client.list_pods(self.selector)]

    def watch(self) -> Iterator[NodeEvent]:
        for ev in self.client.watch_pods(self.selector):
            t = ev.get("type", NodeEventType.MODIFIED)
            yield NodeEvent(t, pod_to_node(ev.get("object", {})))


class ElasticJobScaler(Scaler):
    """Master -> operator: every ScalePlan of the job master becomes a
    ``ScalePlan`` custom object (``createPods`` / ``removePods`` /
    ``replicaResourceSpecs``) that the operator applies (vs ``PodScaler``,
    which creates the pods itself).  Parity: reference
    ``master/scaler/elasticjob_scaler.py``."""

    def __init__(self, job_name: str, client: K8sClient):
        super().__init__(job_name)
        self.client = client
        self._n = 0

    @staticmethod
    def _res(node: Node) -> Dict:
        r: NodeResource = node.config_resource
        out = {}
        if r.gpu_num:
            out["amd.com/gpu"] = str(r.gpu_num)
        if r.cpu:
            out["cpu"] = str(r.cpu)
        if r.memory:
            out["memory"] = f"{r.memory}Mi"
        return out

    def plan_object(self, plan: ScalePlan) -> Dict:
        self._n += 1
        spec: Dict = {"ownerJob": self.job_name, "manualScaling": False}
        if plan.node_group_resources:
            spec["replicaResourceSpecs"] = {
                t: {"replicas": int(g.count),
                    "resource": {k: v for k, v in (("cpu", g.node_resource.cpu),
                                                   ("memory", f"{g.node_resource.memory}Mi"
                                                    if g.node_resource.memory else 0),
                                                   ("amd.com/gpu", g.node_resource.gpu_num)) if v}}
                for t, g in plan.node_group_resources.items()}
        if plan.launch_nodes:
            spec["createPods"] = [{"name": pod_name(self.job_name, n.type, n.id), "type": n.type, "id": n.id,
                                   "rankIndex": n.rank_index, "resource": self._res(n)} for n in plan.launch_nodes]
        if plan.remove_nodes:
            spec["removePods"] = [{"name": pod_name(self.job_name, n.type, n.id), "type": n.type, "id": n.id}
                                  for n in plan.remove_nodes]
        return {"apiVersion": f"{GROUP}/{VERSION}", "kind": "ScalePlan",
                "metadata": {"name": f"{self.job_name}-{int(time.time())}-{self._n}",
                             "labels": {JOB_LABEL: self.job_name, "scale-type": "auto"}},
                "spec": spec}

    def scale(self, plan: ScalePlan):
        if plan is None or plan.empty():
            return
        obj = self.plan_object(plan)
        logger.info(f"k8s: ScalePlan {obj['metadata']['name']} for ElasticJob {self.job_name}")
        self.client.create_custom("scaleplans", obj)


class K8sScalePlanWatcher:
    """Manual scaling: ``ScalePlan`` objects of this job with
    ``spec.manualScaling: true`` become master-side ScalePlans (replica
    counts / resources per node type, explicit pod removals); each is
    consumed once (status ``Succeeded``).  Parity: reference
    ``master/watcher/k8s_watcher.py:267`` (``K8sScalePlanWatcher``)."""

    def __init__(self, job_name: str, client: K8sClient):
        self.job_name, self.client = job_name, client

    @staticmethod
    def _mem_mb(v) -> int:
        s = str(v)
        for suf, mul in (("Gi", 1024), ("Mi", 1), ("G", 1000), ("M", 1)):
            if s.endswith(suf):
                return int(float(s[:-len(suf)]) * mul)
        return int(float(s)) // (1 << 20) if s else 0

    def to_plan(self, obj: Dict) -> ScalePlan:
        from ..common.node import NodeGroupResource

        sp = ScalePlan()
        for t, v in (obj.get("spec", {}).get("replicaResourceSpecs") or {}).items():
            r = v.get("resource") or {}
            sp.node_group_resources[t] = NodeGroupResource(
                int(v.get("replicas", 0)),
                NodeResource(cpu=float(r.get("cpu", 0) or 0), memory=self._mem_mb(r.get("memory", 0) or 0),
                             gpu_num=int(r.get("amd.com/gpu", r.get("gpu", 0)) or 0)))
        for p in obj.get("spec", {}).get("removePods") or []:
            sp.remove_nodes.append(Node(type=p.get("type", NodeType.WORKER), id=int(p.get("id", 0)),
                                        name=p.get("name", "")))
        return sp

    def poll(self) -> List[ScalePlan]:
        out = []
        for obj in self.client.list_custom("scaleplans"):
            spec, st = obj.get("spec", {}), obj.get("status") or {}
            if spec.get("ownerJob") != self.job_name or not spec.get("manualScaling") or st.get("phase") in (
                    "Succeeded", "Failed"):
                continue
            out.append(self.to_plan(obj))
            self.client.patch_custom_status("scaleplans", obj["metadata"]["name"], {"phase": "Succeeded"})
        return out

    def watch(self, interval: float = 5.0, stop: Optional[threading.Event] = None) -> Iterator[ScalePlan]:
        stop = stop or threading.Event()
        while not stop.is_set():
            for p in self.poll():
                yield p
            stop.wait(interval)


# ----------------------------------------------------------------------------- operator


class ElasticJobOperator:
    """Reconciles ``ElasticJob`` and ``ScalePlan`` custom objects (CRDs in
    ``deploy/crds/``).

    * ElasticJob: create the job master pod + service (image/resources from
      ``replicaSpecs["dlrover-master"].template`` when given, ``spec.envs``
      forwarded), mirror the master pod's phase into ``status.phase``, and
      on a terminal phase clean up the job's remaining worker pods;
    * ScalePlan: ``replicaResourceSpecs`` patch the job's replica counts
      (the master scales to them); ``createPods`` / ``removePods`` /
      ``migratePods`` create pods from the job's per-type pod template and
      delete the named ones (migration: the new pod first, then the old).

    Parity: reference Go operator ``go/operator/pkg/controllers``
    (ElasticJob + ScalePlan reconcilers, master pod/service creation).
    """

    def __init__(self, client: K8sClient, master_image: str, master_port: int = 50001):
        self.client, self.image, self.port = client, master_image, master_port
        self._stop = threading.Event()

    @staticmethod
    def _envs(job: Dict) -> List[Dict]:
        envs = (job.get("spec") or {}).get("envs") or {}
        return [{"name": k, "value": str(v)} for k, v in envs.items()]

    def master_pod(self, job: Dict) -> Dict:
        name = job["metadata"]["name"]
        spec = job.get("spec", {})
        rs = spec.get("replicaSpecs", {})
        workers = rs.get("worker", {}).get("replicas", 1)
        cmd = ["python", "-m", "dlrover_wuqiong_amd.master.master", "--platform", "k8s", "--job_name", name,
               "--namespace", self.client.ns, "--port", str(self.port), "--node_num", str(workers)]
        container = {"name": "master", "image": self.image, "command": cmd,
                     "ports": [{"containerPort": self.port}], "env": self._envs(job)}
        tmpl = ((rs.get("dlrover-master") or {}).get("template") or {}).get("spec") or {}
        tc = (tmpl.get("containers") or [{}])[0]
        for k in ("image", "resources", "volumeMounts", "imagePullPolicy"):
            if k in tc:
                container[k] = tc[k]
        pod_spec = {"restartPolicy": "Never", "containers": [container]}
        for k in ("volumes", "nodeSelector", "tolerations", "priorityClassName", "serviceAccountName"):
            if k in tmpl:
                pod_spec[k] = tmpl[k]
        return {"apiVersion": "v1", "kind": "Pod",
                "metadata": {"name": f"elasticjob-{name}-dlrover-master",
                             "labels": {JOB_LABEL: name, TYPE_LABEL: NodeType.MASTER},
                             "ownerReferences": [{"apiVersion": f"{GROUP}/{VERSION}", "kind": "ElasticJob",
                                                  "name": name, "uid": job["metadata"].get("uid", "")}]},
                "spec": pod_spec}

    def master_service(self, job: Dict) -> Dict:
        name = job["metadata"]["name"]
        return {"apiVersion": "v1", "kind": "Service",
                "metadata": {"name": f"elasticjob-{name}-dlrover-master", "labels": {JOB_LABEL: name}},
                "spec": {"selector": {JOB_LABEL: name, TYPE_LABEL: NodeType.MASTER},
                         "ports": [{"port": self.port, "targetPort": self.port}]}}

    def replica_pod(self, job: Dict, node_type: str, node_id: int, rank: int, resource: Optional[Dict] = None,
                    name: Optional[str] = None) -> Dict:
        """A worker (or other replica type) pod from the job's pod template."""
        import copy

        jname = job["metadata"]["name"]
        tmpl = copy.deepcopy(((job.get("spec", {}).get("replicaSpecs", {}).get(node_type) or {})
                              .get("template") or {}))
        spec = tmpl.get("spec") or {"containers": [{"name": "main", "image": self.image}]}
        spec.setdefault("restartPolicy", "Never")
        c = spec["containers"][0]
        env = [e for e in c.get("env", []) if e.get("name") not in ("DWAMD_MASTER_ADDR", "NODE_RANK", "NODE_ID")]
        env += [{"name": "DWAMD_MASTER_ADDR", "value": f"elasticjob-{jname}-dlrover-master:{self.port}"},
                {"name": "NODE_RANK", "value": str(rank)}, {"name": "NODE_ID", "value": str(node_id)},
                {"name": "DWAMD_JOB_NAME", "value": jname}] + self._envs(job)
        c["env"] = env
        if resource:
            lim = dict((c.get("resources") or {}).get("limits") or {})
            for k, v in resource.items():
                lim[{"gpu": "amd.com/gpu"}.get(k, k)] = str(v)
            c["resources"] = {"limits": lim, "requests": dict(lim)}
        meta = tmpl.get("metadata") or {}
        labels = dict(meta.get("labels") or {})
        labels.update({JOB_LABEL: jname, TYPE_LABEL: node_type, ID_LABEL: str(node_id), RANK_LABEL: str(rank)})
        return {"apiVersion": "v1", "kind": "Pod",
                "metadata": {"name": name or pod_name(jname, node_type, node_id), "labels": labels,
                             "ownerReferences": [{"apiVersion": f"{GROUP}/{VERSION}", "kind": "ElasticJob",
                                                  "name": jname, "uid": job["metadata"].get("uid", "")}]},
                "spec": spec}

    def reconcile_job(self, job: Dict):
        name = job["metadata"]["name"]
        mname = f"elasticjob-{name}-dlrover-master"
        pod = self.client.get_pod(mname)
        phase = (job.get("status") or {}).get("phase", "")
        if pod is None:
            if phase in ("Succeeded", "Failed"):
                return
            logger.info(f"operator: creating master of ElasticJob {name}")
            self.client.create_pod(self.master_pod(job))
            if self.client.get_service(mname) is None:
                self.client.create_service(self.master_service(job))
            self.client.patch_custom_status("elasticjobs", name, {"phase": "Pending"})
            return
        pphase = (pod.get("status") or {}).get("phase", "Pending")
        new = {"Pending": "Pending", "Running": "Running", "Succeeded": "Succeeded", "Failed": "Failed"}.get(pphase)
        if new and new != phase:
            st = {"phase": new}
            if new in ("Succeeded", "Failed"):
                import datetime

                st["completionTime"] = datetime.datetime.now(datetime.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")
                # the job is over: its workers must not keep the GPUs
                for p in self.client.list_pods(f"{JOB_LABEL}={name}"):
                    if p["metadata"]["name"] != mname:
                        self.client.delete_pod(p["metadata"]["name"])
            elif new == "Running" and not (job.get("status") or {}).get("startTime"):
                import datetime

                st["startTime"] = datetime.datetime.now(datetime.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")
            self.client.patch_custom_status("elasticjobs", name, st)

    def reconcile_scaleplan(self, plan: Dict):
        st = plan.get("status") or {}
        if st.get("phase") in ("Succeeded", "Failed"):
            return
        spec = plan.get("spec", {})
        jname = spec.get("ownerJob")
        job = self.client.get_custom("elasticjobs", jname) if jname else None
        if job is None:
            logger.warning(f"operator: ScalePlan {plan['metadata']['name']} names unknown job {jname}")
            self.client.patch_custom_status("scaleplans", plan["metadata"]["name"], {"phase": "Failed"})
            return
        rs = spec.get("replicaResourceSpecs", {})
        if rs:
            patch = {"spec": {"replicaSpecs": {t: {"replicas": int(v.get("replicas", 0))} for t, v in rs.items()}}}
            self.client.patch_custom("elasticjobs", jname, patch)
        pname = plan["metadata"]["name"]
        creates = [(item, item.get("name")) for item in spec.get("createPods") or []]
        # migration: the replacement (fresh name) is created before the old pod goes
        creates += [(item, f"{pod_name(jname, item.get('type', NodeType.WORKER), int(item.get('id', 0)))}"
                           f"-mig-{pname}"[:63]) for item in spec.get("migratePods") or []]
        for item, new_name in creates:
            t, i = item.get("type", NodeType.WORKER), int(item.get("id", 0))
            pod = self.replica_pod(job, t, i, int(item.get("rankIndex", i)), item.get("resource"), new_name)
            if self.client.get_pod(pod["metadata"]["name"]) is None:
                self.client.create_pod(pod)
        for item in (spec.get("removePods") or []) + (spec.get("migratePods") or []):
            n = item.get("name") or pod_name(jname, item.get("type", NodeType.WORKER), int(item.get("id", 0)))
            if self.client.get_pod(n) is not None:
                self.client.delete_pod(n)
        self.client.patch_custom_status("scaleplans", plan["metadata"]["name"], {"phase": "Succeeded"})

    def reconcile_once(self):
        for job in self.client.list_custom("elasticjobs"):
            self.reconcile_job(job)
        for plan in self.client.list_custom("scaleplans"):
            self.reconcile_scaleplan(plan)

    def run(self, interval: float = 5.0):
        while not self._stop.is_set():
            try:
                self.reconcile_once()
            except Exception as e:  # keep reconciling through API hiccups
                logger.warning(f"operator reconcile failed: {e}")
            self._stop.wait(interval)

    def stop(self):
        self._stop.set()


def main(argv=None):
    import argparse

    p = argparse.ArgumentParser("dwamd-operator")
    p.add_argument("--namespace", default="default")
    p.add_argument("--master-image", required=True)
    p.add_argument("--interval", type=float, default=5.0)
    a = p.parse_args(argv)
    ElasticJobOperator(K8sClient(a.namespace), a.master_image).run(a.interval)


if __name__ == "__main__":
    main()
