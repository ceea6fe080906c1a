"""Kubernetes platform layer against an in-process fake API server: pod
scaler / watcher and the ElasticJob operator reconcile loop.
Parity: reference dlrover/python/tests/test_k8s_*.py (mocked k8s client) and
the Go operator's controller tests."""

import json
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from urllib.parse import parse_qs, urlparse

import pytest


class FakeK8s:
    def __init__(self):
        self.objs = {}  # (kind-path, name) -> obj
        self.events = []

    def handler(self):
        store = self

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def _send(self, code, obj=None):
                body = json.dumps(obj if obj is not None else {}).encode()
                self.send_response(code)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def _split(self):
                u = urlparse(self.path)
                parts = u.path.strip("/").split("/")
                q = parse_qs(u.query)
                status = parts[-1] == "status"
                if status:
                    parts = parts[:-1]
                # .../namespaces/{ns}/{plural}[/{name}]
                i = parts.index("namespaces") if "namespaces" in parts else None
                if i is None:  # cluster-scoped: /api/v1/nodes/{name}
                    return parts[-2], parts[-1], q, status
                plural = parts[i + 2]
                name = parts[i + 3] if len(parts) > i + 3 else ""
                return plural, name, q, status

            def _body(self):
                n = int(self.headers.get("Content-Length", 0))
                return json.loads(self.rfile.read(n)) if n else {}

            def do_GET(self):
                plural, name, q, _ = self._split()
                if name:
                    o = store.objs.get((plural, name))
                    return self._send(200, o) if o else self._send(404, {"reason": "NotFound"})
                items = [o for (p, _n), o in store.objs.items() if p == plural]
                sel = q.get("labelSelector", [""])[0]
                if sel:
                    k, v = sel.split("=")
                    items = [o for o in items if o["metadata"].get("labels", {}).get(k) == v]
                if q.get("watch"):
                    body = "".join(json.dumps(e) + "\n" for e in store.events).encode()
                    self.send_response(200)
                    self.send_header("Content-Length", str(len(body)))
                    self.end_headers()
                    self.wfile.write(body)
                    return
                return self._send(200, {"items": items})

            def do_POST(self):
                plural, _, _, _ = self._split()
                o = self._body()
                o.setdefault("status", {"phase": "Pending"} if plural == "pods" else {})
                store.objs[(plural, o["metadata"]["name"])] = o
                store.events.append({"type": "ADDED", "object": o})
                return self._send(201, o)

            def do_DELETE(self):
                plural, name, _, _ = self._split()
                o = store.objs.pop((plural, name), None)
                if o is None:
                    return self._send(404)
                store.events.append({"type": "DELETED", "object": o})
                return self._send(200, o)

            def do_PATCH(self):
                plural, name, _, status = self._split()
                o = store.objs.get((plural, name))
                if o is None:
                    return self._send(404)
                patch = self._body()

                def merge(a, b):
                    for k, v in b.items():
                        if isinstance(v, dict) and isinstance(a.get(k), dict):
                            merge(a[k], v)
                        else:
                            a[k] = v
                merge(o, patch)
                return self._send(200, o)

        return H


@pytest.fixture()
def k8s():
    fake = FakeK8s()
    srv = ThreadingHTTPServer(("127.0.0.1", 0), fake.handler())
    t = threading.Thread(target=srv.serve_forever, daemon=True)
    t.start()
    from dlrover_wuqiong_amd.platform.k8s import K8sClient

    yield fake, K8sClient("ns1", base_url=f"http://127.0.0.1:{srv.server_port}", token="t")
    srv.shutdown()


def test_pod_scaler_and_watcher(k8s):
    from dlrover_wuqiong_amd.common.node import Node
    from dlrover_wuqiong_amd.master.scaler import ScalePlan
    from dlrover_wuqiong_amd.platform.k8s import PodScaler, PodWatcher, pod_to_node

    fake, cli = k8s
    sc = PodScaler("job1", cli, "img:1", "job1-master:50001", ["dwamd-run", "train.py"], gpus_per_node=8)
    sc.scale(ScalePlan(launch_nodes=[Node(id=i, rank_index=i) for i in range(3)]))
    pods = cli.list_pods("elasticjob.dlrover/name=job1")
    assert sorted(p["metadata"]["name"] for p in pods) == ["job1-worker-0", "job1-worker-1", "job1-worker-2"]
    c = pods[0]["spec"]["containers"][0]
    assert c["resources"]["limits"]["amd.com/gpu"] == "8"
    assert {"name": "DWAMD_MASTER_ADDR", "value": "job1-master:50001"} in c["env"]
    w = PodWatcher("job1", cli)
    assert len(w.list()) == 3
    # a pod OOMKilled -> node exit reason
    fake.objs[("pods", "job1-worker-1")]["status"] = {
        "phase": "Failed", "containerStatuses": [{"state": {"terminated": {"reason": "OOMKilled", "exitCode": 137}}}]}
    n = pod_to_node(cli.get_pod("job1-worker-1"))
    assert n.status == "Failed" and n.exit_reason == "OOMKilled" and n.rank_index == 1
    sc.scale(ScalePlan(remove_nodes=[Node(id=2)]))
    assert len(w.list()) == 2
    evs = list(w.watch())
    assert [e.event_type for e in evs].count("ADDED") == 3 and evs[-1].event_type == "DELETED"
    cli.cordon_node("host-a") if ("nodes", "host-a") in fake.objs else None


def test_elasticjob_operator_reconcile(k8s):
    from dlrover_wuqiong_amd.platform.k8s import ElasticJobOperator

    fake, cli = k8s
    cli.create_custom("elasticjobs", {"apiVersion": "elastic.iml.github.io/v1alpha1", "kind": "ElasticJob",
                                      "metadata": {"name": "llama", "uid": "u1"},
                                      "spec": {"replicaSpecs": {"worker": {"replicas": 4}}}})
    op = ElasticJobOperator(cli, "img:1")
    op.reconcile_once()
    pod = cli.get_pod("elasticjob-llama-dlrover-master")
    assert pod is not None and "--node_num" in pod["spec"]["containers"][0]["command"]
    assert cli.get_service("elasticjob-llama-dlrover-master") is not None
    assert cli.get_custom("elasticjobs", "llama")["status"]["phase"] == "Pending"
    fake.objs[("pods", "elasticjob-llama-dlrover-master")]["status"]["phase"] = "Running"
    op.reconcile_once()
    assert cli.get_custom("elasticjobs", "llama")["status"]["phase"] == "Running"
    cli.create_custom("scaleplans", {"metadata": {"name": "sp1"},
                                     "spec": {"ownerJob": "llama", "replicaResourceSpecs": {"worker": {"replicas": 8}}}})
    op.reconcile_once()
    assert cli.get_custom("elasticjobs", "llama")["spec"]["replicaSpecs"]["worker"]["replicas"] == 8
    assert cli.get_custom("scaleplans", "sp1")["status"]["phase"] == "Succeeded"
    n_pods = len([k for k in fake.objs if k[0] == "pods"])
    op.reconcile_once()  # idempotent
    assert len([k for k in fake.objs if k[0] == "pods"]) == n_pods


def test_operator_scaleplan_pods_master_template_and_cleanup(k8s):
    from dlrover_wuqiong_amd.platform.k8s import ElasticJobOperator

    fake, cli = k8s
    tmpl = {"spec": {"containers": [{"name": "main", "image": "train:1", "command": ["dwamd-run", "t.py"],
                                     "resources": {"limits": {"amd.com/gpu": 8}}}]}}
    cli.create_custom("elasticjobs", {"metadata": {"name": "j2", "uid": "u2"},
                                      "spec": {"envs": {"FOO": "1"},
                                               "replicaSpecs": {"worker": {"replicas": 2, "template": tmpl},
                                                                "dlrover-master": {"template": {"spec": {
                                                                    "containers": [{"image": "master:2"}],
                                                                    "nodeSelector": {"pool": "cpu"}}}}}}})
    op = ElasticJobOperator(cli, "img:1")
    op.reconcile_once()
    mp = cli.get_pod("elasticjob-j2-dlrover-master")
    assert mp["spec"]["containers"][0]["image"] == "master:2" and mp["spec"]["nodeSelector"] == {"pool": "cpu"}
    assert {"name": "FOO", "value": "1"} in mp["spec"]["containers"][0]["env"]
    cli.create_custom("scaleplans", {"metadata": {"name": "sp2"},
                                     "spec": {"ownerJob": "j2", "manualScaling": True,
                                              "createPods": [{"type": "worker", "id": 5, "rankIndex": 1,
                                                              "resource": {"gpu": 4}}]}})
    op.reconcile_once()
    w = cli.get_pod("j2-worker-5")
    c = w["spec"]["containers"][0]
    assert c["image"] == "train:1" and c["resources"]["limits"]["amd.com/gpu"] == "4"
    assert {"name": "NODE_RANK", "value": "1"} in c["env"] and w["metadata"]["labels"]["elasticjob.dlrover/name"] == "j2"
    cli.create_custom("scaleplans", {"metadata": {"name": "sp3"},
                                     "spec": {"ownerJob": "j2", "migratePods": [{"type": "worker", "id": 5}]}})
    op.reconcile_once()
    assert cli.get_pod("j2-worker-5") is None and cli.get_pod("j2-worker-5-mig-sp3") is not None
    cli.create_custom("scaleplans", {"metadata": {"name": "sp4"},
                                     "spec": {"ownerJob": "j2", "removePods": [{"name": "j2-worker-5-mig-sp3"}]}})
    op.reconcile_once()
    assert cli.get_pod("j2-worker-5-mig-sp3") is None
    cli.create_custom("scaleplans", {"metadata": {"name": "bad"}, "spec": {"ownerJob": "nope"}})
    op.reconcile_once()
    assert cli.get_custom("scaleplans", "bad")["status"]["phase"] == "Failed"
    # master finished -> status + remaining workers cleaned up
    cli.create_pod(op.replica_pod(cli.get_custom("elasticjobs", "j2"), "worker", 0, 0))
    fake.objs[("pods", "elasticjob-j2-dlrover-master")]["status"]["phase"] = "Succeeded"
    op.reconcile_once()
    st = cli.get_custom("elasticjobs", "j2")["status"]
    assert st["phase"] == "Succeeded" and st["completionTime"]
    assert cli.get_pod("j2-worker-0") is None


def test_deploy_manifests():
    import os

    import yaml

    root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "deploy")
    docs = {}
    for dirpath, _d, files in os.walk(root):
        for f in files:
            with open(os.path.join(dirpath, f)) as fh:
                docs[f] = [d for d in yaml.safe_load_all(fh) if d]
    ej = docs["elastic.iml.github.io_elasticjobs.yaml"][0]
    sp = docs["elastic.iml.github.io_scaleplans.yaml"][0]
    from dlrover_wuqiong_amd.platform.k8s import GROUP, VERSION

    for crd, plural in ((ej, "elasticjobs"), (sp, "scaleplans")):
        assert crd["kind"] == "CustomResourceDefinition" and crd["spec"]["group"] == GROUP
        assert crd["metadata"]["name"] == f"{plural}.{GROUP}" and crd["spec"]["names"]["plural"] == plural
        v = crd["spec"]["versions"][0]
        assert v["name"] == VERSION and "status" in v["subresources"]
    # every spec field the operator reads is in the schema
    ejs = ej["spec"]["versions"][0]["schema"]["openAPIV3Schema"]["properties"]["spec"]["properties"]
    assert {"replicaSpecs", "envs"} <= set(ejs)
    assert "template" in ejs["replicaSpecs"]["additionalProperties"]["properties"]
    sps = sp["spec"]["versions"][0]["schema"]["openAPIV3Schema"]["properties"]["spec"]["properties"]
    assert {"ownerJob", "replicaResourceSpecs", "createPods", "removePods", "migratePods"} <= set(sps)
    kinds = [d["kind"] for d in docs["operator.yaml"]]
    assert kinds == ["ServiceAccount", "ClusterRole", "ClusterRoleBinding", "Deployment"]
    ex = docs["llama3_8b_fsdp_mi355x.yaml"][0]
    assert ex["apiVersion"] == f"{GROUP}/{VERSION}" and ex["kind"] == "ElasticJob"
    limits = ex["spec"]["replicaSpecs"]["worker"]["template"]["spec"]["containers"][0]["resources"]["limits"]
    assert limits["amd.com/gpu"] == 8


def test_elasticjob_scaler_to_operator_and_manual_scaleplan_watcher(k8s):
    from dlrover_wuqiong_amd.common.node import Node, NodeGroupResource, NodeResource
    from dlrover_wuqiong_amd.master.scaler import ScalePlan
    from dlrover_wuqiong_amd.platform.k8s import ElasticJobOperator, ElasticJobScaler, K8sScalePlanWatcher

    fake, cli = k8s
    tmpl = {"spec": {"containers": [{"name": "main", "image": "train:1"}]}}
    cli.create_custom("elasticjobs", {"metadata": {"name": "j3"},
                                      "spec": {"replicaSpecs": {"worker": {"replicas": 1, "template": tmpl}}}})
    sc = ElasticJobScaler("j3", cli)
    n = Node(id=4, rank_index=2)
    n.config_resource = NodeResource(gpu_num=8, memory=1024)
    sc.scale(ScalePlan(launch_nodes=[n], node_group_resources={"worker": NodeGroupResource(3, NodeResource(gpu_num=8))}))
    plans = cli.list_custom("scaleplans")
    assert len(plans) == 1 and plans[0]["spec"]["createPods"][0]["rankIndex"] == 2
    assert plans[0]["spec"]["replicaResourceSpecs"]["worker"]["replicas"] == 3
    ElasticJobOperator(cli, "img").reconcile_once()
    pod = cli.get_pod("j3-worker-4")
    assert pod is not None and pod["spec"]["containers"][0]["resources"]["limits"]["amd.com/gpu"] == "8"
    # a manual plan by the user -> a master-side ScalePlan, consumed once
    cli.create_custom("scaleplans", {"metadata": {"name": "manual-1"},
                                     "spec": {"ownerJob": "j3", "manualScaling": True,
                                              "replicaResourceSpecs": {"worker": {"replicas": 5, "resource": {
                                                  "memory": "64Gi", "amd.com/gpu": 8}}},
                                              "removePods": [{"type": "worker", "id": 1}]}})
    w = K8sScalePlanWatcher("j3", cli)
    got = w.poll()
    assert len(got) == 1 and got[0].node_group_resources["worker"].count == 5
    assert got[0].node_group_resources["worker"].node_resource.memory == 65536 and got[0].remove_nodes[0].id == 1
    assert w.poll() == []


def test_dist_job_manager_applies_manual_plan():
    from dlrover_wuqiong_amd.common.constants import NodeStatus
    from dlrover_wuqiong_amd.common.node import JobResource, Node, NodeGroupResource, NodeResource
    from dlrover_wuqiong_amd.master.dist_job_manager import DistributedJobManager
    from dlrover_wuqiong_amd.master.scaler import ScalePlan, Scaler
    from dlrover_wuqiong_amd.master.watcher import NodeWatcher

    class Rec(Scaler):
        def __init__(self):
            super().__init__("j")
            self.plans = []

        def scale(self, plan):
            self.plans.append(plan)

    class W(NodeWatcher):
        def list(self):
            return []

        def watch(self):
            return iter(())

    jr = JobResource()
    jr.node_group_resources["worker"] = NodeGroupResource(2, NodeResource(gpu_num=8))
    rec = Rec()
    jm = DistributedJobManager(jr, rec, W())
    for n in jm.nodes.values():
        n.status = NodeStatus.RUNNING
    out = jm.apply_scale_plan(ScalePlan(node_group_resources={"worker": NodeGroupResource(4, NodeResource())}))
    assert len(out.launch_nodes) == 2 and rec.plans
    out = jm.apply_scale_plan(ScalePlan(remove_nodes=[Node(id=0)]))
    assert [n.id for n in out.remove_nodes] == [0]
