"""Brain cluster side (brain/k8s_monitor.py) against the in-process fake API
server: ElasticJobs and their pods are recorded into the job / job_node
tables, an OOMKilled pod becomes an oom metric, and the optimizer's
creation-OOM plan for the re-submitted job uses it (parity: reference
go/brain cmd/k8smonitor + watchhandler + mysql recorders)."""

import pytest

from test_k8s_platform import k8s  # noqa: F401  (fixture)


def test_monitor_records_jobs_nodes_and_ooms(k8s):  # noqa: F811
    from dlrover_wuqiong_amd.brain.k8s_monitor import K8sMonitor
    from dlrover_wuqiong_amd.brain.service import BrainDatastore, BrainOptimizer

    fake, client = k8s
    client.create_custom("elasticjobs", {"apiVersion": "elastic.iml.github.io/v1alpha1", "kind": "ElasticJob",
                                         "metadata": {"name": "gpt", "uid": "u-gpt",
                                                      "creationTimestamp": "2026-10-17T01:00:00Z",
                                                      "labels": {"scenario": "llm"}},
                                         "status": {"phase": "Running", "startTime": "2026-10-17T01:00:05Z"}})
    for i, (phase, reason) in enumerate([("Running", ""), ("Failed", "OOMKilled")]):
        client.create_pod({"metadata": {"name": f"gpt-worker-{i}", "uid": f"p{i}",
                                        "labels": {"elasticjob-name": "gpt", "replica-type": "worker"}},
                           "spec": {"containers": [{"name": "main", "resources": {"requests": {
                               "cpu": "16", "memory": "64Gi", "amd.com/gpu": "8"}}}]}})
        fake.objs[("pods", f"gpt-worker-{i}")]["status"] = {
            "phase": phase, "containerStatuses": [{"state": {"terminated": {"reason": reason}}}] if reason else []}
    client.create_pod({"metadata": {"name": "unrelated", "labels": {"app": "x"}}, "spec": {"containers": []}})
    store = BrainDatastore()
    mon = K8sMonitor(client, store)
    mon.sync_once()
    mon.sync_once()  # idempotent upserts
    jobs = mon.recorder.jobs("gpt")
    assert len(jobs) == 1 and jobs[0]["uid"] == "u-gpt" and jobs[0]["status"] == "Running"
    assert jobs[0]["scenario"] == "llm" and jobs[0]["created_at"] is not None
    nodes = {n["name"]: n for n in mon.recorder.nodes("gpt")}
    assert set(nodes) == {"gpt-worker-0", "gpt-worker-1"}
    assert nodes["gpt-worker-0"]["resource"] == {"cpu": 16.0, "memory_mb": 65536, "gpu": 8}
    assert nodes["gpt-worker-1"]["exit_reason"] == "OOMKilled" and nodes["gpt-worker-1"]["finished_at"]
    ooms = store.query(job_name="gpt", metrics_type="oom")
    assert len(ooms) == 1 and ooms[0]["metrics"]["memory_mb"] == 65536  # recorded once
    # the pod is deleted (watch event): the node keeps its history, marked finished
    client.delete_pod("gpt-worker-0")
    mon.watch_pods_once(timeout_s=1)
    assert {n["name"]: n for n in mon.recorder.nodes("gpt")}["gpt-worker-0"]["finished_at"] is not None
    plan = BrainOptimizer(store).optimize({"opt_type": "job_worker_create_oom_resource", "job_name": "gpt",
                                           "job_uuid": "u-gpt2"})
    assert plan.get("memory_mb", plan.get("worker", {}).get("memory_mb", 0)) > 65536, plan
