"""Control plane: the Rancher-style environment/registration API the roles call
(ranchermaster/tasks/main.yml:29-52, rancherhost/tasks/main.yml:11-34), node leases,
the amd.com/gpu scheduler and the DaemonSet / Job / Deployment controllers."""
import json
import subprocess
import sys
import time
from pathlib import Path

import pytest

from tritonk8ssupervisor_amd.controlplane.client import ApiError, Client, client_from_kubeconfig

REPO = Path(__file__).resolve().parents[1]
GPU = "amd.com/gpu"


def _start(tmp_path, grace=0.6, state_dir=None):
    ready = tmp_path / f"ready-{time.monotonic_ns()}.json"
    argv = [sys.executable, "-m", "tritonk8ssupervisor_amd.controlplane", "--host", "127.0.0.1", "--port", "0",
            "--node-grace", str(grace), "--ready-file", str(ready)]
    if state_dir:
        argv += ["--state-dir", str(state_dir)]
    from conftest import die_with_parent

    p = subprocess.Popen(argv, cwd=REPO, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, preexec_fn=die_with_parent())
    deadline = time.monotonic() + 30
    while not ready.exists():
        assert p.poll() is None, p.stdout.read().decode()
        assert time.monotonic() < deadline
        time.sleep(0.01)
    info = json.loads(ready.read_text())
    # the server admin token (controlplane/authn.py): what the roles read from the master
    return p, Client(info["base"], token=info["adminToken"], timeout=10)


def _stop(p):
    p.terminate()
    try:
        p.wait(10)
    except subprocess.TimeoutExpired:
        p.kill()


@pytest.fixture
def cp(tmp_path):
    p, c = _start(tmp_path)
    yield c
    _stop(p)


def _env(c, name="k8s dev"):
    tmpl = c.get("/v2-beta/projectTemplates", query={"name": "kubernetes"})
    body = {"description": name, "name": name, "projectTemplateId": tmpl["data"][0]["id"], "allowSystemRole": False,
            "members": [], "virtualMachine": False, "servicesPortRange": None, "projectLinks": []}
    proj = c.post("/v2-beta/projects", body)
    return proj


def _join(c, pid, name, ngpu=1, validated=True):
    tok = c.post("/v1/registrationtokens", query={"projectId": pid})
    url = c.get(tok["links"]["self"].split(c.base, 1)[1])["registrationUrl"]
    path = url.split(c.base, 1)[1]
    boot = c.get(path)
    assert boot["projectId"] == pid
    devs = [{"id": f"gpu{i}", "health": "Healthy"} for i in range(ngpu)]
    reg = c.post(path, {"name": name, "ip": "127.0.0.1", "devices": devs, "capacity": {"cpu": "8"}})
    nc = Client(c.base, token=reg["nodeToken"], prefix=reg["apiPrefix"])
    return nc, reg


def _heartbeat(nc, name):
    return nc.put(nc.k8s(f"/api/v1/nodes/{name}/status"), {})


def _set_pod(nc, ns, pod, phase, result=None):
    st = {"phase": phase}
    if result is not None:
        st["result"] = result
    return nc.put(nc.k8s(f"/api/v1/namespaces/{ns}/pods/{pod}/status"), {"status": st})


def test_environment_and_registration_flow(cp):
    # exactly the calls of ranchermaster (29-49) and rancherhost (11-24): 201s and links.self
    tmpl = cp.get("/v2-beta/projectTemplates", query={"name": "kubernetes"})
    assert tmpl["data"][0]["name"] == "kubernetes"
    proj = _env(cp)
    assert proj["id"] and proj["name"] == "k8s dev"
    with pytest.raises(ApiError) as ei:
        cp.post("/v1/registrationtokens", query={"projectId": "nope"})
    assert ei.value.status == 404
    nc, reg = _join(cp, proj["id"], "kubenode1", ngpu=2)
    kc = cp.get(f"/env/{proj['id']}/kubernetes/kubectl", query={"format": "json"})
    k = client_from_kubeconfig(kc)
    n = k.get(k.k8s("/api/v1/nodes/kubenode1"))
    assert n["status"]["capacity"][GPU] == "2" and n["status"]["allocatable"][GPU] == "2"
    assert n["metadata"]["labels"]["amd.com/gpu.family"] == "gfx950"
    conds = {c["type"]: c["status"] for c in n["status"]["conditions"]}
    assert conds["Ready"] == "True" and conds["AMDGPUValidated"] == "Unknown"
    with pytest.raises(ApiError):
        cp.post(reg["apiPrefix"].replace("/kubernetes", "") + "/bad")  # unknown route
    with pytest.raises(ApiError) as ei:
        cp.get("/v1/scripts/not-a-token")
    assert ei.value.status == 403


def test_dashboard_is_the_readiness_oracle(cp):
    proj = _env(cp)
    with pytest.raises(ApiError) as ei:  # setup.sh:66-68: "Service Unavailable" until a node is up
        cp.get(f"/r/projects/{proj['id']}/kubernetes-dashboard:9090/", raw=True)
    assert ei.value.status == 503
    _join(cp, proj["id"], "kubenode1", ngpu=0)
    body = cp.get(f"/r/projects/{proj['id']}/kubernetes-dashboard:9090/", raw=True)
    assert "kubernetes" in body and "kubenode1" in body


def test_writes_need_the_project_token(cp):
    proj = _env(cp)
    pod = {"metadata": {"name": "p"}, "spec": {"containers": [{"name": "c", "command": ["true"]}]}}
    with pytest.raises(ApiError) as ei:
        Client(cp.base).post(f"/r/projects/{proj['id']}/kubernetes/api/v1/namespaces/default/pods", pod)
    assert ei.value.status == 401
    k = client_from_kubeconfig(cp.get(f"/env/{proj['id']}/kubernetes/kubectl", query={"format": "json"}))
    assert k.post(k.k8s("/api/v1/namespaces/default/pods"), pod)["metadata"]["name"] == "p"
    with pytest.raises(ApiError) as ei:
        k.post(k.k8s("/api/v1/namespaces/default/pods"), pod)
    assert ei.value.status == 409


def test_only_the_bound_node_writes_agent_annotations(cp):
    """A pod's agent-owned annotations (tk8s.amd.com/gpu-devices: which GPUs a gpu-peers rank may
    open) arrive with its status, from the node it is bound to: not through the pod API, and not
    on an unbound pod's status from anyone else."""
    proj = _env(cp)
    k = client_from_kubeconfig(cp.get(f"/env/{proj['id']}/kubernetes/kubectl", query={"format": "json"}))
    k.post(k.k8s("/api/v1/namespaces/default/pods"),
           {"metadata": {"name": "u"}, "spec": {"nodeSelector": {"none": "x"}, "containers": [{"name": "c", "command": ["true"]}]}})
    forged = {"status": {"phase": "Pending"}, "annotations": {"tk8s.amd.com/gpu-devices": '[{"renderMinor": 129}]'}}
    with pytest.raises(ApiError) as ei:
        k.put(k.k8s("/api/v1/namespaces/default/pods/u/status"), forged)
    assert ei.value.status == 403
    with pytest.raises(ApiError) as ei:
        k.request("PATCH", k.k8s("/api/v1/namespaces/default/pods/u"), {"metadata": {"annotations": forged["annotations"]}},
                  content_type="application/merge-patch+json")
    assert ei.value.status == 403
    assert "tk8s.amd.com/gpu-devices" not in (k.get(k.k8s("/api/v1/namespaces/default/pods/u"))["metadata"].get(
        "annotations") or {})


def test_workload_templates_cannot_carry_node_or_scheduler_records(cp):
    """the controllers copy a template's annotations into the pods they create, so a
    Job (or any workload) template naming another tenant's GPU in gpu-devices -- or the
    scheduler's host-claims -- is refused at admission, for every workload kind."""
    proj = _env(cp)
    k = client_from_kubeconfig(cp.get(f"/env/{proj['id']}/kubernetes/kubectl", query={"format": "json"}))
    forged = [{"node": "kubenode1", "id": "gpu7", "ordinal": 7, "renderMinor": 135}]
    tmpl = {"metadata": {"labels": {"a": "f"}, "annotations": {"tk8s.amd.com/gpu-peers": "job",
                                                              "tk8s.amd.com/gpu-devices": json.dumps(forged)}},
            "spec": {"restartPolicy": "Never", "containers": [{"name": "c", "command": ["true"]}]}}
    job = {"apiVersion": "batch/v1", "kind": "Job", "metadata": {"name": "forge"},
           "spec": {"completions": 2, "parallelism": 2, "completionMode": "Indexed", "template": tmpl}}
    with pytest.raises(ApiError) as ei:
        k.post(k.k8s("/apis/batch/v1/namespaces/default/jobs"), job)
    assert ei.value.status == 403 and "gpu-devices" in str(ei.value)
    for key, val in (("amd.com/gpu-ids", "gpu7"), ("tk8s.amd.com/host-claims", "{}"), ("tk8s.amd.com/host-devices", "[]")):
        dep = {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": "d"}, "spec": {
            "replicas": 1, "selector": {"matchLabels": {"a": "d"}},
            "template": {"metadata": {"labels": {"a": "d"}, "annotations": {key: val}},
                         "spec": {"containers": [{"name": "c", "command": ["true"]}]}}}}
        with pytest.raises(ApiError) as ei:
            k.post(k.k8s("/apis/apps/v1/namespaces/default/deployments"), dep)
        assert ei.value.status == 403 and key in str(ei.value)
    cj = {"apiVersion": "batch/v1", "kind": "CronJob", "metadata": {"name": "cj"}, "spec": {
        "schedule": "* * * * *", "jobTemplate": {"spec": {"completionMode": "Indexed", "completions": 1, "template": tmpl}}}}
    with pytest.raises(ApiError) as ei:
        k.post(k.k8s("/apis/batch/v1/namespaces/default/cronjobs"), cj)
    assert ei.value.status == 403
    # and a pod the Job controller makes never inherits one (controllers._new_pod strips them)
    from tritonk8ssupervisor_amd.controlplane.objects import strip_owned

    assert strip_owned({"tk8s.amd.com/gpu-devices": "[]", "amd.com/gpu-ids": "gpu1", "tk8s.amd.com/host-claims": "{}",
                        "tk8s.amd.com/gpu-peers": "job", "x": "y"}) == {"tk8s.amd.com/gpu-peers": "job", "x": "y"}


def test_node_lease_expiry_and_recovery(cp):
    proj = _env(cp)
    nc, _ = _join(cp, proj["id"], "kubenode1", ngpu=1)
    st = cp.get("/v1/cluster/status", query={"project": proj["id"]})
    assert st["nodes_ready"] == 1
    time.sleep(1.5)  # grace 0.6 s, no heartbeats
    st = cp.get("/v1/cluster/status", query={"project": proj["id"]})
    assert st["nodes_ready"] == 0 and st["gpus_allocatable"] == 0
    _heartbeat(nc, "kubenode1")
    st = cp.get("/v1/cluster/status", query={"project": proj["id"]})
    assert st["nodes_ready"] == 1
    evs = cp.get(f"/r/projects/{proj['id']}/kubernetes/api/v1/events")["items"]
    assert any(e["reason"] == "NodeNotReady" for e in evs)


def test_gpu_scheduler_respects_capacity_and_validation(cp):
    proj = _env(cp)
    k = client_from_kubeconfig(cp.get(f"/env/{proj['id']}/kubernetes/kubectl", query={"format": "json"}))
    n1, _ = _join(cp, proj["id"], "kubenode1", ngpu=1)
    n2, _ = _join(cp, proj["id"], "kubenode2", ngpu=2)

    def gpod(name, g):
        return {"metadata": {"name": name}, "spec": {"restartPolicy": "Never", "containers": [
            {"name": "c", "command": ["true"], "resources": {"limits": {GPU: g}}}]}}

    k.post(k.k8s("/api/v1/namespaces/default/pods"), gpod("a", 1))
    p = k.get(k.k8s("/api/v1/namespaces/default/pods/a"))
    assert "nodeName" not in p["spec"]  # nodes not validated yet: GPU pods wait
    assert any(c["type"] == "PodScheduled" and c["status"] == "False" for c in p["status"]["conditions"])
    # validate both nodes through the validation DaemonSet
    ds = {"metadata": {"name": "val", "labels": {"tk8s.amd.com/validation": "true"}},
          "spec": {"selector": {"matchLabels": {"app": "val"}}, "template": {"spec": {"restartPolicy": "Never",
                   "nodeSelector": {"amd.com/gpu.family": "gfx950"}, "containers": [{"name": "p", "command": ["true"]}]}}}}
    k.post(k.k8s("/apis/apps/v1/namespaces/kube-system/daemonsets"), ds)
    pods = k.get(k.k8s("/api/v1/namespaces/kube-system/pods"))["items"]
    assert sorted(o["spec"]["nodeName"] for o in pods) == ["kubenode1", "kubenode2"]
    for o, nc in zip(sorted(pods, key=lambda o: o["spec"]["nodeName"]), (n1, n2)):
        _set_pod(nc, "kube-system", o["metadata"]["name"], "Succeeded", {"hbm": {"gbps": 4400.0}})
    st = cp.get("/v1/cluster/status", query={"project": proj["id"]})
    assert st["nodes_validated"] == 2 and st["gpus_allocatable"] == 3
    node = k.get(k.k8s("/api/v1/nodes/kubenode1"))
    assert node["metadata"]["annotations"]["tk8s.amd.com/hbm-write-gbps"] == "4400.0"
    # now the pending pod binds; a 2-GPU pod can only go to kubenode2; a third GPU pod cannot fit
    assert k.get(k.k8s("/api/v1/namespaces/default/pods/a"))["spec"].get("nodeName")
    k.post(k.k8s("/api/v1/namespaces/default/pods"), gpod("b", 2))
    b = k.get(k.k8s("/api/v1/namespaces/default/pods/b"))
    a = k.get(k.k8s("/api/v1/namespaces/default/pods/a"))
    assert b["spec"].get("nodeName") == "kubenode2" and a["spec"]["nodeName"] == "kubenode1"
    k.post(k.k8s("/api/v1/namespaces/default/pods"), gpod("c", 1))
    assert "nodeName" not in k.get(k.k8s("/api/v1/namespaces/default/pods/c"))["spec"]
    # finishing "a" frees its GPU for "c"
    _set_pod(n1, "default", "a", "Succeeded")
    assert k.get(k.k8s("/api/v1/namespaces/default/pods/c"))["spec"]["nodeName"] == "kubenode1"


def test_validation_failure_marks_node(cp):
    proj = _env(cp)
    k = client_from_kubeconfig(cp.get(f"/env/{proj['id']}/kubernetes/kubectl", query={"format": "json"}))
    nc, _ = _join(cp, proj["id"], "kubenode1", ngpu=1)
    ds = {"metadata": {"name": "val", "labels": {"tk8s.amd.com/validation": "true"}},
          "spec": {"template": {"spec": {"restartPolicy": "Never", "containers": [{"name": "p", "command": ["true"]}]}}}}
    k.post(k.k8s("/apis/apps/v1/namespaces/kube-system/daemonsets"), ds)
    (pod,) = k.get(k.k8s("/api/v1/namespaces/kube-system/pods"))["items"]
    _set_pod(nc, "kube-system", pod["metadata"]["name"], "Failed")
    w = cp.get("/v1/cluster/wait", query={"project": proj["id"], "nodes": 1, "gpus": 1, "validated": 1, "timeout": 5})
    assert w["failed"] and not w["ready"] and w["nodes_validation_failed"] == 1


def test_indexed_job_gang_and_completion(cp):
    proj = _env(cp)
    k = client_from_kubeconfig(cp.get(f"/env/{proj['id']}/kubernetes/kubectl", query={"format": "json"}))
    ncs = [_join(cp, proj["id"], f"kubenode{i}", ngpu=0)[0] for i in (1, 2)]
    job = {"metadata": {"name": "rccl"}, "spec": {"completions": 2, "parallelism": 2, "completionMode": "Indexed",
                                                  "backoffLimit": 0, "template": {"spec": {"restartPolicy": "Never",
                                                  "containers": [{"name": "r", "command": ["true"]}]}}}}
    k.post(k.k8s("/apis/batch/v1/namespaces/kube-system/jobs"), job)
    pods = k.get(k.k8s("/api/v1/namespaces/kube-system/pods"), query={"labelSelector": "job-name=rccl"})["items"]
    assert len(pods) == 2
    idx = sorted(int(next(e["value"] for e in o["spec"]["containers"][0]["env"] if e["name"] == "JOB_COMPLETION_INDEX"))
                 for o in pods)
    assert idx == [0, 1]
    assert len({o["spec"]["nodeName"] for o in pods}) == 2  # spread: one rank per node
    by_node = {f"kubenode{i}": nc for i, nc in zip((1, 2), ncs)}
    for o in pods:
        _set_pod(by_node[o["spec"]["nodeName"]], "kube-system", o["metadata"]["name"], "Succeeded")
    j = k.get(k.k8s("/apis/batch/v1/namespaces/kube-system/jobs/rccl"))
    assert j["status"]["succeeded"] == 2
    assert any(c["type"] == "Complete" and c["status"] == "True" for c in j["status"]["conditions"])
    w = cp.get("/v1/cluster/wait", query={"project": proj["id"], "nodes": 2, "validated": 0, "job": "kube-system/rccl",
                                          "timeout": 2})
    assert w["ready"] and w["job"] == "Complete"


def test_job_backoff_exceeded_fails(cp):
    proj = _env(cp)
    k = client_from_kubeconfig(cp.get(f"/env/{proj['id']}/kubernetes/kubectl", query={"format": "json"}))
    nc, _ = _join(cp, proj["id"], "kubenode1", ngpu=0)
    job = {"metadata": {"name": "j"}, "spec": {"completions": 1, "backoffLimit": 0, "template": {"spec": {
        "restartPolicy": "Never", "containers": [{"name": "r", "command": ["false"]}]}}}}
    k.post(k.k8s("/apis/batch/v1/namespaces/default/jobs"), job)
    (pod,) = k.get(k.k8s("/api/v1/namespaces/default/pods"))["items"]
    _set_pod(nc, "default", pod["metadata"]["name"], "Failed")
    j = k.get(k.k8s("/apis/batch/v1/namespaces/default/jobs/j"))
    assert any(c["type"] == "Failed" and c.get("reason") == "BackoffLimitExceeded" for c in j["status"]["conditions"])


def test_deployment_scales_and_delete_cascades(cp):
    proj = _env(cp)
    k = client_from_kubeconfig(cp.get(f"/env/{proj['id']}/kubernetes/kubectl", query={"format": "json"}))
    _join(cp, proj["id"], "kubenode1", ngpu=0)
    dep = {"metadata": {"name": "guestbook"}, "spec": {"replicas": 3, "selector": {"matchLabels": {"app": "gb"}},
                                                       "template": {"spec": {"containers": [{"name": "c", "command": ["sleep", "1"]}]}}}}
    k.post(k.k8s("/apis/apps/v1/namespaces/default/deployments"), dep)
    pods = k.get(k.k8s("/api/v1/namespaces/default/pods"), query={"labelSelector": "app=gb"})["items"]
    assert len(pods) == 3 and all(o["spec"].get("nodeName") == "kubenode1" for o in pods)
    k.delete(k.k8s("/apis/apps/v1/namespaces/default/deployments/guestbook"))
    assert k.get(k.k8s("/api/v1/namespaces/default/pods"))["items"] == []


def test_kv_rendezvous_long_poll(cp):
    import threading

    got = {}

    def reader():
        got["v"] = cp.get("/v1/kv/job/uid", query={"wait": "5"}, raw=True)

    t = threading.Thread(target=reader)
    t.start()
    time.sleep(0.2)
    with pytest.raises(ApiError) as ei:  # the KV answers no anonymous caller (controlplane/authn.py)
        Client(cp.base).put("/v1/kv/job/uid", "evil")
    assert ei.value.status == 401
    Client(cp.base, token=cp.token).put("/v1/kv/job/uid", "abc123")
    t.join(10)
    assert got["v"] == "abc123"
    with pytest.raises(ApiError):
        cp.get("/v1/kv/none", raw=True)


def test_watch_returns_events_after_resource_version(cp):
    proj = _env(cp)
    k = client_from_kubeconfig(cp.get(f"/env/{proj['id']}/kubernetes/kubectl", query={"format": "json"}))
    rv = int(k.get(k.k8s("/api/v1/nodes"))["metadata"]["resourceVersion"])
    _join(cp, proj["id"], "kubenode1", ngpu=0)
    rv2, evs = k.watch(k.k8s("/api/v1/nodes"), rv, timeout=5)
    assert rv2 > rv and any(e["object"]["metadata"]["name"] == "kubenode1" for e in evs)


def test_state_snapshot_survives_restart(tmp_path):
    sd = tmp_path / "cpstate"
    p, c = _start(tmp_path, grace=30, state_dir=sd)
    try:
        proj = _env(c)
        _join(c, proj["id"], "kubenode1", ngpu=1)
    finally:
        _stop(p)
    p, c = _start(tmp_path, grace=30, state_dir=sd)
    try:
        st = c.get("/v1/cluster/status", query={"project": proj["id"]})
        assert st["nodes"] == 1 and st["node_names"] == ["kubenode1"]
    finally:
        _stop(p)


def test_metrics_and_version(cp):
    proj = _env(cp)
    nc, _ = _join(cp, proj["id"], "kubenode1", ngpu=1)
    # a heartbeat with GPU telemetry (AMD SMI) and a usage sample, as the agent sends them
    nc.put(nc.k8s("/api/v1/nodes/kubenode1/status"), {"devices": [{"id": "gpu0", "health": "Healthy", "pciBusId": "0000:75:00.0",
        "telemetry": {"temp_c": {"hotspot": 41}, "power": {"current_w": 212.5}, "vram_used_bytes": 1 << 30,
                      "activity": {"gfx_pct": 87, "umc_pct": 40}, "ecc": {"uncorrectable": 0, "correctable": 2}}}],
        "metrics": {"pods": {"default/train": [{"name": "c", "cpu_cores": 0.5, "memory_bytes": 1024, "gpu_pct": 87.0}]}}})
    text = cp.get("/metrics", raw=True)
    assert "tk8s_nodes" in text
    for line in ('tk8s_gpu_gfx_activity_percent{node="kubenode1",gpu="gpu0",pci="0000:75:00.0"} 87',
                 'tk8s_gpu_power_watts{node="kubenode1",gpu="gpu0",pci="0000:75:00.0"} 212.5',
                 'tk8s_gpu_healthy{node="kubenode1",gpu="gpu0",pci="0000:75:00.0"} 1',
                 'tk8s_gpu_ecc_correctable_total{node="kubenode1",gpu="gpu0",pci="0000:75:00.0"} 2',
                 'tk8s_container_gpu_busy_percent{namespace="default",pod="train",container="c",node="kubenode1"} 87.0'):
        assert line in text, line
    assert "version" in json.dumps(cp.get("/version")).lower()
    # kube-apiserver's request metrics: the node's status PUT, counted with its code and latency
    text = cp.get("/metrics", raw=True)
    assert 'apiserver_request_total{verb="PUT",group="",resource="nodes",subresource="status",code="200"} 1' in text
    assert 'apiserver_request_duration_seconds_count{verb="PUT",group="",resource="nodes",subresource="status"} 1' in text


def test_request_classification():
    from tritonk8ssupervisor_amd.controlplane.reqmetrics import RequestMetrics, classify

    assert classify("GET", "/api/v1/namespaces/default/pods", False) == ("LIST", "", "pods", "")
    assert classify("GET", "/api/v1/pods", True) == ("WATCH", "", "pods", "")
    assert classify("GET", "/r/projects/1a1/kubernetes/apis/apps/v1/namespaces/x/deployments/web/scale", False) == (
        "GET", "apps", "deployments", "scale")
    assert classify("POST", "/v2-beta/projects", False)[2] == "(other)"
    assert classify("GET", "/apis/apps/v1", False)[2] == "(discovery)"
    m = RequestMetrics()
    m.observe("GET", "/api/v1/pods", False, 200, 0.003)
    m.observe("GET", "/api/v1/pods", True, 200, 0.0)
    lines = m.lines()
    assert 'apiserver_request_duration_seconds_bucket{verb="LIST",group="",resource="pods",subresource="",le="0.0025"} 0' in lines
    assert 'apiserver_request_duration_seconds_bucket{verb="LIST",group="",resource="pods",subresource="",le="0.005"} 1' in lines
    assert not any('verb="WATCH"' in x and "duration" in x for x in lines)


def test_put_patch_scale_and_rolling_update(cp):
    proj = _env(cp)
    k = client_from_kubeconfig(cp.get(f"/env/{proj['id']}/kubernetes/kubectl", query={"format": "json"}))
    nc, _ = _join(cp, proj["id"], "kubenode1", ngpu=0)
    base = "/apis/apps/v1/namespaces/default/deployments"
    dep = {"metadata": {"name": "web"}, "spec": {"replicas": 2, "selector": {"matchLabels": {"app": "web"}},
           "template": {"metadata": {"labels": {"app": "web"}}, "spec": {"containers": [{"name": "c", "command": ["v1"]}]}}}}
    d = k.post(k.k8s(base), dep)
    assert d["metadata"]["generation"] == 1
    pods = lambda: k.get(k.k8s("/api/v1/namespaces/default/pods"), query={"labelSelector": "app=web"})["items"]
    v1 = pods()
    assert len(v1) == 2 and len({p["metadata"]["labels"]["pod-template-hash"] for p in v1}) == 1
    for p in v1:
        _set_pod(nc, "default", p["metadata"]["name"], "Running")
    # stale resourceVersion -> 409; clusterIP-style immutability for Jobs -> 422
    stale = dict(dep, metadata={"name": "web", "resourceVersion": "1"})
    with pytest.raises(ApiError) as ei:
        k.put(k.k8s(base + "/web"), stale)
    assert ei.value.status == 409
    # a new template: maxSurge 1, maxUnavailable 0 -> one extra pod, no old pod gone yet
    k.request("PATCH", k.k8s(base + "/web"), body={"spec": {"template": {"spec": {"containers": [{"name": "c", "command": ["v2"]}]}}}})
    d = k.get(k.k8s(base + "/web"))
    assert d["metadata"]["generation"] == 2
    now = pods()
    new = [p for p in now if p["spec"]["containers"][0]["command"] == ["v2"]]
    assert len(now) == 3 and len(new) == 1
    # each new pod that runs releases one old pod, until the rollout is complete; a released pod
    # is Terminating until its node's agent (played here) confirms it has stopped
    terminating = set()
    for _ in range(4):
        for p in pods():
            if p["metadata"].get("deletionTimestamp"):
                terminating.add(p["metadata"]["name"])
                nc.delete(nc.k8s(f"/api/v1/namespaces/default/pods/{p['metadata']['name']}"),
                          query={"gracePeriodSeconds": "0"})
            elif p["spec"]["containers"][0]["command"] == ["v2"] and p["status"].get("phase") != "Running":
                _set_pod(nc, "default", p["metadata"]["name"], "Running")
    assert terminating == {p["metadata"]["name"] for p in v1}
    final = pods()
    assert len(final) == 2 and all(p["spec"]["containers"][0]["command"] == ["v2"] for p in final)
    st = k.get(k.k8s(base + "/web"))["status"]
    assert st["updatedReplicas"] == 2 and st["readyReplicas"] == 2 and st["observedGeneration"] == 2
    # scale subresource
    sc = k.request("PATCH", k.k8s(base + "/web/scale"), body={"spec": {"replicas": 1}})
    live = [p for p in pods() if not p["metadata"].get("deletionTimestamp")]
    assert sc["kind"] == "Scale" and sc["spec"]["replicas"] == 1 and len(live) == 1 and len(pods()) == 2
    with pytest.raises(ApiError) as ei:
        k.request("PATCH", k.k8s(base + "/web/scale"), body={"spec": {"replicas": -1}})
    assert ei.value.status == 422
    # labels: merge patch adds and (null) removes
    k.request("PATCH", k.k8s(base + "/web"), body={"metadata": {"labels": {"tier": "fe"}}})
    k.request("PATCH", k.k8s(base + "/web"), body={"metadata": {"labels": {"tier": None}}})
    assert "tier" not in k.get(k.k8s(base + "/web"))["metadata"]["labels"]


def test_configmaps_secrets_and_service_update(cp):
    import base64

    proj = _env(cp)
    k = client_from_kubeconfig(cp.get(f"/env/{proj['id']}/kubernetes/kubectl", query={"format": "json"}))
    s = k.post(k.k8s("/api/v1/namespaces/default/secrets"), {"metadata": {"name": "s"}, "stringData": {"pw": "x"}})
    assert s["data"] == {"pw": base64.b64encode(b"x").decode()} and s["type"] == "Opaque" and "stringData" not in s
    with pytest.raises(ApiError) as ei:
        k.post(k.k8s("/api/v1/namespaces/default/secrets"), {"metadata": {"name": "bad"}, "data": {"k": "%%%"}})
    assert ei.value.status == 422
    with pytest.raises(ApiError) as ei:
        k.post(k.k8s("/api/v1/namespaces/default/configmaps"), {"metadata": {"name": "c"}, "data": {"n": 1}})
    assert ei.value.status == 422
    k.post(k.k8s("/api/v1/namespaces/default/configmaps"), {"metadata": {"name": "c"}, "data": {"n": "1"}})
    assert k.get(k.k8s("/api/v1/configmaps"))["items"][0]["data"] == {"n": "1"}
    svc = k.post(k.k8s("/api/v1/namespaces/default/services"), {"metadata": {"name": "web"}, "spec": {
        "type": "NodePort", "selector": {"app": "web"}, "ports": [{"port": 8000}]}})
    cip, np = svc["spec"]["clusterIP"], svc["spec"]["ports"][0]["nodePort"]
    upd = k.put(k.k8s("/api/v1/namespaces/default/services/web"), {"metadata": {"name": "web"}, "spec": {
        "type": "NodePort", "selector": {"app": "web2"}, "ports": [{"port": 8000}]}})
    assert upd["spec"]["clusterIP"] == cip and upd["spec"]["ports"][0]["nodePort"] == np
    assert upd["spec"]["selector"] == {"app": "web2"}
    with pytest.raises(ApiError) as ei:
        k.put(k.k8s("/api/v1/namespaces/default/services/web"), {"metadata": {"name": "web"}, "spec": {
            "clusterIP": "127.96.9.9", "ports": [{"port": 8000}]}})
    assert ei.value.status == 422


def test_cluster_dns_names():
    from tritonk8ssupervisor_amd.controlplane import dns
    from tritonk8ssupervisor_amd.controlplane.server import ControlPlane

    cpl = ControlPlane("127.0.0.1", 0)
    cpl.store.put("projects", "1a1", {"id": "1a1", "created_seq": 1, "metadata": {"name": "1a1"}})
    cpl.store.put("services", "1a1/shop/cart", {"_project": "1a1", "metadata": {"name": "cart", "namespace": "shop"},
                                                "spec": {"clusterIP": "127.96.0.9", "ports": [{"port": 80}]}})
    assert cpl.dns_resolve("cart.shop.svc.cluster.local") == ["127.96.0.9"]
    assert cpl.dns_resolve("cart.shop.svc") == ["127.96.0.9"] == cpl.dns_resolve("cart.shop")
    assert cpl.dns_resolve("127-128-0-7.shop.pod.cluster.local") == ["127.128.0.7"]
    assert cpl.dns_resolve("nope.shop.svc.cluster.local") is None
    assert cpl.dns_resolve("example.com") is False
    q = dns.query("cart.shop.svc.cluster.local")
    qid, flags, labels, qtype, qclass, question = dns.parse_query(q)
    assert labels == ["cart", "shop", "svc", "cluster", "local"] and qtype == 1
    assert dns.parse_reply(dns.build_reply(qid, flags, question, 0, ["127.96.0.9"])) == (0, ["127.96.0.9"])
    assert dns.parse_reply(dns.build_reply(qid, flags, question, dns.NXDOMAIN, [])) == (dns.NXDOMAIN, [])


def test_external_name_services_and_session_affinity():
    """An ExternalName Service is a DNS alias (CNAME, no IP, no proxy); ClientIP session affinity
    keeps a client on one endpoint."""
    import asyncio

    from tritonk8ssupervisor_amd.controlplane import dns
    from tritonk8ssupervisor_amd.controlplane.httpserver import HttpError
    from tritonk8ssupervisor_amd.controlplane.proxy import ServiceProxy
    from tritonk8ssupervisor_amd.controlplane.server import ControlPlane

    cpl = ControlPlane("127.0.0.1", 0)
    cpl.store.put("projects", "1a1", {"id": "1a1", "created_seq": 1, "metadata": {"name": "1a1"}})
    o = cpl.create("1a1", "services", "shop", {"metadata": {"name": "db"}, "spec": {
        "type": "ExternalName", "externalName": "db.prod.example.com"}})
    assert "clusterIP" not in o["spec"] and not any(k[0].endswith("/db") for k in cpl._proxy_wanted())
    ans = cpl.dns_resolve("db.shop.svc.cluster.local")
    assert isinstance(ans, dns.CName) and ans == "db.prod.example.com"
    qid, flags, _l, _t, _c, question = dns.parse_query(dns.query("db.shop.svc.cluster.local"))
    cn = []
    assert dns.parse_reply(dns.build_reply(qid, flags, question, 0, [], cname=ans), cn) == (0, []) and cn == [ans]
    with pytest.raises(HttpError):
        cpl.create("1a1", "services", "shop", {"metadata": {"name": "bad"}, "spec": {"type": "ExternalName"}})
    s = cpl.create("1a1", "services", "shop", {"metadata": {"name": "web"}, "spec": {
        "ports": [{"port": 80}], "sessionAffinity": "ClientIP"}})
    assert cpl._svc_affinity("1a1/shop/web") == 10800.0

    async def run():  # two backends; with affinity every connection from 127.0.0.1 lands on the same one
        hits = []

        async def backend(tag, r, w):
            hits.append(tag)
            w.close()

        s1 = await asyncio.start_server(lambda r, w: backend("a", r, w), "127.0.0.1", 0)
        s2 = await asyncio.start_server(lambda r, w: backend("b", r, w), "127.0.0.1", 0)
        eps = [("127.0.0.1", s1.sockets[0].getsockname()[1]), ("127.0.0.1", s2.sockets[0].getsockname()[1])]
        for aff in (0, 60):
            hits.clear()
            px = ServiceProxy(lambda svc, pk: eps, affinity=lambda svc, a=aff: a)
            await px.sync({("svc", "127.0.0.1", 0): "80"})
            port = next(iter(px.listeners.values())).sockets[0].getsockname()[1]
            for _ in range(4):
                r, w = await asyncio.open_connection("127.0.0.1", port)
                await r.read()
                w.close()
            await asyncio.sleep(0.05)
            await px.close()
            yield sorted(set(hits))
        s1.close()
        s2.close()

    async def collect():
        return [x async for x in run()]

    spread, sticky = asyncio.run(collect())
    assert spread == ["a", "b"] and len(sticky) == 1
