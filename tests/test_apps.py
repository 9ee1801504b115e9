"""The reference's acceptance demos on a tk8s cluster (docs/detailed.md:255-370) and the
Kubernetes workload API they lean on: the three-tier Guestbook (redis leader + followers +
frontend, images mapped to built-in apps) through kubectl, Ghost through the dashboard's deploy
form, Service env vars, ConfigMaps/Secrets, rolling updates, scale, Ingress, cluster DNS, drain."""
import asyncio
import json
import os
import shutil
import socket
import subprocess
import sys
import threading
import time
import urllib.error
import urllib.request
from pathlib import Path

import pytest

from tritonk8ssupervisor_amd.apps import image_name, resolve
from tritonk8ssupervisor_amd.apps.redis import Redis
from tritonk8ssupervisor_amd.apps.resp import RespError, call
from tritonk8ssupervisor_amd.controlplane.ingress import match_route
from tritonk8ssupervisor_amd.utils.k8senv import field_path, service_env
from tritonk8ssupervisor_amd.utils.net import host_port

REPO = Path(__file__).resolve().parents[1]


# ---- units ----------------------------------------------------------------------------------
def test_image_catalogue():
    assert image_name("gcr.io/google-samples/gb-frontend:v4") == "gb-frontend"
    assert image_name("registry.k8s.io/redis:e2e@sha256:abc") == "redis"
    assert resolve("ghost:5")[-1] == "tritonk8ssupervisor_amd.apps.ghost"
    assert resolve("gcr.io/google_samples/gb-redisslave:v1")[-2:] == ["--follow", "redis-master,redis-leader"]
    assert resolve("busybox") is None and resolve(None) is None


def test_host_port_remap(monkeypatch):
    monkeypatch.setenv("TK8S_REMAP_PRIVILEGED_PORTS", "1")
    assert host_port(80) == 20080 and host_port(6379) == 6379
    monkeypatch.setenv("TK8S_REMAP_PRIVILEGED_PORTS", "0")
    assert host_port(80) == 80


def test_service_env_matches_the_kubelet(monkeypatch):
    monkeypatch.setenv("TK8S_REMAP_PRIVILEGED_PORTS", "0")
    svcs = [{"metadata": {"name": "redis-master"}, "spec": {"clusterIP": "127.96.0.5", "ports": [
        {"name": "redis", "port": 6379, "protocol": "TCP"}]}},
        {"metadata": {"name": "headless"}, "spec": {"clusterIP": "None", "ports": [{"port": 1}]}}]
    env = service_env(svcs, "http://127.0.1.1:8080")
    assert env["REDIS_MASTER_SERVICE_HOST"] == "127.96.0.5" and env["REDIS_MASTER_SERVICE_PORT"] == "6379"
    assert env["REDIS_MASTER_SERVICE_PORT_REDIS"] == "6379"
    assert env["REDIS_MASTER_PORT"] == "tcp://127.96.0.5:6379"
    assert env["REDIS_MASTER_PORT_6379_TCP_ADDR"] == "127.96.0.5"
    assert env["KUBERNETES_SERVICE_HOST"] == "127.0.1.1" and env["KUBERNETES_SERVICE_PORT"] == "8080"
    assert not any(k.startswith("HEADLESS") for k in env)
    pod = {"metadata": {"name": "p", "namespace": "ns", "labels": {"app": "x"}}, "spec": {"nodeName": "n1"}}
    assert field_path(pod, "metadata.labels['app']") == "x" and field_path(pod, "spec.nodeName") == "n1"
    assert field_path(pod, "status.podIP", "127.128.0.2") == "127.128.0.2"
    with pytest.raises(ValueError):
        field_path(pod, "spec.bogus")


def test_ingress_rule_matching():
    routes = [("", "/", "Prefix", "svc-default", "80"), ("shop.local", "/api", "Prefix", "svc-api", "80"),
              ("shop.local", "/api/v2", "Exact", "svc-v2", "80"), ("", "/static", "Prefix", "svc-static", "80")]
    assert match_route(routes, "shop.local:80", "/api/cart") == ("svc-api", "80")
    assert match_route(routes, "shop.local", "/api/v2") == ("svc-v2", "80")
    assert match_route(routes, "other", "/static/x.css") == ("svc-static", "80")
    assert match_route(routes, "other", "/staticky") == ("svc-default", "80")
    assert match_route(routes[1:3], "other", "/api") is None


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture
def redis_pair():
    """A leader and a follower on one private event loop thread."""
    loop = asyncio.new_event_loop()
    leader, follower = Redis(), Redis(sync_interval=0.02)
    ports = (_free_port(), _free_port())
    follower.leader = ("127.0.0.1", ports[0])

    async def start():
        servers = [await asyncio.start_server(db.handle, "127.0.0.1", p) for db, p in zip((leader, follower), ports)]
        tasks = [asyncio.ensure_future(follower.follow_loop())]
        return servers, tasks

    servers, tasks = loop.run_until_complete(start())
    t = threading.Thread(target=loop.run_forever, daemon=True)
    t.start()
    yield ports

    async def stop():
        for task in tasks:
            task.cancel()
        await asyncio.gather(*tasks, return_exceptions=True)
        for srv in servers:
            srv.close()

    asyncio.run_coroutine_threadsafe(stop(), loop).result(5)
    loop.call_soon_threadsafe(loop.stop)
    t.join(5)


def test_redis_commands_and_replication(redis_pair):
    lp, fp = redis_pair
    assert call("127.0.0.1", lp, "PING") == "PONG"
    assert call("127.0.0.1", lp, "SET", "messages", "hello,world") == "OK"
    assert call("127.0.0.1", lp, "GET", "messages") == b"hello,world"
    assert call("127.0.0.1", lp, "RPUSH", "l", "a", "b", "c") == 3
    assert call("127.0.0.1", lp, "LRANGE", "l", "0", "-1") == [b"a", b"b", b"c"]
    assert call("127.0.0.1", lp, "INCR", "n") == 1 and call("127.0.0.1", lp, "INCRBY", "n", "41") == 42
    with pytest.raises(RespError, match="WRONGTYPE"):
        call("127.0.0.1", lp, "GET", "l")
    with pytest.raises(RespError, match="unknown command"):
        call("127.0.0.1", lp, "NOPE")
    assert call("127.0.0.1", lp, "ROLE")[0] == b"master"
    # the follower replicates by whole snapshots (TK8S.DUMP): wait for the LAST write; a snapshot
    # holding it holds every earlier one (waiting for the first raced the later RPUSH)
    deadline = time.monotonic() + 5
    while call("127.0.0.1", fp, "GET", "n") != b"42":
        assert time.monotonic() < deadline
        time.sleep(0.02)
    assert call("127.0.0.1", fp, "GET", "messages") == b"hello,world"
    assert call("127.0.0.1", fp, "LRANGE", "l", "0", "-1") == [b"a", b"b", b"c"]
    with pytest.raises(RespError, match="READONLY"):
        call("127.0.0.1", fp, "SET", "x", "1")
    assert b"role:slave" in call("127.0.0.1", fp, "INFO")
    assert call("127.0.0.1", fp, "REPLICAOF", "NO", "ONE") == "OK"  # promote
    assert call("127.0.0.1", fp, "SET", "x", "1") == "OK"


# ---- end to end on a local cluster ------------------------------------------------------------


@pytest.fixture
def cluster(tmp_path, monkeypatch):
    from tritonk8ssupervisor_amd.orchestrator import init_workspace

    monkeypatch.setenv("TK8S_REMAP_PRIVILEGED_PORTS", "1")  # the test's view of the shifted ports too
    init_workspace(tmp_path)
    for f in ("setup.sh", "tk8s", "kubectl"):
        shutil.copy2(REPO / f, tmp_path / f)
    env = dict(os.environ, PYTHONPATH=str(REPO), TK8S_PYTHON=sys.executable, TK8S_FAKE_GPUS="8",
               TK8S_REMAP_PRIVILEGED_PORTS="1",  # exercise the non-root port shift even as root
               TK8S_METRICS_PERIOD="0.5", TK8S_VOLUME_SYNC_PERIOD="0.5")
    env.pop("TK8S_FAULTS", None)
    r = subprocess.run(["./setup.sh", "--yes", "--json", "--port", "0", "--nodes", "2", "--rccl", "off"], cwd=tmp_path,
                       env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    summary = json.loads(r.stdout.strip().splitlines()[-1])

    def kc(*a, check=True):
        p = subprocess.run(["./kubectl", *a], cwd=tmp_path, env=env, capture_output=True, text=True, timeout=120)
        if check:
            assert p.returncode == 0, f"kubectl {' '.join(a)}: {p.stdout}{p.stderr}"
        return p

    yield tmp_path, env, kc, summary
    subprocess.run(["./setup.sh", "-c", "--yes"], cwd=tmp_path, env=env, capture_output=True, timeout=120)


def _get(url, timeout=5.0):
    return urllib.request.urlopen(url, timeout=timeout).read().decode()


def _until(fn, timeout=20.0):
    deadline = time.monotonic() + timeout
    while True:
        try:
            v = fn()
            if v:
                return v
        except OSError:
            pass
        assert time.monotonic() < deadline, "condition not met in time"
        time.sleep(0.05)


@pytest.mark.slow
def test_guestbook_all_in_one_through_kubectl(cluster):
    ws, env, kc, _ = cluster
    out = kc("apply", "-f", str(REPO / "manifests" / "examples" / "guestbook-all-in-one.yaml")).stdout
    assert "deployment/frontend created" in out and "service/redis-master created" in out
    for d in ("redis-master", "redis-slave", "frontend"):
        assert "successfully rolled out" in kc("rollout", "status", f"deploy/{d}", "--timeout", "60s").stdout
    svc = json.loads(kc("get", "svc", "frontend", "-o", "json").stdout)
    url = f"http://{svc['status']['loadBalancer']['ingress'][0]['ip']}:{host_port(80)}"
    assert "(host 20080)" in kc("get", "svc").stdout
    assert "<title>Guestbook</title>" in _until(lambda: _get(url + "/"))
    assert json.loads(_get(url + "/guestbook.php?cmd=set&key=messages&value=hello,tk8s")) == {"message": "Updated"}
    # reads go to a follower, which replicates the leader
    _until(lambda: json.loads(_get(url + "/guestbook.php?cmd=get&key=messages"))["data"] == "hello,tk8s")
    # apply again: unchanged; scale; a template change rolls out pod by pod
    assert "deployment/frontend unchanged" in kc("apply", "-f", str(REPO / "manifests" / "examples" / "guestbook-all-in-one.yaml")).stdout
    kc("scale", "deploy/frontend", "--replicas", "1")
    kc("rollout", "status", "deploy/frontend", "--timeout", "60s")
    pods = json.loads(kc("get", "pods", "-l", "tier=frontend", "-o", "json").stdout)["items"]
    assert len([p for p in pods if p["status"].get("phase") == "Running"]) == 1
    old_hash = pods[0]["metadata"]["labels"]["pod-template-hash"]
    kc("rollout", "restart", "deploy/frontend")
    kc("rollout", "status", "deploy/frontend", "--timeout", "60s")
    pods = json.loads(kc("get", "pods", "-l", "tier=frontend", "-o", "json").stdout)["items"]
    assert {p["metadata"]["labels"]["pod-template-hash"] for p in pods} != {old_hash}
    _until(lambda: json.loads(_get(url + "/guestbook.php?cmd=get&key=messages"))["data"] == "hello,tk8s")


@pytest.mark.slow
def test_config_env_ingress_dns_and_drain(cluster, tmp_path_factory):
    ws, env, kc, summary = cluster
    from tritonk8ssupervisor_amd.controlplane import dns

    d = tmp_path_factory.mktemp("m")
    kc("create", "configmap", "app-config", "--from-literal", "GREETING=hello", "--from-literal", "COLOR=blue")
    kc("create", "secret", "generic", "app-secret", "--from-literal", "password=s3cr3t")
    assert "app-config" in kc("get", "cm").stdout and "Opaque" in kc("get", "secrets").stdout
    (d / "env.yaml").write_text(json.dumps({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "envpod", "labels": {"app": "envpod"}},
        "spec": {"restartPolicy": "Never", "containers": [{"name": "c", "command": ["sh", "-c", "env | sort"],
                 "envFrom": [{"configMapRef": {"name": "app-config"}, "prefix": "CFG_"}],
                 "env": [{"name": "PW", "valueFrom": {"secretKeyRef": {"name": "app-secret", "key": "password"}}},
                         {"name": "ME", "valueFrom": {"fieldRef": {"fieldPath": "metadata.labels['app']"}}},
                         {"name": "LATE", "valueFrom": {"configMapKeyRef": {"name": "late-config", "key": "v"}}}]}]}}))
    kc("apply", "-f", str(d / "env.yaml"))
    pod = _until(lambda: json.loads(kc("get", "pod", "envpod", "-o", "json").stdout))
    _until(lambda: json.loads(kc("get", "pod", "envpod", "-o", "json").stdout)["status"].get("reason") == "CreateContainerConfigError")
    kc("create", "configmap", "late-config", "--from-literal", "v=arrived")  # the kubelet retries
    _until(lambda: json.loads(kc("get", "pod", "envpod", "-o", "json").stdout)["status"].get("phase") == "Succeeded")
    log = kc("logs", "envpod").stdout
    for line in ("CFG_GREETING=hello", "CFG_COLOR=blue", "PW=s3cr3t", "ME=envpod", "LATE=arrived", "KUBERNETES_SERVICE_HOST="):
        assert line in log, line
    # a web app behind a Service, reached through an Ingress rule and cluster DNS
    kc("apply", "-f", str(REPO / "manifests" / "examples" / "ingress-nginx.yaml"))
    kc("rollout", "status", "deploy/web", "--timeout", "60s")
    ing = json.loads(kc("get", "ingress", "web", "-o", "json").stdout)
    ip = ing["status"]["loadBalancer"]["ingress"][0]["ip"]
    req = urllib.request.Request(f"http://{ip}:{host_port(80)}/", headers={"Host": "web.local"})
    assert "Welcome to nginx!" in _until(lambda: urllib.request.urlopen(req, timeout=5).read().decode())
    req = urllib.request.Request(f"http://{ip}:{host_port(80)}/", headers={"Host": "elsewhere"})
    with pytest.raises(urllib.error.HTTPError) as e:
        urllib.request.urlopen(req, timeout=5)
    assert e.value.code == 404
    svc = json.loads(kc("get", "svc", "web", "-o", "json").stdout)
    with socket.socket(socket.AF_INET, socket.SOCK_DGRAM) as s:
        s.settimeout(5)
        s.sendto(dns.query("web.default.svc.cluster.local"), (ip, host_port(53)))
        assert dns.parse_reply(s.recv(512)) == (0, [svc["spec"]["clusterIP"]])
        s.sendto(dns.query("nope.default.svc.cluster.local"), (ip, host_port(53)))
        assert dns.parse_reply(s.recv(512))[0] == dns.NXDOMAIN
    # drain: pods leave the node, the Deployment re-creates them on the other node
    node = json.loads(kc("get", "pods", "-l", "app=web", "-o", "json").stdout)["items"][0]["spec"]["nodeName"]
    out = kc("drain", node).stdout
    assert "drained" in out and "evicting pod default/web-" in out
    kc("rollout", "status", "deploy/web", "--timeout", "60s")
    pods = json.loads(kc("get", "pods", "-l", "app=web", "-o", "json").stdout)["items"]
    assert pods and all(p["spec"]["nodeName"] != node for p in pods if p["status"].get("phase") == "Running")
    assert "SchedulingDisabled" in kc("get", "nodes").stdout
    top = kc("top", "nodes").stdout
    assert "GPU(USED/ALLOC)" in top and "kubenode1" in top and "CPU(cores)" in top
    kc("label", "node", node, "pool=mi355x")
    assert json.loads(kc("get", "node", node, "-o", "json").stdout)["metadata"]["labels"]["pool"] == "mi355x"
    kc("label", "node", node, "pool-")
    assert "pool" not in json.loads(kc("get", "node", node, "-o", "json").stdout)["metadata"]["labels"]


@pytest.mark.slow
def test_ghost_from_the_dashboard_deploy_form(cluster):
    ws, env, kc, summary = cluster
    dash = summary["dashboard"]
    body = json.dumps({"name": "ghost", "containerImage": "ghost", "replicas": 1, "isExternal": True,
                       "portMappings": [{"port": 2368, "targetPort": 2368, "protocol": "TCP"}]}).encode()
    tok = json.loads((ws / ".tk8s" / "kubeconfig.json").read_text())["users"][0]["user"]["token"]
    with pytest.raises(urllib.error.HTTPError) as ei:  # the form needs the environment's token (authn.py)
        urllib.request.urlopen(urllib.request.Request(dash + "api/v1/appdeployment", data=body, method="POST",
                                                      headers={"Content-Type": "application/json"}), timeout=10)
    assert ei.value.code == 401
    r = urllib.request.urlopen(urllib.request.Request(dash + "api/v1/appdeployment", data=body, method="POST",
                                                      headers={"Content-Type": "application/json",
                                                               "Authorization": f"Bearer {tok}"}), timeout=10)
    assert r.status == 201
    kc("rollout", "status", "deploy/ghost", "--timeout", "60s")
    svc = json.loads(kc("get", "svc", "ghost", "-o", "json").stdout)
    url = f"http://{svc['status']['loadBalancer']['ingress'][0]['ip']}:2368"
    assert "<title>Ghost</title>" in _until(lambda: _get(url + "/"))
    post = json.dumps({"posts": [{"title": "MI355X is Ready", "html": "all 8 GPUs allocatable"}]}).encode()
    urllib.request.urlopen(urllib.request.Request(url + "/ghost/api/v0.1/posts", data=post, method="POST",
                                                  headers={"Content-Type": "application/json"}), timeout=5)
    assert "MI355X is Ready" in _get(url + "/")
    assert "Deploy a containerized app" not in _get(dash)  # anonymous: the node table only
    page = _get(dash + f"?token={tok}")
    assert "Deploy a containerized app" in page and "ghost" in page


@pytest.mark.slow
def test_kubectl_exec_and_logs_follow(cluster, tmp_path_factory):
    ws, env, kc, _ = cluster
    d = tmp_path_factory.mktemp("x")
    (d / "p.yaml").write_text(json.dumps({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "sleeper"},
        "spec": {"containers": [{"name": "c", "command": ["sh", "-c", "echo started; sleep 30"],
                                 "env": [{"name": "GREETING", "value": "hi-from-pod"}]}]}}))
    kc("apply", "-f", str(d / "p.yaml"))
    _until(lambda: json.loads(kc("get", "pod", "sleeper", "-o", "json").stdout)["status"].get("phase") == "Running")
    r = kc("exec", "sleeper", "--", "sh", "-c", "echo $GREETING $POD_NAME; pwd; echo oops >&2; exit 3", check=False)
    assert r.returncode == 3 and "hi-from-pod sleeper" in r.stdout and "oops" in r.stderr
    assert r.stdout.splitlines()[1].endswith("/pods/sleeper")
    r = kc("exec", "sleeper", "--", "no-such-binary", check=False)
    assert r.returncode == 127
    (d / "j.yaml").write_text(json.dumps({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "talker"},
        "spec": {"restartPolicy": "Never", "containers": [{"name": "c", "command": [
            "sh", "-c", "for i in 1 2 3; do echo line$i; sleep 0.3; done"]}]}}))
    kc("apply", "-f", str(d / "j.yaml"))
    _until(lambda: json.loads(kc("get", "pod", "talker", "-o", "json").stdout)["status"].get("phase") in ("Running", "Succeeded"))
    out = kc("logs", "talker", "-f").stdout
    assert out.split() == ["line1", "line2", "line3"]


@pytest.mark.slow
def test_imperative_create_deployment_and_expose(cluster):
    """kubectl create deployment / expose: nginx behind a LoadBalancer Service, no manifest."""
    ws, env, kc, _ = cluster
    assert "deployment.apps/hello created" in kc("create", "deployment", "hello", "--image", "nginx:1.25",
                                                 "--replicas", "2", "--port", "80").stdout
    kc("rollout", "status", "deploy/hello", "--timeout", "60s")
    assert "service/hello exposed" in kc("expose", "deployment", "hello", "--port", "80", "--type", "LoadBalancer").stdout
    svc = json.loads(kc("get", "svc", "hello", "-o", "json").stdout)
    assert svc["spec"]["selector"] == {"app": "hello"} and svc["spec"]["type"] == "LoadBalancer"
    url = f"http://{_until(lambda: json.loads(kc('get', 'svc', 'hello', '-o', 'json').stdout)['status']['loadBalancer']['ingress'])[0]['ip']}:{host_port(80)}/"
    assert "Welcome to nginx!" in _until(lambda: _get(url))
    assert kc("create", "deployment", "broken", check=False).returncode != 0  # --image is required


def test_statefulset_cronjob_and_port_forward_on_a_real_cluster(cluster):
    """A StatefulSet behind a headless Service (stable names, DNS per pod, HOSTNAME), a CronJob
    whose Jobs run, and ./kubectl port-forward to a pod's own IP -- with real node agents."""
    from tritonk8ssupervisor_amd.controlplane import dns

    ws, env, kc, summary = cluster
    (ws / "sts.json").write_text(json.dumps({"apiVersion": "v1", "kind": "List", "items": [
        {"apiVersion": "v1", "kind": "Service", "metadata": {"name": "web"},
         "spec": {"clusterIP": "None", "selector": {"app": "web"}, "ports": [{"port": 8000}]}},
        {"apiVersion": "apps/v1", "kind": "StatefulSet", "metadata": {"name": "web"},
         "spec": {"replicas": 2, "serviceName": "web", "selector": {"matchLabels": {"app": "web"}},
                  "template": {"metadata": {"labels": {"app": "web"}}, "spec": {"containers": [{
                      "name": "c", "image": "python",
                      "command": ["sh", "-c", "echo host=$HOSTNAME; exec python3 -m http.server 8000 --bind $(POD_IP)"]}]}}}},
        {"apiVersion": "batch/v1", "kind": "CronJob", "metadata": {"name": "tick"},
         "spec": {"schedule": "@every 2s", "jobTemplate": {"spec": {"template": {"spec": {
             "restartPolicy": "Never", "containers": [{"name": "c", "image": "busybox", "command": ["echo", "tick"]}]}}}}}}]}))
    kc("apply", "-f", "sts.json")

    def pods():
        return {p["metadata"]["name"]: p for p in json.loads(kc("get", "pods", "-o", "json").stdout)["items"]}

    _until(lambda: all(pods().get(n, {}).get("status", {}).get("phase") == "Running" for n in ("web-0", "web-1")), 60)
    assert "host=web-1" in kc("logs", "web-1").stdout
    ip = kc("cluster-info").stdout.split("://", 1)[1].split(":", 1)[0]  # the master's address
    p0 = pods()["web-0"]["status"]["podIP"]
    with socket.socket(socket.AF_INET, socket.SOCK_DGRAM) as s:
        s.settimeout(5)
        s.sendto(dns.query("web-0.web.default.svc.cluster.local"), (ip, host_port(53)))
        assert dns.parse_reply(s.recv(512)) == (0, [p0])
    assert "web" in kc("get", "sts").stdout
    assert "roll out complete" in kc("rollout", "status", "sts/web", "--timeout", "30s").stdout
    kc("rollout", "restart", "sts/web")  # a new template: the ordinals are replaced, highest first
    out = kc("rollout", "status", "sts/web", "--timeout", "60s").stdout
    assert "roll out complete" in out
    assert "roll out complete" in kc("rollout", "status", "sts/web").stdout
    # a CronJob's Jobs run to completion
    _until(lambda: any(j.get("status", {}).get("succeeded") for j in json.loads(kc("get", "jobs", "-o", "json").stdout)["items"]
                       if j["metadata"]["name"].startswith("tick-")), 30)
    assert "@every 2s" in kc("get", "cronjobs").stdout
    # port-forward to web-0's own address
    pf = subprocess.Popen(["./kubectl", "port-forward", "pod/web-0", ":8000"], cwd=ws, env=env,
                          stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        line = pf.stdout.readline()
        local = int(line.split(":")[1].split()[0])
        assert "Directory listing" in _get(f"http://127.0.0.1:{local}/")
    finally:
        pf.terminate()
        pf.wait(10)
    kc("scale", "sts/web", "--replicas", "1")
    _until(lambda: "web-1" not in pods(), 30)
    kc("delete", "cronjob", "tick")


def test_init_and_multi_container_pod_on_a_real_cluster(cluster):
    ws, env, kc, summary = cluster
    (ws / "multi.json").write_text(json.dumps({
        "apiVersion": "v1", "kind": "Pod", "metadata": {"name": "multi"},
        "spec": {"restartPolicy": "Never",
                 "initContainers": [{"name": "prep", "image": "busybox",
                                     "command": ["sh", "-c", "echo prepared > $(TK8S_VOLUME_SHARED)/ready"]}],
                 "containers": [{"name": "app", "image": "busybox", "command": ["sh", "-c", "cat $(TK8S_VOLUME_SHARED)/ready"]},
                                {"name": "helper", "image": "busybox", "command": ["sh", "-c", "echo helper ran"]}],
                 "volumes": [{"name": "shared", "emptyDir": {}}]}}))
    kc("apply", "-f", "multi.json")
    _until(lambda: json.loads(kc("get", "pod", "multi", "-o", "json").stdout)["status"].get("phase") == "Succeeded", 30)
    assert kc("logs", "multi").stdout.strip() == "prepared"
    st = json.loads(kc("get", "pod", "multi", "-o", "json").stdout)["status"]
    assert [c["name"] for c in st["containerStatuses"]] == ["app", "helper"]
    assert [c["name"] for c in st["initContainerStatuses"]] == ["prep"]
    assert kc("logs", "multi", "-c", "helper").stdout.strip() == "helper ran"
    assert kc("logs", "multi", "-c", "nope", check=False).returncode != 0


def test_readiness_and_liveness_probes_on_a_real_cluster(cluster):
    """A pod is Ready only once its readiness probe passes (and only then a Service endpoint); a
    failing liveness probe restarts it."""
    ws, env, kc, summary = cluster
    (ws / "probes.json").write_text(json.dumps({"apiVersion": "v1", "kind": "List", "items": [
        {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "slow", "labels": {"app": "slow"}},
         "spec": {"containers": [{"name": "c", "image": "busybox",
                                  "command": ["sh", "-c", "sleep 4; touch marker; sleep 60"],
                                  "readinessProbe": {"exec": {"command": ["test", "-f", "marker"]}, "periodSeconds": 0.2,
                                                     "failureThreshold": 1}}]}},
        {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "sick"},
         "spec": {"containers": [{"name": "c", "image": "busybox", "command": ["sleep", "60"],
                                  "livenessProbe": {"exec": {"command": ["false"]}, "periodSeconds": 0.2,
                                                    "failureThreshold": 2}}]}}]}))
    kc("apply", "-f", "probes.json")

    def pod(n):
        return json.loads(kc("get", "pod", n, "-o", "json").stdout)

    def ready(n):
        return next((c["status"] for c in pod(n)["status"].get("conditions", []) if c["type"] == "Ready"), None)

    _until(lambda: pod("slow")["status"].get("phase") == "Running", 20)
    assert ready("slow") == "False"
    _until(lambda: ready("slow") == "True", 20)
    _until(lambda: pod("sick")["status"]["containerStatuses"][0]["restartCount"] >= 1, 30)


def test_kubectl_top_pods_from_the_metrics_api(cluster):
    ws, env, kc, summary = cluster
    (ws / "burn.json").write_text(json.dumps({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "burn"},
        "spec": {"containers": [{"name": "c", "image": "busybox", "command": ["sh", "-c", "while :; do :; done"]}]}}))
    kc("apply", "-f", "burn.json")

    def cpu_m():
        out = kc("top", "pods", check=False).stdout
        row = next((line.split() for line in out.splitlines() if line.startswith("burn ")), None)
        return int(row[1].rstrip("m")) if row else 0

    assert _until(lambda: cpu_m() > 300, 30)  # a busy loop uses most of a core
    kc("delete", "pod", "burn")


def test_rollout_history_and_undo_on_a_real_cluster(cluster):
    ws, env, kc, summary = cluster
    kc("create", "deployment", "hist", "--image", "nginx", "--replicas", "1")
    kc("rollout", "status", "deploy/hist", "--timeout", "60s")
    d = json.loads(kc("get", "deploy", "hist", "-o", "json").stdout)
    first = json.loads(json.dumps(d["spec"]["template"]))
    d["spec"]["template"]["metadata"].setdefault("annotations", {})["v"] = "2"
    (ws / "hist.json").write_text(json.dumps({k: v for k, v in d.items() if k != "status"}))
    kc("apply", "-f", "hist.json")
    kc("rollout", "status", "deploy/hist", "--timeout", "60s")
    hist = kc("rollout", "history", "deploy/hist").stdout
    assert "REVISION" in hist and "\n1 " in hist and "\n2 " in hist, hist
    assert len(json.loads(kc("get", "rs", "-o", "json").stdout)["items"]) >= 2
    kc("rollout", "undo", "deploy/hist")
    kc("rollout", "status", "deploy/hist", "--timeout", "60s")
    back = json.loads(kc("get", "deploy", "hist", "-o", "json").stdout)
    assert back["spec"]["template"] == first and back["metadata"]["annotations"]["deployment.kubernetes.io/revision"] == "3"


def test_pods_call_the_api_with_their_service_account(cluster):
    """A pod's ServiceAccount token is mounted (process pods: TK8S_SERVICEACCOUNT_TOKEN_FILE) and
    the API authorizes it by RBAC: listing pods fails until a RoleBinding grants view."""
    ws, env, kc, summary = cluster
    script = ("import json, os, urllib.request, urllib.error\n"
              "tok = open(os.environ['TK8S_SERVICEACCOUNT_TOKEN_FILE']).read()\n"
              "for path in ('/api/v1/namespaces/default/pods', '/api/v1/namespaces/default/secrets'):\n"
              "    req = urllib.request.Request(os.environ['TK8S_K8S_API'] + path, headers={'Authorization': 'Bearer ' + tok})\n"
              "    try:\n"
              "        print(path.rsplit('/', 1)[1], urllib.request.urlopen(req, timeout=5).status)\n"
              "    except urllib.error.HTTPError as e:\n"
              "        print(path.rsplit('/', 1)[1], e.code)\n")

    def run(name):
        (ws / f"{name}.json").write_text(json.dumps({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name},
            "spec": {"restartPolicy": "Never", "serviceAccountName": "reader",
                     "containers": [{"name": "c", "image": "python", "command": [sys.executable, "-c", script]}]}}))
        kc("apply", "-f", f"{name}.json")
        _until(lambda: json.loads(kc("get", "pod", name, "-o", "json").stdout)["status"].get("phase") == "Succeeded", 30)
        return kc("logs", name).stdout.split()

    (ws / "sa.json").write_text(json.dumps({"apiVersion": "v1", "kind": "ServiceAccount", "metadata": {"name": "reader"}}))
    kc("apply", "-f", "sa.json")
    assert run("before") == ["pods", "403", "secrets", "403"]
    (ws / "rb.json").write_text(json.dumps({"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "RoleBinding",
        "metadata": {"name": "reader-view"}, "roleRef": {"kind": "ClusterRole", "name": "view"},
        "subjects": [{"kind": "ServiceAccount", "name": "reader", "namespace": "default"}]}))
    kc("apply", "-f", "rb.json")
    assert run("after") == ["pods", "200", "secrets", "403"]


def test_kubectl_cp_both_ways(cluster, tmp_path_factory):
    ws, env, kc, summary = cluster
    (ws / "cp.json").write_text(json.dumps({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "store"},
        "spec": {"containers": [{"name": "c", "image": "busybox", "command": ["sleep", "60"]}]}}))
    kc("apply", "-f", "cp.json")
    _until(lambda: json.loads(kc("get", "pod", "store", "-o", "json").stdout)["status"].get("phase") == "Running")
    src = tmp_path_factory.mktemp("cpsrc")
    (src / "data").mkdir()
    (src / "data" / "weights.bin").write_bytes(bytes(range(256)) * 100)
    (src / "data" / "cfg.txt").write_text("lr=3e-4\n")
    kc("cp", str(src / "data"), "store:incoming")
    r = kc("exec", "store", "--", "sh", "-c", "wc -c < incoming/weights.bin; cat incoming/cfg.txt")
    assert r.stdout.split() == ["25600", "lr=3e-4"], r.stdout
    back = tmp_path_factory.mktemp("cpback") / "out"
    kc("cp", "store:incoming", str(back))
    assert (back / "weights.bin").read_bytes() == bytes(range(256)) * 100 and (back / "cfg.txt").read_text() == "lr=3e-4\n"


def test_configmap_volume_updates_reach_a_running_pod(cluster):
    """kubectl apply of a changed ConfigMap: the running pod's volume shows the new data within a
    sync period, and a lifecycle preStop hook runs when the pod is deleted."""
    ws, env, kc, summary = cluster
    cm = lambda v: {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "live"}, "data": {"mode": v}}
    (ws / "cm.json").write_text(json.dumps(cm("slow")))
    kc("apply", "-f", str(ws / "cm.json"))
    (ws / "pod.json").write_text(json.dumps({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "watcher"}, "spec": {
        "terminationGracePeriodSeconds": 5,
        "containers": [{"name": "c", "command": ["sh", "-c", "sleep 300"],
                        "volumeMounts": [{"name": "cfg", "mountPath": "/etc/live"}],
                        "lifecycle": {"preStop": {"exec": {"command": ["sh", "-c", "echo bye > $TK8S_VOLUME_SCRATCH/bye"]}}}}],
        "volumes": [{"name": "cfg", "configMap": {"name": "live"}}, {"name": "scratch", "hostPath": {
            "path": str(ws / "scratch"), "type": "DirectoryOrCreate"}}]}}))
    kc("apply", "-f", str(ws / "pod.json"))
    read = lambda: kc("exec", "watcher", "--", "sh", "-c", "cat $TK8S_VOLUME_CFG/mode", check=False).stdout
    assert _until(lambda: read() == "slow", timeout=30)
    (ws / "cm.json").write_text(json.dumps(cm("fast")))
    kc("apply", "-f", str(ws / "cm.json"))
    assert _until(lambda: read() == "fast", timeout=20)
    kc("delete", "pod", "watcher")
    assert _until(lambda: (ws / "scratch" / "bye").exists(), timeout=20)


def test_gpu_pod_waits_for_a_terminating_pods_gpus(cluster):
    """A deleted GPU pod is Terminating and keeps its GPUs through its grace period (a trainer
    writing a checkpoint); a new pod that needs them waits and starts once they are free."""
    ws, env, kc, summary = cluster
    node = json.loads(kc("get", "nodes", "-o", "json").stdout)["items"][0]
    nn, gpus = node["metadata"]["name"], int(node["status"]["allocatable"]["amd.com/gpu"])
    pod = lambda name, cmd, grace: {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name}, "spec": {
        "nodeSelector": {"kubernetes.io/hostname": nn}, "terminationGracePeriodSeconds": grace,
        "containers": [{"name": "c", "command": ["sh", "-c", cmd], "resources": {"limits": {"amd.com/gpu": str(gpus)}}}]}}
    (ws / "old.json").write_text(json.dumps(pod("old", "trap '' TERM; while true; do sleep 0.1; done", 3)))
    kc("apply", "-f", str(ws / "old.json"))
    _until(lambda: json.loads(kc("get", "pod", "old", "-o", "json").stdout)["status"].get("phase") == "Running", 30)
    kc("delete", "pod", "old", "--wait=false")
    t0 = time.monotonic()
    assert any(l.split()[:1] == ["old"] and "Terminating" in l for l in kc("get", "pods").stdout.splitlines())
    (ws / "new.json").write_text(json.dumps(pod("new", "sleep 60", 30)))
    kc("apply", "-f", str(ws / "new.json"))
    _until(lambda: json.loads(kc("get", "pod", "new", "-o", "json").stdout)["status"].get("phase") == "Running", 30)
    assert time.monotonic() - t0 > 1.5  # it waited for the old pod's grace period
    assert json.loads(kc("get", "pod", "new", "-o", "json").stdout)["status"]["phase"] == "Running"


def test_logs_previous_selector_and_all_containers(cluster):
    ws, env, kc, summary = cluster
    (ws / "crash.json").write_text(json.dumps({"apiVersion": "v1", "kind": "Pod",
        "metadata": {"name": "crashy", "labels": {"app": "crashy"}}, "spec": {"restartPolicy": "Always", "containers": [
            {"name": "main", "command": ["sh", "-c", "n=$(cat $TK8S_VOLUME_S/n 2>/dev/null || echo 0); n=$((n+1)); "
                                                     "echo $n > $TK8S_VOLUME_S/n; echo run $n; "
                                                     "if [ $n -lt 2 ]; then exit 1; fi; sleep 60"],
             "volumeMounts": [{"name": "s", "mountPath": "/s"}]},
            {"name": "side", "command": ["sh", "-c", "echo from side; sleep 60"]}],
            "volumes": [{"name": "s", "emptyDir": {}}]}}))
    kc("apply", "-f", str(ws / "crash.json"))
    assert _until(lambda: kc("logs", "crashy", check=False).stdout == "run 2\n", 30)
    assert kc("logs", "crashy", "-p").stdout == "run 1\n"
    out = kc("logs", "-l", "app=crashy", "--prefix").stdout
    assert "[pod/crashy/main] run 2" in out and "[pod/crashy/side] from side" in out
    assert "from side" in kc("logs", "crashy", "--all-containers").stdout
    r = kc("logs", "crashy", "-c", "side", "--previous", check=False)
    assert r.returncode != 0 and "previous terminated container" in r.stderr
