"""A pod cannot reach the cluster's credentials, and the API answers no one it does not know
(VERDICT r3 "next round" 1; controlplane/authn.py, native/tools/gpujail.h, agent._jail_layers).

The reference ran its workloads in Docker containers with their own root file system
(/root/reference/ansible/roles/rancherhost/tasks/main.yml:26-34), so a workload never saw the
machine's Rancher credentials. tk8s process pods run as the node agent's user; the Landlock jail
is what keeps the workspace's ``.tk8s/`` (admin kubeconfig and token, the cluster SSH key, other
pods' ServiceAccount tokens) out of their reach."""
import json
import os
import shutil
import subprocess
import sys
import time
import urllib.error
import urllib.request
from pathlib import Path

import pytest

from tritonk8ssupervisor_amd.agent.runtime import gpu_jail
from tritonk8ssupervisor_amd.controlplane.client import ApiError, Client, client_from_kubeconfig

from test_controlplane import _env, _join, _start, _stop

REPO = Path(__file__).resolve().parents[1]

needs_jail = pytest.mark.skipif(not gpu_jail()[0], reason="Landlock unavailable on this kernel")


@pytest.fixture(scope="module")
def cluster(tmp_path_factory):
    from tritonk8ssupervisor_amd.orchestrator import init_workspace

    ws = tmp_path_factory.mktemp("iso")
    init_workspace(ws)
    for f in ("setup.sh", "tk8s", "kubectl"):
        shutil.copy2(REPO / f, ws / f)
    env = dict(os.environ, PYTHONPATH=str(REPO), TK8S_PYTHON=sys.executable, TK8S_FAKE_GPUS="8")
    env.pop("TK8S_FAULTS", None)
    r = subprocess.run(["./setup.sh", "--yes", "--json", "--port", "0", "--nodes", "2", "--rccl", "off"], cwd=ws,
                       env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    summary = json.loads(r.stdout.strip().splitlines()[-1])

    def kc(*a, check=True, stdin=None):
        p = subprocess.run(["./kubectl", *a], cwd=ws, env=env, capture_output=True, text=True, timeout=120, input=stdin)
        if check:
            assert p.returncode == 0, f"kubectl {' '.join(a)}: {p.stdout}{p.stderr}"
        return p

    yield ws, env, kc, summary
    subprocess.run(["./setup.sh", "-c", "--yes"], cwd=ws, env=env, capture_output=True, timeout=120)


def _pod(kc, name, script, node=None, gpus=0, env=None):
    spec = {"restartPolicy": "Never", "containers": [{"name": "c", "command": ["sh", "-c", script],
                                                      "env": [{"name": k, "value": v} for k, v in (env or {}).items()]}]}
    if node:
        spec["nodeName"] = node
    if gpus:
        spec["containers"][0]["resources"] = {"limits": {"amd.com/gpu": gpus}}
    kc("apply", "-f", "-", stdin=json.dumps({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name}, "spec": spec}))


def _wait(kc, name, phases=("Succeeded", "Failed"), timeout=60.0):
    deadline = time.monotonic() + timeout
    while True:
        o = json.loads(kc("get", "pod", name, "-o", "json").stdout)
        if o.get("status", {}).get("phase") in phases:
            return o
        assert time.monotonic() < deadline, o.get("status")
        time.sleep(0.1)


PROBE = r"""
for f in "$KC" "$KEY" "$TOKEN_OF_VICTIM" "$REG_URL" "$ADMIN"; do
  if cat "$f" > /dev/null 2>&1; then echo "read $f"; else echo "denied $f"; fi
done
if cat "$TK8S_SERVICEACCOUNT_TOKEN_FILE" > /dev/null 2>&1; then echo "own-token ok"; fi
if (echo x > "$TK8S_HOME/pwned-by-pod") 2> /dev/null || mv "$TK8S_HOME/setup.sh" "$TK8S_HOME/setup.moved" 2> /dev/null; then
  echo "wrote install"; else echo "install read-only"; fi
if cat "$TK8S_HOME/tritonk8ssupervisor_amd/__init__.py" > /dev/null; then echo "install readable"; fi
echo hi > "$TMPDIR/scratch" && cat "$TMPDIR/scratch" > /dev/null && echo "tmpdir ok"
echo "isolation=$TK8S_GPU_ISOLATION"
"""


@needs_jail
def test_a_pod_cannot_read_the_cluster_credentials(cluster):
    ws, env, kc, _ = cluster
    st = ws / ".tk8s"
    _pod(kc, "victim", "sleep 30", node="kubenode1")
    v = _wait(kc, "victim", ("Running",))
    victim_dir = Path(v["metadata"]["annotations"]["tk8s.amd.com/log-path"]).parent
    assert (victim_dir / "serviceaccount" / "token").exists()
    files = {"KC": str(st / "kubeconfig.json"), "KEY": str(next((st / "keys").glob("*"))),
             "TOKEN_OF_VICTIM": str(victim_dir / "serviceaccount" / "token"),
             "REG_URL": str(st / "machines" / "kubenode2" / "run" / "registration-url"),
             "ADMIN": str(st / "admin-token")}
    for f in files.values():
        assert Path(f).exists(), f
    _pod(kc, "thief", PROBE, node="kubenode2", env=files)
    o = _wait(kc, "thief")
    out = kc("logs", "thief").stdout
    assert o["status"]["phase"] == "Succeeded", out
    for f in files.values():
        assert f"denied {f}" in out, out
    assert "own-token ok" in out and "install read-only" in out and "install readable" in out and "tmpdir ok" in out, out
    assert "isolation=landlock:" in out, out
    assert not (REPO / "pwned-by-pod").exists()
    ann = o["metadata"]["annotations"]["tk8s.amd.com/gpu-isolation"]
    assert "node state denied" in ann and str(st) in ann, ann
    # kubectl exec runs under the same jail as the pod
    r = kc("exec", "victim", "--", "cat", files["KC"], check=False)
    assert r.returncode != 0 and "Permission denied" in (r.stderr + r.stdout)
    r = kc("exec", "victim", "--", "cat", files["TOKEN_OF_VICTIM"])
    assert r.stdout.strip()
    kc("delete", "pod", "victim", "thief", "--grace-period", "0", "--force", check=False)


@needs_jail
def test_a_pod_cannot_mknod_a_device(cluster):
    _ws, _env, kc, _ = cluster
    _pod(kc, "mknod", 'mknod "$TMPDIR/gpu" c 226 128 2>&1 && echo made || echo refused')
    _wait(kc, "mknod")
    assert "refused" in kc("logs", "mknod").stdout
    kc("delete", "pod", "mknod", check=False)


def test_anonymous_callers_get_discovery_and_nothing_else(cluster):
    ws, _env, kc, summary = cluster
    kc("create", "configmap", "cfg", "--from-literal", "k=v")
    _pod(kc, "logger", "echo secret-log-line")
    _wait(kc, "logger")
    kcfg = json.loads((ws / ".tk8s" / "kubeconfig.json").read_text())
    server = kcfg["clusters"][0]["cluster"]["server"]
    base = summary["api"]

    def code(url, method="GET", data=None):
        try:
            return urllib.request.urlopen(urllib.request.Request(url, method=method, data=data), timeout=10).status
        except urllib.error.HTTPError as e:
            return e.code

    for path in ("/api/v1/namespaces/default/pods", "/api/v1/namespaces/default/pods/logger/log",
                 "/api/v1/namespaces/default/configmaps", "/api/v1/namespaces/default/secrets", "/api/v1/nodes"):
        assert code(server + path) == 401, path
    assert code(f"{base}/env/{summary['project']}/kubernetes/kubectl") == 401  # the kubeconfig holds the token
    assert code(f"{base}/v1/kv/x", "PUT", b"v") == 401
    assert code(f"{base}/v1/registrationtokens?projectId={summary['project']}", "POST", b"{}") == 401
    assert code(f"{base}/v2-beta/projects", "POST", b"{}") == 401
    for ok in ("/healthz", "/version", "/v2-beta/projectTemplates"):
        assert code(base + ok) == 200, ok
    for ok in ("/api", "/apis", "/api/v1", "/apis/apps/v1"):
        assert code(server + ok) == 200, ok
    # the environment's token reads them
    k = client_from_kubeconfig(kcfg)
    assert "secret-log-line" in k.get(k.k8s("/api/v1/namespaces/default/pods/logger/log"), raw=True)


@needs_jail
def test_a_hostpath_into_the_node_state_is_refused(cluster):
    """a hostPath volume at or beneath a denied path (the workspace's .tk8s/) would
    win over the jail's deny (the most specific layer decides) and re-open the admin token: the
    agent refuses the pod, whatever the namespace's Pod Security level. One above it is fine."""
    ws, env, kc, _ = cluster
    st = ws / ".tk8s"
    for name, path in (("grab-state", st), ("grab-machine", st / "machines" / "kubenode1")):
        pod = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name}, "spec": {
            "restartPolicy": "Never", "nodeName": "kubenode1",
            "volumes": [{"name": "s", "hostPath": {"path": str(path)}}],
            "containers": [{"name": "c", "command": ["sh", "-c", f"cat {st}/admin-token"],
                            "volumeMounts": [{"name": "s", "mountPath": str(path)}]}]}}
        kc("apply", "-f", "-", stdin=json.dumps(pod))
        o = _wait(kc, name)
        assert o["status"]["phase"] == "Failed", o["status"]
        assert "HostPathDenied" in json.dumps(o["status"]), o["status"]
    data = ws / "shared-data"
    data.mkdir(exist_ok=True)
    pod = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "data-ok"}, "spec": {
        "restartPolicy": "Never", "nodeName": "kubenode1",
        "volumes": [{"name": "s", "hostPath": {"path": str(data)}}],
        "containers": [{"name": "c", "command": ["sh", "-c", f"echo ok > {data}/x && cat {data}/x"],
                        "volumeMounts": [{"name": "s", "mountPath": str(data)}]}]}}
    kc("apply", "-f", "-", stdin=json.dumps(pod))
    assert _wait(kc, "data-ok")["status"]["phase"] == "Succeeded"


def test_node_tokens_reach_their_own_node_only(tmp_path):
    """NodeRestriction + the Node authorizer (authn.node_allows)."""
    p, c = _start(tmp_path)
    try:
        proj = _env(c)
        n1, _ = _join(c, proj["id"], "kubenode1", ngpu=0)
        n2, _ = _join(c, proj["id"], "kubenode2", ngpu=0)
        k = client_from_kubeconfig(c.get(f"/env/{proj['id']}/kubernetes/kubectl", query={"format": "json"}))
        k.post(k.k8s("/api/v1/namespaces/default/secrets"), {"metadata": {"name": "s1"}, "stringData": {"a": "b"}})
        k.post(k.k8s("/api/v1/namespaces/default/configmaps"), {"metadata": {"name": "c1"}, "data": {"a": "b"}})
        k.post(k.k8s("/api/v1/namespaces/default/pods"), {"metadata": {"name": "p1"}, "spec": {
            "nodeName": "kubenode1", "containers": [{"name": "c", "command": ["true"], "envFrom": [
                {"secretRef": {"name": "s1"}}, {"configMapRef": {"name": "c1"}}]}]}})

        def status(client, method, path, body=None):
            try:
                client.request(method, client.k8s(path), body=body)
                return 200
            except ApiError as e:
                return e.status

        # its own node: yes; another node: 403
        assert status(n1, "PATCH", "/api/v1/nodes/kubenode1", {"metadata": {"labels": {"x": "1"}}}) == 200
        assert status(n1, "PATCH", "/api/v1/nodes/kubenode2", {"metadata": {"labels": {"x": "1"}}}) == 403
        assert status(n1, "PUT", "/api/v1/nodes/kubenode2/status", {}) in (401, 403)
        # pods: no creating any; status and deletion only of pods bound to it
        assert status(n1, "POST", "/api/v1/namespaces/default/pods",
                      {"metadata": {"name": "evil"}, "spec": {"containers": [{"name": "c", "command": ["id"]}]}}) == 403
        assert status(n1, "POST", "/api/v1/namespaces/kube-system/pods",
                      {"metadata": {"name": "evil"}, "spec": {"containers": [{"name": "c", "command": ["id"]}]}}) == 403
        assert status(n2, "PUT", "/api/v1/namespaces/default/pods/p1/status", {"status": {"phase": "Failed"}}) == 403
        assert status(n1, "PUT", "/api/v1/namespaces/default/pods/p1/status", {"status": {"phase": "Running"}}) == 200
        assert status(n2, "DELETE", "/api/v1/namespaces/default/pods/p1") == 403
        # Secrets / ConfigMaps: only those a pod bound to the node uses, never a list
        assert status(n1, "GET", "/api/v1/namespaces/default/secrets/s1") == 200
        assert status(n1, "GET", "/api/v1/namespaces/default/configmaps/c1") == 200
        assert status(n2, "GET", "/api/v1/namespaces/default/secrets/s1") == 403
        assert status(n2, "GET", "/api/v1/namespaces/default/configmaps/c1") == 403
        assert status(n1, "GET", "/api/v1/namespaces/default/secrets") == 403
        assert status(n1, "GET", "/api/v1/namespaces/default/pods/p1/log") == 403
        # reads a kubelet needs
        assert status(n2, "GET", "/api/v1/pods") == 200 and status(n2, "GET", "/api/v1/namespaces/default/services") == 200
        assert status(n2, "GET", "/api/v1/nodes") == 200 and status(n2, "GET", "/api/v1/namespaces/default/endpoints") == 200
        # ... and nothing a kubelet's system:node role does not grant: no
        # workload specs, no RBAC, no Secret lists, no ServiceAccounts
        k.post(k.k8s("/apis/apps/v1/namespaces/default/deployments"), {"metadata": {"name": "d"}, "spec": {
            "replicas": 0, "selector": {"matchLabels": {"a": "d"}},
            "template": {"metadata": {"labels": {"a": "d"}}, "spec": {"containers": [{"name": "c", "command": ["true"]}]}}}})
        for path in ("/apis/apps/v1/namespaces/default/deployments", "/apis/apps/v1/namespaces/default/deployments/d",
                     "/apis/apps/v1/deployments", "/apis/rbac.authorization.k8s.io/v1/namespaces/default/roles",
                     "/apis/rbac.authorization.k8s.io/v1/namespaces/default/rolebindings",
                     "/apis/rbac.authorization.k8s.io/v1/clusterroles", "/apis/rbac.authorization.k8s.io/v1/clusterrolebindings",
                     "/api/v1/secrets", "/api/v1/namespaces/default/secrets", "/api/v1/namespaces/default/serviceaccounts",
                     "/api/v1/namespaces/default/configmaps", "/apis/batch/v1/namespaces/default/jobs",
                     "/apis/apps/v1/namespaces/default/statefulsets", "/api/v1/namespaces/default/persistentvolumeclaims"):
            assert status(n1, "GET", path) == 403, path
        # a PVC and the Job of a pod bound to it: yes; of another node's pod: no
        k.post(k.k8s("/api/v1/namespaces/default/persistentvolumeclaims"), {"metadata": {"name": "data"}, "spec": {
            "accessModes": ["ReadWriteOnce"], "resources": {"requests": {"storage": "1Gi"}}}})
        k.post(k.k8s("/api/v1/namespaces/default/pods"), {"metadata": {"name": "p2"}, "spec": {
            "nodeName": "kubenode2", "volumes": [{"name": "v", "persistentVolumeClaim": {"claimName": "data"}}],
            "containers": [{"name": "c", "command": ["true"]}]}})
        assert status(n2, "GET", "/api/v1/namespaces/default/persistentvolumeclaims/data") == 200
        assert status(n1, "GET", "/api/v1/namespaces/default/persistentvolumeclaims/data") == 403
        # node tokens do not open the Rancher side either
        nc = Client(c.base, token=n1.token)
        with pytest.raises(ApiError) as ei:
            nc.get(f"/env/{proj['id']}/kubernetes/kubectl", query={"format": "json"})
        assert ei.value.status == 403
        with pytest.raises(ApiError) as ei:
            nc.post("/v1/registrationtokens", query={"projectId": proj["id"]})
        assert ei.value.status == 403
    finally:
        _stop(p)


@needs_jail
def test_a_pod_without_a_pid_namespace_cannot_signal_the_agent(tmp_path):
    """On a node without user namespaces (the GPU tier) a CPU pod shares the host's PID namespace,
    as GPU pods always do: the jail scopes its signals to the pod (Landlock ABI >= 6), so it
    cannot kill the node agent or another pod, while signalling its own processes still works."""
    from tritonk8ssupervisor_amd.agent.runtime import jail_signal_scoping
    from tritonk8ssupervisor_amd.orchestrator import init_workspace

    if not jail_signal_scoping():
        pytest.skip("Landlock ABI < 6: no signal scoping on this kernel")
    init_workspace(tmp_path)
    for f in ("setup.sh", "tk8s", "kubectl"):
        shutil.copy2(REPO / f, tmp_path / f)
    env = dict(os.environ, PYTHONPATH=str(REPO), TK8S_PYTHON=sys.executable, TK8S_FAKE_GPUS="1",
               TK8S_POD_ISOLATION="none")
    env.pop("TK8S_FAULTS", None)
    try:
        r = subprocess.run(["./setup.sh", "--yes", "--json", "--port", "0", "--nodes", "1", "--rccl", "off"],
                           cwd=tmp_path, env=env, capture_output=True, text=True, timeout=180)
        assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
        agent = json.loads((tmp_path / ".tk8s" / "machines" / "kubenode1" / "run" / "agent.pid").read_text())["pid"]
        kc = lambda *a, stdin=None: subprocess.run(["./kubectl", *a], cwd=tmp_path, env=env, capture_output=True,
                                                   text=True, timeout=60, input=stdin)
        script = (f"if kill -0 {agent} 2>/dev/null; then echo agent-signalled; else echo agent-refused; fi; "
                  "sleep 30 & if kill $! 2>/dev/null; then echo own-ok; fi")
        kc("apply", "-f", "-", stdin=json.dumps({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "sig"},
                                                  "spec": {"restartPolicy": "Never", "containers": [
                                                      {"name": "c", "command": ["sh", "-c", script]}]}}))
        _wait(lambda *a, **k: kc(*a), "sig")
        out = kc("logs", "sig").stdout
        assert "agent-refused" in out and "own-ok" in out, out
        d = kc("describe", "pod", "sig").stdout
        assert "signals scoped to the pod" in d, d
    finally:
        subprocess.run(["./setup.sh", "-c", "--yes"], cwd=tmp_path, env=env, capture_output=True, timeout=120)


@needs_jail
def test_a_pod_cannot_plant_code_for_the_operator(cluster):
    """What the operator's next login or bring-up would run is out of a pod's reach: its home is
    read-only to pods (shell start-up files, ~/.local/bin on the PATH, the user site-packages),
    tk8s's parse/rewrite caches and the host registry are denied -- while the workloads' own
    caches under ~/.cache stay writable."""
    from tritonk8ssupervisor_amd.agent.agent import operator_state_dirs

    _ws, _env, kc, _ = cluster
    home = Path.home()
    tag = f"tk8s-test-{os.getpid()}"
    targets = {"RC": str(home / f".{tag}rc"), "LOCALBIN": str(home / ".local" / "bin" / tag),
               "CACHE": str(operator_state_dirs()[0] / f"{tag}.marshal"),
               "REG": str(operator_state_dirs()[1] / tag), "OK": str(home / ".cache" / tag)}
    script = "".join(f'if (mkdir -p "$(dirname "${k}")" && echo x > "${k}") 2>/dev/null; then echo "{k}=wrote"; '
                     f'else echo "{k}=refused"; fi; ' for k in targets)
    try:
        _pod(kc, "planter", script, env=targets)
        o = _wait(kc, "planter")
        out = dict(x.split("=", 1) for x in kc("logs", "planter").stdout.split() if "=" in x)
        assert o["status"]["phase"] == "Succeeded", out
        assert out == {"RC": "refused", "LOCALBIN": "refused", "CACHE": "refused", "REG": "refused", "OK": "wrote"}, out
    finally:
        for f in targets.values():
            Path(f).unlink(missing_ok=True)
        kc("delete", "pod", "planter", "--grace-period", "0", "--force", check=False)
