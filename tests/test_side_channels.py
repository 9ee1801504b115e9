"""The control plane's side channels are scoped like its Kubernetes API (VERDICT r4 missing-1).

In the reference every environment is its own Rancher project, and hosts join it with a
registration token bound to its projectId (ansible/roles/ranchermaster/tasks/main.yml:37-49,
ansible/roles/rancherhost/tasks/main.yml:11-17). Here the KV rendezvous store (RCCL unique ids,
torch addresses), the change feed ``/v1/events``, ``/v1/cluster/status|wait``, ``/metrics`` and
``GET /v2-beta/projects`` keep that scope: a pod's ServiceAccount token reaches its own namespace's
keys only, a node token none of them, an environment's API token its own environment."""
from __future__ import annotations

import base64

import pytest

from tritonk8ssupervisor_amd.controlplane.client import ApiError, Client, client_from_kubeconfig
from test_controlplane import _env, _join, _start, _stop


@pytest.fixture
def two_envs(tmp_path):
    p, admin = _start(tmp_path)
    try:
        a, b = _env(admin, "env a"), _env(admin, "env b")
        ka = client_from_kubeconfig(admin.get(f"/env/{a['id']}/kubernetes/kubectl", query={"format": "json"}))
        kb = client_from_kubeconfig(admin.get(f"/env/{b['id']}/kubernetes/kubectl", query={"format": "json"}))
        for k in (ka, kb):
            for ns in ("team-a", "team-b"):
                k.post(k.k8s("/api/v1/namespaces"), {"metadata": {"name": ns}})
        yield admin, a, b, ka, kb
    finally:
        _stop(p)


def _sa_token(k, ns: str, name: str = "rank") -> str:
    try:
        k.post(k.k8s(f"/api/v1/namespaces/{ns}/serviceaccounts"), {"metadata": {"name": name}})
    except ApiError as e:
        assert e.status == 409
    sec = k.get(k.k8s(f"/api/v1/namespaces/{ns}/secrets/{name}-token"))
    return base64.b64decode(sec["data"]["token"]).decode()


def _status(fn, *a, **kw) -> int:
    try:
        fn(*a, **kw)
    except ApiError as e:
        return e.status
    return 200


def _kv(base: str, tok: str) -> Client:
    return Client(base, token=tok, timeout=10)


def test_a_service_account_reaches_only_its_own_namespace(two_envs):
    admin, a, b, ka, kb = two_envs
    victim = _kv(admin.base, _sa_token(ka, "team-a"))
    attacker_ns = _kv(admin.base, _sa_token(ka, "team-b"))
    attacker_env = _kv(admin.base, _sa_token(kb, "team-a"))  # same namespace name, other environment
    # the fabric Job's key, exactly as a rank writes it ($TK8S_KV_URL/<job>/uid)
    victim.put("/v1/kv/rccl-allreduce-1/uid", "victim-unique-id")
    assert victim.get("/v1/kv/rccl-allreduce-1/uid", raw=True) == "victim-unique-id"
    # another namespace of the same environment, or the same namespace of another one: its own
    # (empty) keyspace -- the key is not there, and writing it does not touch the victim's
    for other in (attacker_ns, attacker_env):
        assert _status(other.get, "/v1/kv/rccl-allreduce-1/uid", raw=True) == 404
        other.put("/v1/kv/rccl-allreduce-1/uid", "attacker-unique-id")
        other.delete("/v1/kv/rccl-allreduce-1/uid")
    assert victim.get("/v1/kv/rccl-allreduce-1/uid", raw=True) == "victim-unique-id"
    # naming the victim's namespace explicitly is refused
    assert _status(attacker_ns.get, "/v1/kv/rccl-allreduce-1/uid", query={"namespace": "team-a"}, raw=True) == 403
    assert _status(attacker_ns.put, "/v1/kv/rccl-allreduce-1/uid", "x", query={"namespace": "team-a"}) == 403
    # the environment's administrator reaches it by namespace; the server admin by project too
    k_admin = _kv(admin.base, ka.token)
    assert k_admin.get("/v1/kv/rccl-allreduce-1/uid", query={"namespace": "team-a"}, raw=True) == "victim-unique-id"
    assert _status(k_admin.get, "/v1/kv/rccl-allreduce-1/uid", query={"project": b["id"], "namespace": "team-a"},
                   raw=True) == 403
    assert admin.get("/v1/kv/rccl-allreduce-1/uid", query={"project": a["id"], "namespace": "team-a"},
                     raw=True) == "victim-unique-id"
    # deleting the environment drops its keyspace
    admin.delete(f"/v2-beta/projects/{b['id']}")
    assert admin.get("/v1/kv/rccl-allreduce-1/uid", query={"project": a["id"], "namespace": "team-a"},
                     raw=True) == "victim-unique-id"


def test_a_node_token_reaches_no_workload_keys(two_envs):
    admin, a, _b, ka, _kb = two_envs
    nc1, r1 = _join(admin, a["id"], "kubenode1", ngpu=0)
    nc2, r2 = _join(admin, a["id"], "kubenode2", ngpu=0)
    pod = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "rank0"},
           "spec": {"nodeName": "kubenode2", "containers": [{"name": "c", "command": ["sleep", "60"]}]}}
    ka.post(ka.k8s("/api/v1/namespaces/team-a/pods"), pod)
    sa = _kv(admin.base, _sa_token(ka, "team-a"))
    sa.put("/v1/kv/job/uid", "uid-of-team-a")
    n1, n2 = _kv(admin.base, r1["nodeToken"]), _kv(admin.base, r2["nodeToken"])
    # kubenode2 runs a pod of team-a, kubenode1 none: neither reads or writes the rendezvous keys
    # (pods of one namespace run on many nodes: a namespace cannot hold a node to its own pods')
    for n in (n1, n2):
        for ns in ("team-a", "team-b", None):
            q = {"namespace": ns} if ns else None
            assert _status(n.get, "/v1/kv/job/uid", query=q, raw=True) == 403
            assert _status(n.put, "/v1/kv/job/uid", "evil", query=q) == 403
    assert sa.get("/v1/kv/job/uid", raw=True) == "uid-of-team-a"


def test_cluster_status_events_metrics_and_projects_are_scoped(two_envs):
    admin, a, b, ka, kb = two_envs
    sa_a = _kv(admin.base, _sa_token(ka, "team-a"))
    env_a = _kv(admin.base, ka.token)
    # /v1/cluster/status|wait: the caller's own environment; another one is 403
    assert sa_a.get("/v1/cluster/status")["project"] == a["id"]
    assert env_a.get("/v1/cluster/status", query={"project": a["id"]})["project"] == a["id"]
    for c in (sa_a, env_a):
        assert _status(c.get, "/v1/cluster/status", query={"project": b["id"]}) == 403
        assert _status(c.get, "/v1/cluster/wait", query={"project": b["id"], "timeout": "0.1"}) == 403
    assert admin.get("/v1/cluster/status", query={"project": b["id"]})["project"] == b["id"]
    # /v1/events: an environment sees its own objects, a ServiceAccount its namespace's, never Secrets
    kb.post(kb.k8s("/api/v1/namespaces/team-a/configmaps"), {"metadata": {"name": "b-secret-plan"}, "data": {}})
    ka.post(ka.k8s("/api/v1/namespaces/team-b/configmaps"), {"metadata": {"name": "a-other-ns"}, "data": {}})
    ka.post(ka.k8s("/api/v1/namespaces/team-a/configmaps"), {"metadata": {"name": "a-mine"}, "data": {}})
    names = lambda c: {e["name"] for e in c.get("/v1/events")["events"]}  # noqa: E731
    every = names(admin)
    assert {"b-secret-plan", "a-other-ns", "a-mine"} <= every
    in_a = names(env_a)
    assert "a-mine" in in_a and "a-other-ns" in in_a and "b-secret-plan" not in in_a
    mine = names(sa_a)
    assert "a-mine" in mine and "a-other-ns" not in mine and "b-secret-plan" not in mine
    assert not any(e["kind"] in ("secrets", "kv", "nodesecrets") for e in sa_a.get("/v1/events")["events"])
    # /metrics and the project list: the server admin or an environment's API token only
    assert _status(sa_a.get, "/metrics", raw=True) == 403
    text = env_a.get("/metrics", raw=True)
    assert f'project="{a["id"]}"' in text and f'project="{b["id"]}"' not in text
    assert f'project="{b["id"]}"' in admin.get("/metrics", raw=True)
    assert _status(sa_a.get, "/v2-beta/projects") == 403
    assert [p["id"] for p in env_a.get("/v2-beta/projects")["data"]] == [a["id"]]
    assert {p["id"] for p in admin.get("/v2-beta/projects")["data"]} == {a["id"], b["id"]}
    assert _status(env_a.get, f"/v2-beta/projects/{b['id']}") == 403
    assert _status(sa_a.get, f"/v2-beta/projects/{a['id']}") == 403
    assert env_a.get(f"/v2-beta/projects/{a['id']}")["id"] == a["id"]


def _pod(k, ns, name, job=None, node=None, sa="default"):
    md = {"name": name}
    if job:
        md["ownerReferences"] = [{"apiVersion": "batch/v1", "kind": "Job", "name": job, "uid": f"uid-{job}",
                                  "controller": True}]
    spec = {"serviceAccountName": sa, "containers": [{"name": "c", "command": ["sleep", "60"]}]}
    if node:
        spec["nodeName"] = node
    return k.post(k.k8s(f"/api/v1/namespaces/{ns}/pods"), {"apiVersion": "v1", "kind": "Pod", "metadata": md, "spec": spec})


def _bound(k, ns, pod, sa="default", **spec):
    body = {"spec": {"boundObjectRef": {"kind": "Pod", "name": pod["metadata"]["name"], "uid": pod["metadata"]["uid"]},
                     **spec}}
    return k.post(k.k8s(f"/api/v1/namespaces/{ns}/serviceaccounts/{sa}/token"), body)


def test_a_pod_bound_token_reaches_only_its_own_jobs_keys(two_envs):
    """the rendezvous is scoped to the Job. Two Jobs' pods -- same namespace, same
    ServiceAccount -- each reach their own Job's keys: another Job's rank can neither read nor
    overwrite ``rccl-allreduce-X/uid``; the token dies with its pod."""
    admin, a, _b, ka, _kb = two_envs
    pa = _pod(ka, "team-a", "rccl-x-0", job="rccl-allreduce-x")
    pb = _pod(ka, "team-a", "other-0", job="other-job")
    ta, tb = _bound(ka, "team-a", pa), _bound(ka, "team-a", pb)
    assert ta["kind"] == "TokenRequest" and ta["status"]["token"].startswith("tk8sb.")
    assert ta["spec"]["audiences"] and 3500 <= ta["spec"]["expirationSeconds"] <= 3600
    ra, rb = _kv(admin.base, ta["status"]["token"]), _kv(admin.base, tb["status"]["token"])
    ra.put("/v1/kv/rccl-allreduce-x/uid", "the-real-unique-id")
    assert ra.get("/v1/kv/rccl-allreduce-x/uid", raw=True) == "the-real-unique-id"
    # the other Job's pod: its own (empty) keyspace; its writes never reach the fabric Job's key
    assert _status(rb.get, "/v1/kv/rccl-allreduce-x/uid", raw=True) == 404
    rb.put("/v1/kv/rccl-allreduce-x/uid", "forged")
    rb.delete("/v1/kv/rccl-allreduce-x/uid")
    assert ra.get("/v1/kv/rccl-allreduce-x/uid", raw=True) == "the-real-unique-id"
    # naming the other Job's keyspace is refused
    assert _status(rb.get, "/v1/kv/rccl-allreduce-x/uid", query={"job": "rccl-allreduce-x"}, raw=True) == 403
    # the legacy namespace-wide token of the same ServiceAccount does not see the Job's key either
    legacy = _kv(admin.base, _sa_token(ka, "team-a", "default"))
    assert _status(legacy.get, "/v1/kv/rccl-allreduce-x/uid", raw=True) == 404
    # the environment's administrator reaches the Job's keyspace by name
    assert _kv(admin.base, ka.token).get("/v1/kv/rccl-allreduce-x/uid", query={"namespace": "team-a", "job":
                                                                               "rccl-allreduce-x"}, raw=True) == \
        "the-real-unique-id"
    # a pod no Job owns shares its namespace's keys (as a legacy token does)
    free = _kv(admin.base, _bound(ka, "team-a", _pod(ka, "team-a", "solo"))["status"]["token"])
    free.put("/v1/kv/shared/x", "1")
    assert legacy.get("/v1/kv/shared/x", raw=True) == "1"
    # deleting the pod revokes its token
    ka.delete(ka.k8s("/api/v1/namespaces/team-a/pods/rccl-x-0"), query={"gracePeriodSeconds": "0"})
    import time

    deadline = time.monotonic() + 10
    while _status(ra.get, "/v1/kv/rccl-allreduce-x/uid", raw=True) != 401 and time.monotonic() < deadline:
        time.sleep(0.05)
    assert _status(ra.get, "/v1/kv/rccl-allreduce-x/uid", raw=True) == 401


def test_token_requests_are_bound_checked_and_node_restricted(two_envs):
    admin, a, _b, ka, _kb = two_envs
    nc1, r1 = _join(admin, a["id"], "kubenode1", ngpu=0)
    _join(admin, a["id"], "kubenode2", ngpu=0)
    mine = _pod(ka, "team-a", "on-1", node="kubenode1")
    theirs = _pod(ka, "team-a", "on-2", node="kubenode2")
    n1 = Client(admin.base, token=r1["nodeToken"], prefix=ka.prefix, timeout=10)
    assert _bound(n1, "team-a", mine)["status"]["token"]
    assert _status(_bound, n1, "team-a", theirs) == 403            # a pod bound to another node
    _sa_token(ka, "team-a", "other-sa")
    assert _status(_bound, n1, "team-a", mine, sa="other-sa") == 403  # not the pod's own ServiceAccount
    assert _status(n1.post, n1.k8s("/api/v1/namespaces/team-a/serviceaccounts/default/token"), {"spec": {}}) == 403
    stale = {**mine, "metadata": {**mine["metadata"], "uid": "not-the-uid"}}
    assert _status(_bound, ka, "team-a", stale) == 409
    # an audience this server does not serve: the token is not accepted here
    odd = _bound(ka, "team-a", mine, audiences=["https://vault.example"])["status"]["token"]
    assert _status(_kv(admin.base, odd).get, "/v1/kv/x", raw=True) == 401
    # a forged signature is nobody
    good = _bound(ka, "team-a", mine)["status"]["token"]
    assert _status(_kv(admin.base, good[:-2] + ("AA" if not good.endswith("AA") else "BB")).get, "/v1/kv/x", raw=True) == 401


def test_an_expired_bound_token_is_refused(monkeypatch):
    """Expiry, pod uid and audience checks of authn._bound, on the class itself (no server)."""
    import time

    from tritonk8ssupervisor_amd.controlplane.authn import Authentication

    pod = {"metadata": {"name": "p0", "namespace": "ns", "uid": "u1",
                        "ownerReferences": [{"kind": "Job", "name": "j1"}]}}

    class Store:
        def get(self, kind, key):
            return pod if kind == "pods" and key.endswith("p0") else None

    auth = Authentication()
    auth.store, auth.state_dir = Store(), None
    tok, exp = auth.issue_bound_token("1a1", "ns", "default", pod, ["tk8s"], 60)  # clamped to 10 min
    assert 590 <= exp - time.time() <= 600
    assert auth._bound(tok) == ("sa", "1a1", "ns", "default", {"pod": "p0", "uid": "u1", "job": "j1"})
    real = time.time
    monkeypatch.setattr(time, "time", lambda: real() + 601)
    assert auth._bound(tok) is None  # expired
    monkeypatch.setattr(time, "time", real)
    pod["metadata"]["uid"] = "u2"  # the pod was deleted and re-created under the same name
    assert auth._bound(tok) is None
