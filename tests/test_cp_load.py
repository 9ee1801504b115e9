"""The control plane under load, and across a kill.

Load: 8 nodes, 2,000 ConfigMaps, 400 pods plus a 100-replica Deployment (500 pods), 50 concurrent
watches that must each see every ConfigMap, then a rolling update of the 100 replicas -- with
request latency (p50/p99) and the server's resident set recorded (``TK8S_LOAD_OUT`` writes them
to a file: profiles/r4_cp_load/). Restart: a control plane SIGKILLed mid-rollout comes back from
its snapshot + write-ahead journal (controlplane/store.py) with every acknowledged write, hands
out no name twice, and finishes the rollout with exactly the replicas asked for.

The nodes' kubelets are played by a thread that marks the pods bound to each node Running with
that node's own token (the Node authorizer's view: authn.node_allows) and confirms deletions."""
import json
import os
import signal
import threading
import time

import pytest

from tritonk8ssupervisor_amd.controlplane.client import ApiError, Client, client_from_kubeconfig

from test_controlplane import _env, _join, _start, _stop

DEPLOY = {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": "web"},
          "spec": {"replicas": 100, "selector": {"matchLabels": {"app": "web"}},
                   "strategy": {"rollingUpdate": {"maxSurge": "25%", "maxUnavailable": "25%"}},
                   "template": {"metadata": {"labels": {"app": "web"}},
                                "spec": {"containers": [{"name": "c", "image": "web:1", "command": ["sleep", "1"]}]}}}}


class Kubelets(threading.Thread):
    """Every node's kubelet, as far as the API sees it: pods bound to a node go Running (PUT
    status with that node's token), deleted ones are confirmed (DELETE, grace 0)."""

    def __init__(self, admin: Client, nodes: dict):
        super().__init__(daemon=True)
        admin = Client(admin.base, token=admin.token, prefix=admin.prefix, timeout=30)  # long-polls
        self.admin, self.nodes, self.stop = admin, nodes, threading.Event()
        self.seen: dict[str, set] = {}   # pod name -> uids seen under it
        self.errors: list[str] = []

    def rebase(self, base: str) -> None:  # the control plane came back on another port
        self.admin = Client(base, token=self.admin.token, prefix=self.admin.prefix, timeout=30)
        self.nodes = {n: Client(base, token=c.token, prefix=c.prefix, timeout=10) for n, c in self.nodes.items()}

    def run(self):
        since = None
        while not self.stop.is_set():
            try:
                if since is None:  # list once, then watch -- as an agent does (agent.watch_loop)
                    lst = self.admin.get(self.admin.k8s("/api/v1/pods"))
                    since, pods = int(lst["metadata"]["resourceVersion"]), lst["items"]
                else:
                    since, evs = self.admin.watch(self.admin.k8s("/api/v1/pods"), since, timeout=2.0)
                    pods = [e["object"] for e in evs if e["type"] != "DELETED"]
            except (ApiError, OSError):
                since = None
                self.stop.wait(0.05)
                continue
            for p in pods:
                self._handle(p)

    def _handle(self, p: dict) -> None:
        md, node = p["metadata"], p["spec"].get("nodeName")
        self.seen.setdefault(md["name"], set()).add(md["uid"])
        nc = self.nodes.get(node)
        if nc is None:
            return
        path = nc.k8s(f"/api/v1/namespaces/{md['namespace']}/pods/{md['name']}")
        try:
            if md.get("deletionTimestamp"):
                nc.delete(path, query={"gracePeriodSeconds": "0"})
            elif p.get("status", {}).get("phase") == "Pending":
                nc.put(path + "/status", {"status": {"phase": "Running", "containerStatuses": [
                    {"name": "c", "ready": True, "restartCount": 0, "state": {"running": {}}}]}})
        except ApiError as e:
            if e.status not in (404, 409):
                self.errors.append(str(e))
        except OSError:
            pass


def _timed(c: Client, lat: list):
    """Wrap a client so every request's latency lands in ``lat`` (ms)."""
    orig = c.request

    def request(method, path, *a, **kw):
        t = time.perf_counter()
        try:
            return orig(method, path, *a, **kw)
        finally:
            lat.append((time.perf_counter() - t) * 1e3)

    c.request = request
    return c


def _until(fn, timeout=120.0, what=""):
    deadline = time.monotonic() + timeout
    while True:
        v = fn()
        if v:
            return v
        assert time.monotonic() < deadline, f"timed out: {what}"
        time.sleep(0.05)


def _rss_kib(pid: int) -> int:
    for line in open(f"/proc/{pid}/status"):
        if line.startswith("VmRSS:"):
            return int(line.split()[1])
    return 0


def _rolled(k: Client, replicas: int, image: str):
    d = k.get(k.k8s("/apis/apps/v1/namespaces/default/deployments/web"))
    st = d.get("status") or {}
    pods = [p for p in k.get(k.k8s("/api/v1/namespaces/default/pods"), query={"labelSelector": "app=web"})["items"]
            if not p["metadata"].get("deletionTimestamp")]
    ok = (st.get("updatedReplicas") == replicas and st.get("readyReplicas") == replicas and len(pods) == replicas
          and all(p["spec"]["containers"][0]["image"] == image and p["status"].get("phase") == "Running" for p in pods))
    return pods if ok else None


@pytest.mark.timeout(600)
def test_control_plane_load(tmp_path):
    p, c = _start(tmp_path, grace=120)
    lat: list[float] = []
    try:
        proj = _env(c)
        nodes = {f"kubenode{i}": _join(c, proj["id"], f"kubenode{i}", ngpu=0)[0] for i in range(1, 9)}
        k = _timed(client_from_kubeconfig(c.get(f"/env/{proj['id']}/kubernetes/kubectl", query={"format": "json"})), lat)
        kl = Kubelets(client_from_kubeconfig(c.get(f"/env/{proj['id']}/kubernetes/kubectl", query={"format": "json"})),
                      nodes)
        kl.start()
        # 50 concurrent watches on the ConfigMaps, from before the first one exists
        rv0 = int(k.get(k.k8s("/api/v1/namespaces/default/configmaps"))["metadata"]["resourceVersion"])
        counts = [0] * 50
        stop = threading.Event()

        def watcher(i):
            w = Client(k.base, token=k.token, prefix=k.prefix, timeout=30)
            since = rv0
            while not stop.is_set() and counts[i] < 2000:
                try:
                    since, evs = w.watch(w.k8s("/api/v1/namespaces/default/configmaps"), since, timeout=2.0)
                except (ApiError, OSError):
                    continue
                counts[i] += sum(1 for e in evs if e["type"] == "ADDED")

        ws = [threading.Thread(target=watcher, args=(i,), daemon=True) for i in range(50)]
        for t in ws:
            t.start()
        t0 = time.perf_counter()
        for i in range(2000):
            k.post(k.k8s("/api/v1/namespaces/default/configmaps"), {"metadata": {"name": f"cm-{i}"}, "data": {"i": str(i)}})
        cm_s = time.perf_counter() - t0
        for i in range(400):
            k.post(k.k8s("/api/v1/namespaces/default/pods"), {"metadata": {"name": f"bare-{i}"}, "spec": {
                "containers": [{"name": "c", "command": ["sleep", "1"], "resources": {"requests": {"cpu": "10m"}}}]}})
        k.post(k.k8s("/apis/apps/v1/namespaces/default/deployments"), DEPLOY)
        _until(lambda: _rolled(k, 100, "web:1"), what="100 replicas Running")
        _until(lambda: all(x >= 2000 for x in counts), 60, "every watch saw every ConfigMap")
        t_roll = time.perf_counter()
        k.request("PATCH", k.k8s("/apis/apps/v1/namespaces/default/deployments/web"),
                  body={"spec": {"template": {"spec": {"containers": [{"name": "c", "image": "web:2"}]}}}})
        _until(lambda: _rolled(k, 100, "web:2"), what="rolling update of 100 replicas")
        roll_s = time.perf_counter() - t_roll
        running = sum(1 for x in k.get(k.k8s("/api/v1/pods"))["items"] if x["status"].get("phase") == "Running")
        stop.set()
        kl.stop.set()
        rss = _rss_kib(p.pid)
    finally:
        _stop(p)
    srt = sorted(lat)
    p50, p99 = srt[len(srt) // 2], srt[int(len(srt) * 0.99)]
    out = {"nodes": 8, "configmaps": 2000, "pods": 500, "watches": 50, "rollout_replicas": 100,
           "requests": len(srt), "p50_ms": round(p50, 3), "p99_ms": round(p99, 3), "max_ms": round(srt[-1], 3),
           "configmap_creates_per_s": round(2000 / cm_s, 1), "rollout_s": round(roll_s, 3),
           "server_rss_mib": round(rss / 1024, 1), "running_pods": running, "kubelet_errors": kl.errors[:5],
           "loadavg": os.getloadavg()[0]}
    print(json.dumps(out))
    if os.environ.get("TK8S_LOAD_OUT"):
        with open(os.environ["TK8S_LOAD_OUT"], "w") as f:
            json.dump(out, f, indent=1)
    assert running >= 500 and not kl.errors, out
    # the bound: 50 ms at p99 on a quiet dev box; a box this suite shares with 5 other workers gets slack
    bound = 50.0 if os.getloadavg()[0] < 4 else 250.0
    assert p99 < bound, out


@pytest.mark.timeout(300)
def test_control_plane_killed_mid_rollout_recovers(tmp_path):
    state = tmp_path / "cp-state"
    p, c = _start(tmp_path, grace=60, state_dir=state)
    p2 = None
    try:
        proj = _env(c)
        nodes = {f"kubenode{i}": _join(c, proj["id"], f"kubenode{i}", ngpu=0)[0] for i in (1, 2)}
        k = client_from_kubeconfig(c.get(f"/env/{proj['id']}/kubernetes/kubectl", query={"format": "json"}))
        kl = Kubelets(client_from_kubeconfig(c.get(f"/env/{proj['id']}/kubernetes/kubectl", query={"format": "json"})),
                      nodes)
        kl.start()
        dep = json.loads(json.dumps(DEPLOY))
        dep["spec"]["replicas"] = 20
        k.post(k.k8s("/apis/apps/v1/namespaces/default/deployments"), dep)
        _until(lambda: _rolled(k, 20, "web:1"), what="20 replicas Running")
        k.request("PATCH", k.k8s("/apis/apps/v1/namespaces/default/deployments/web"),
                  body={"spec": {"template": {"spec": {"containers": [{"name": "c", "image": "web:2"}]}}}})

        def mid():
            st = k.get(k.k8s("/apis/apps/v1/namespaces/default/deployments/web")).get("status") or {}
            return 0 < (st.get("updatedReplicas") or 0) < 20

        _until(mid, what="mid-rollout")
        before = {x["metadata"]["name"]: x["metadata"]["uid"] for x in k.get(k.k8s("/api/v1/pods"))["items"]}
        rv_before = int(k.get(k.k8s("/api/v1/pods"))["metadata"]["resourceVersion"])
        os.kill(p.pid, signal.SIGKILL)  # no graceful snapshot: the journal has to carry it
        p.wait(10)
        p2, c2 = _start(tmp_path, grace=60, state_dir=state)
        kl.rebase(c2.base)
        k2 = Client(c2.base, token=k.token, prefix=k.prefix, timeout=10)
        after = {x["metadata"]["name"]: x["metadata"]["uid"] for x in k2.get(k2.k8s("/api/v1/pods"))["items"]}
        assert int(k2.get(k2.k8s("/api/v1/pods"))["metadata"]["resourceVersion"]) >= rv_before
        # nothing acknowledged was lost (what the rollout has not deleted since is there, same uid)
        assert {n: u for n, u in before.items() if n in after} == {n: before[n] for n in before if n in after}
        assert len(set(before) - set(after)) <= 5, (sorted(set(before) - set(after)))  # at most the terminations since
        pods = _until(lambda: _rolled(k2, 20, "web:2"), what="the rollout finishes after the restart")
        rss = k2.get(k2.k8s("/apis/apps/v1/namespaces/default/replicasets"))["items"]
        assert sorted(r["spec"]["replicas"] for r in rss) == [0, 20]  # the old one drained, no third one
        assert len({x["metadata"]["name"] for x in pods}) == 20
        kl.stop.set()
        # no name was ever handed out twice (the server's sequence survived the kill)
        assert all(len(uids) == 1 for uids in kl.seen.values()), {n: u for n, u in kl.seen.items() if len(u) > 1}
        assert not kl.errors, kl.errors
    finally:
        if p.poll() is None:
            _stop(p)
        if p2 is not None:
            _stop(p2)


def test_a_torn_journal_tail_does_not_hide_later_writes(tmp_path):
    """A kill in the middle of a journal write leaves a torn last line. The restart replays up to
    it and must cut it off before appending: otherwise the next restart stops at the torn line and
    loses every write acknowledged after the first restart."""
    from tritonk8ssupervisor_amd.controlplane.store import Store

    j = tmp_path / "controlplane.journal"
    s = Store()
    s.open_journal(j)
    for i in range(3):
        s.put("configmaps", f"p/default/c{i}", {"metadata": {"name": f"c{i}"}, "data": {"i": str(i)}})
    s._journal.flush()
    with open(j, "ab") as f:  # the write a SIGKILL cut short
        f.write(b'{"rv": 4, "op": "put", "kind": "configmaps", "key": "p/def')
    s2 = Store()
    assert s2.open_journal(j) == 3
    s2.put("configmaps", "p/default/after", {"metadata": {"name": "after"}, "data": {}})
    s2._journal.flush()
    s3 = Store()
    assert s3.open_journal(j) == 4
    assert s3.get("configmaps", "p/default/after") is not None and s3.get("configmaps", "p/default/c2") is not None
