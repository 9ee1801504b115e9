"""StatefulSets, ReplicaSets, CronJobs and headless Services (controlplane/workloads.py,
controlplane/cron.py), driven in-process: objects go through the API's create/replace, pod phases
are reported the way a node agent does, and reconcile() runs as after every change."""
import json
import os
import socket
from datetime import datetime, timedelta, timezone

import pytest

from tritonk8ssupervisor_amd.controlplane import cron
from tritonk8ssupervisor_amd.controlplane.httpserver import HttpError
from tritonk8ssupervisor_amd.controlplane.objects import _key
from tritonk8ssupervisor_amd.controlplane.server import ControlPlane

UTC = timezone.utc


# ---- cron -----------------------------------------------------------------------------------
def _t(s: str) -> datetime:
    return datetime.strptime(s, "%Y-%m-%d %H:%M").replace(tzinfo=UTC)


@pytest.mark.parametrize("expr,after,want", [
    ("*/15 * * * *", "2026-03-01 10:07", "2026-03-01 10:15"),
    ("0 3 * * *", "2026-03-01 10:07", "2026-03-02 03:00"),
    ("30 9 * * mon-fri", "2026-10-16 10:00", "2026-10-19 09:30"),   # Friday after 9:30 -> Monday
    ("0 0 1 jan,jul *", "2026-03-01 00:00", "2026-07-01 00:00"),
    ("0 12 13 * 5", "2026-10-01 00:00", "2026-10-02 12:00"),        # dom OR dow: Friday the 2nd first
    ("5 4 * * 7", "2026-10-17 00:00", "2026-10-18 04:05"),          # 7 is Sunday
    ("@hourly", "2026-03-01 10:07", "2026-03-01 11:00"),
    ("@weekly", "2026-10-14 10:00", "2026-10-18 00:00"),
    ("0 0 29 2 *", "2026-03-01 00:00", "2028-02-29 00:00"),
])
def test_cron_next(expr, after, want):
    assert cron.parse(expr, "UTC").next_after(_t(after)) == _t(want)


@pytest.mark.parametrize("bad", ["* * * *", "61 * * * *", "* * * 13 *", "*/0 * * * *", "5-1 * * * *", "x * * * *",
                                 "@every", "@every 5q", "* * * * * *"])
def test_cron_rejects(bad):
    with pytest.raises(cron.CronError):
        cron.parse(bad, "UTC")


def test_cron_every_timezones_and_missed_runs():
    s = cron.parse("@every 1m30s")
    assert s.every == 90.0
    t0 = _t("2026-03-01 10:00")
    assert cron.most_recent(s, t0, t0 + timedelta(seconds=89)) == (None, 0)
    assert cron.most_recent(s, t0, t0 + timedelta(seconds=200)) == (t0 + timedelta(seconds=180), 2)
    hourly = cron.parse("0 * * * *", "UTC")
    last, n = cron.most_recent(hourly, t0, t0 + timedelta(hours=5, minutes=10))
    assert last == t0 + timedelta(hours=5) and n == 5
    # a time zone moves the wall clock the schedule is read in
    tokyo = cron.parse("CRON_TZ=Asia/Tokyo 0 9 * * *")
    assert tokyo.next_after(_t("2026-03-01 00:30")) == _t("2026-03-02 00:00")  # 09:00 JST = 00:00 UTC


# ---- in-process control plane -------------------------------------------------------------------
@pytest.fixture
def cp():
    c = ControlPlane("127.0.0.1", 0)
    c.store.put("projects", "1a1", {"id": "1a1", "created_seq": 1, "metadata": {"name": "1a1"}})
    return c


def _pods(c, prefix=""):
    return sorted(o["metadata"]["name"] for o in c.store.list("pods") if o["metadata"]["name"].startswith(prefix))


def _run(c, name, ip="127.128.0.{}"):
    def fn(o):
        o.setdefault("status", {}).update(phase="Running", podIP=ip.format(2 + int(name.rsplit("-", 1)[1], 16) % 200))
    c.store.patch("pods", _key("1a1", "default", name), fn)
    c.reconcile()


def _sts(replicas=3, **spec):
    return {"apiVersion": "apps/v1", "kind": "StatefulSet", "metadata": {"name": "web"},
            "spec": {"replicas": replicas, "serviceName": "web", "selector": {"matchLabels": {"app": "web"}},
                     "template": {"metadata": {"labels": {"app": "web"}},
                                  "spec": {"containers": [{"name": "c", "image": "python", "command": ["sleep", "60"]}]}},
                     **spec}}


def test_statefulset_ordered_scaling_and_stable_names(cp):
    cp.create("1a1", "statefulsets", "default", _sts(3))
    assert _pods(cp, "web") == ["web-0"]  # OrderedReady: one at a time
    p0 = cp.store.get("pods", _key("1a1", "default", "web-0"))
    assert p0["spec"]["hostname"] == "web-0" and p0["spec"]["subdomain"] == "web"
    assert p0["metadata"]["labels"]["apps.kubernetes.io/pod-index"] == "0"
    _run(cp, "web-0")
    assert _pods(cp, "web") == ["web-0", "web-1"]
    _run(cp, "web-1")
    _run(cp, "web-2")
    st = cp.store.get("statefulsets", _key("1a1", "default", "web"))["status"]
    assert st["readyReplicas"] == 3 and st["updatedReplicas"] == 3 and st["currentRevision"] == st["updateRevision"]
    # a deleted pod comes back under its own name
    cp.store.delete("pods", _key("1a1", "default", "web-1"))
    cp.reconcile()
    assert "web-1" in _pods(cp, "web")
    _run(cp, "web-1")
    # scale down: the highest ordinal first, one at a time
    cur = cp.store.get("statefulsets", _key("1a1", "default", "web"))
    body = json.loads(json.dumps(cp._strip(cur)))
    body["spec"]["replicas"] = 1
    cp.replace("1a1", "statefulsets", "default", "web", body)
    assert _pods(cp, "web") == ["web-0", "web-1"]
    cp.reconcile()
    assert _pods(cp, "web") == ["web-0"]
    # identity fields are immutable
    body = json.loads(json.dumps(cp._strip(cp.store.get("statefulsets", _key("1a1", "default", "web")))))
    body["spec"]["serviceName"] = "other"
    with pytest.raises(HttpError) as e:
        cp.replace("1a1", "statefulsets", "default", "web", body)
    assert e.value.status == 422


def test_statefulset_rolling_update_and_parallel(cp):
    cp.create("1a1", "statefulsets", "default", _sts(3, podManagementPolicy="Parallel"))
    assert _pods(cp, "web") == ["web-0", "web-1", "web-2"]
    for n in ("web-0", "web-1", "web-2"):
        _run(cp, n)
    old = {n: cp.store.get("pods", _key("1a1", "default", n))["metadata"]["uid"] for n in _pods(cp, "web")}
    body = json.loads(json.dumps(cp._strip(cp.store.get("statefulsets", _key("1a1", "default", "web")))))
    body["spec"]["template"]["spec"]["containers"][0]["command"] = ["sleep", "61"]
    cp.replace("1a1", "statefulsets", "default", "web", body)

    def uid(n):
        return cp.store.get("pods", _key("1a1", "default", n))["metadata"]["uid"]

    assert uid("web-2") != old["web-2"] and uid("web-1") == old["web-1"]  # highest ordinal first
    _run(cp, "web-2")
    assert uid("web-1") != old["web-1"] and uid("web-0") == old["web-0"]
    _run(cp, "web-1")
    _run(cp, "web-0")
    st = cp.store.get("statefulsets", _key("1a1", "default", "web"))["status"]
    assert st["updatedReplicas"] == 3 and st["currentRevision"] == st["updateRevision"]


def test_headless_service_dns_for_statefulset_pods(cp):
    cp.create("1a1", "services", "default", {"metadata": {"name": "web"}, "spec": {
        "clusterIP": "None", "selector": {"app": "web"}, "ports": [{"port": 29500}]}})
    assert cp.store.get("services", _key("1a1", "default", "web"))["spec"]["clusterIP"] == "None"
    assert not any(k[1] == "None" for k in cp._proxy_wanted())  # no proxy listener for a headless Service
    cp.create("1a1", "statefulsets", "default", _sts(2))
    assert cp.dns_resolve("web-0.web.default.svc.cluster.local") is None  # not running yet
    _run(cp, "web-0")
    _run(cp, "web-1")
    ip0 = cp.store.get("pods", _key("1a1", "default", "web-0"))["status"]["podIP"]
    ip1 = cp.store.get("pods", _key("1a1", "default", "web-1"))["status"]["podIP"]
    assert cp.dns_resolve("web-0.web.default.svc.cluster.local") == [ip0]
    assert cp.dns_resolve("web-1.web.default.svc") == [ip1]
    assert cp.dns_resolve("web.default.svc.cluster.local") == sorted([ip0, ip1])
    assert cp.dns_resolve("web-7.web.default.svc.cluster.local") is None
    with pytest.raises(HttpError):
        cp.create("1a1", "services", "default", {"metadata": {"name": "bad"}, "spec": {
            "clusterIP": "None", "type": "NodePort", "ports": [{"port": 80}]}})


def test_replicaset(cp):
    with pytest.raises(HttpError):  # the selector must match the template's labels
        cp.create("1a1", "replicasets", "default", {"metadata": {"name": "rs"}, "spec": {
            "selector": {"matchLabels": {"app": "x"}}, "template": {"metadata": {"labels": {"app": "y"}},
                                                                 "spec": {"containers": [{"name": "c"}]}}}})
    cp.create("1a1", "replicasets", "default", {"metadata": {"name": "rs"}, "spec": {
        "replicas": 3, "selector": {"matchLabels": {"app": "rs"}},
        "template": {"metadata": {"labels": {"app": "rs"}}, "spec": {"containers": [{"name": "c", "command": ["true"]}]}}}})
    names = _pods(cp, "rs-")
    assert len(names) == 3
    _run(cp, names[0])
    body = json.loads(json.dumps(cp._strip(cp.store.get("replicasets", _key("1a1", "default", "rs")))))
    body["spec"]["replicas"] = 1
    cp.replace("1a1", "replicasets", "default", "rs", body)
    assert _pods(cp, "rs-") == [names[0]]  # the pods not yet running go first


def _cronjob(**spec):
    return {"apiVersion": "batch/v1", "kind": "CronJob", "metadata": {"name": "tick"},
            "spec": {"schedule": "@every 10s", "jobTemplate": {"spec": {"template": {"spec": {
                "restartPolicy": "Never", "containers": [{"name": "c", "command": ["true"]}]}}}}, **spec}}


def _jobs(c):
    return sorted(o["metadata"]["name"] for o in c.store.list("jobs"))


def _finish(c, name, kind="Complete"):
    c.store.patch("jobs", _key("1a1", "default", name), lambda o: o.setdefault("status", {}).update(
        conditions=[{"type": kind, "status": "True"}], completionTime="2026-01-01T00:00:00Z"))


def test_cronjob_schedules_policies_and_history(cp):
    with pytest.raises(HttpError) as e:
        cp.create("1a1", "cronjobs", "default", _cronjob(schedule="61 * * * *"))
    assert e.value.status == 422
    cj = cp.create("1a1", "cronjobs", "default", _cronjob(concurrencyPolicy="Forbid"))
    t0 = datetime.strptime(cj["metadata"]["creationTimestamp"], "%Y-%m-%dT%H:%M:%SZ").replace(tzinfo=UTC)
    cp._ctl_cronjobs("1a1", now=t0 + timedelta(seconds=5))
    assert _jobs(cp) == []
    cp._ctl_cronjobs("1a1", now=t0 + timedelta(seconds=11))
    assert len(_jobs(cp)) == 1
    job = cp.store.get("jobs", _key("1a1", "default", _jobs(cp)[0]))
    assert job["metadata"]["ownerReferences"][0]["kind"] == "CronJob"
    assert job["metadata"]["annotations"]["batch.kubernetes.io/cronjob-scheduled-timestamp"]
    assert cp.store.list("pods", lambda o: o["metadata"]["name"].startswith(job["metadata"]["name"]))  # the Job ran
    st = cp.store.get("cronjobs", _key("1a1", "default", "tick"))["status"]
    assert len(st["active"]) == 1 and st["lastScheduleTime"]
    cp._ctl_cronjobs("1a1", now=t0 + timedelta(seconds=21))  # Forbid: the first is still active
    assert len(_jobs(cp)) == 1
    _finish(cp, _jobs(cp)[0])
    for k in range(3, 8):  # more runs than the history keeps
        cp._ctl_cronjobs("1a1", now=t0 + timedelta(seconds=10 * k + 1))
        for j in _jobs(cp):
            _finish(cp, j)
    cp._ctl_cronjobs("1a1", now=t0 + timedelta(seconds=81))
    st = cp.store.get("cronjobs", _key("1a1", "default", "tick"))["status"]
    done = [j for j in _jobs(cp) if j != (st.get("active") or [{}])[0].get("name")]
    assert len(done) <= 3 and st.get("lastSuccessfulTime")
    # Replace: a new run replaces the active one; suspend: nothing runs
    body = json.loads(json.dumps(cp._strip(cp.store.get("cronjobs", _key("1a1", "default", "tick")))))
    body["spec"]["concurrencyPolicy"] = "Replace"
    cp.replace("1a1", "cronjobs", "default", "tick", body)
    before = set(_jobs(cp))
    cp._ctl_cronjobs("1a1", now=t0 + timedelta(seconds=91))
    active = cp.store.get("cronjobs", _key("1a1", "default", "tick"))["status"]["active"]
    assert len(active) == 1 and active[0]["name"] not in before
    body = json.loads(json.dumps(cp._strip(cp.store.get("cronjobs", _key("1a1", "default", "tick")))))
    body["spec"]["suspend"] = True
    cp.replace("1a1", "cronjobs", "default", "tick", body)
    n = len(_jobs(cp))
    cp._ctl_cronjobs("1a1", now=t0 + timedelta(seconds=200))
    assert len(_jobs(cp)) == n


def test_cronjob_starting_deadline_skips_a_late_run(cp):
    cj = cp.create("1a1", "cronjobs", "default", _cronjob(startingDeadlineSeconds=5))
    t0 = datetime.strptime(cj["metadata"]["creationTimestamp"], "%Y-%m-%dT%H:%M:%SZ").replace(tzinfo=UTC)
    cp._ctl_cronjobs("1a1", now=t0 + timedelta(seconds=18))  # due at +10, 8 s late > 5 s
    assert _jobs(cp) == []
    cp._ctl_cronjobs("1a1", now=t0 + timedelta(seconds=21))  # due at +20, 1 s late
    assert len(_jobs(cp)) == 1


def test_pvc_binds_on_first_use_and_pins_later_pods(cp):
    for n in ("kubenode1", "kubenode2"):
        cp.store.put("nodes", _key("1a1", n), {"_project": "1a1", "metadata": {"name": n, "labels": {
            "kubernetes.io/hostname": n}}, "spec": {}, "status": {"allocatable": {"amd.com/gpu": "0"}, "conditions": [
                {"type": "Ready", "status": "True"}, {"type": "AMDGPUValidated", "status": "True"}]}})
    with pytest.raises(HttpError):
        cp.create("1a1", "persistentvolumeclaims", "default", {"metadata": {"name": "nosize"}, "spec": {}})
    pvc = cp.create("1a1", "persistentvolumeclaims", "default", {"metadata": {"name": "data"}, "spec": {
        "resources": {"requests": {"storage": "10Gi"}}}})
    assert pvc["status"]["phase"] == "Bound" and pvc["spec"]["storageClassName"] == "tk8s-local"
    pod = {"metadata": {"name": "{}"}, "spec": {"containers": [{"name": "c", "command": ["true"]}],
                                                 "volumes": [{"name": "d", "persistentVolumeClaim": {"claimName": "data"}}]}}
    first = json.loads(json.dumps(pod).replace("{}", "user-a"))
    cp.create("1a1", "pods", "default", first)
    node = cp.store.get("pods", _key("1a1", "default", "user-a"))["spec"]["nodeName"]
    assert cp.store.get("persistentvolumeclaims", _key("1a1", "default", "data"))["metadata"]["annotations"][
        "volume.kubernetes.io/selected-node"] == node
    for k in range(4):  # every later user of the claim lands on the same node
        cp.create("1a1", "pods", "default", json.loads(json.dumps(pod).replace("{}", f"user-{k}b")))
        assert cp.store.get("pods", _key("1a1", "default", f"user-{k}b"))["spec"]["nodeName"] == node
    lost = json.loads(json.dumps(pod).replace("{}", "lost").replace('"data"', '"missing"'))
    cp.create("1a1", "pods", "default", lost)
    p = cp.store.get("pods", _key("1a1", "default", "lost"))
    assert not p["spec"].get("nodeName") and "not found" in p["status"]["conditions"][0]["message"]
    # the claim's spec is immutable but for its size
    body = json.loads(json.dumps(cp._strip(cp.store.get("persistentvolumeclaims", _key("1a1", "default", "data")))))
    body["spec"]["accessModes"] = ["ReadWriteMany"]
    with pytest.raises(HttpError):
        cp.replace("1a1", "persistentvolumeclaims", "default", "data", body)


def test_statefulset_volume_claim_templates(cp):
    cp.create("1a1", "statefulsets", "default", _sts(2, podManagementPolicy="Parallel", volumeClaimTemplates=[
        {"metadata": {"name": "data"}, "spec": {"resources": {"requests": {"storage": "1Gi"}}}}]))
    claims = sorted(o["metadata"]["name"] for o in cp.store.list("persistentvolumeclaims"))
    assert claims == ["data-web-0", "data-web-1"]
    p1 = cp.store.get("pods", _key("1a1", "default", "web-1"))
    assert {"name": "data", "persistentVolumeClaim": {"claimName": "data-web-1"}} in p1["spec"]["volumes"]
    # the ordinal's replacement gets the same claim; scaling down keeps the claims
    cp.store.delete("pods", _key("1a1", "default", "web-1"))
    cp.reconcile()
    assert cp.store.get("pods", _key("1a1", "default", "web-1"))["spec"]["volumes"][-1]["persistentVolumeClaim"][
        "claimName"] == "data-web-1"
    body = json.loads(json.dumps(cp._strip(cp.store.get("statefulsets", _key("1a1", "default", "web")))))
    body["spec"]["replicas"] = 1
    cp.replace("1a1", "statefulsets", "default", "web", body)
    assert len(cp.store.list("persistentvolumeclaims")) == 2


def test_volume_materialisation_unit(tmp_path):
    import base64
    import os
    import stat

    from tritonk8ssupervisor_amd.agent.volumes import VolumeError, mounts, volume_dirs

    objs = {("configmaps", "cfg"): {"data": {"app.conf": "x=1\n", "other": "y"},
                                   "binaryData": {"blob": base64.b64encode(b"\x00\x01").decode()}},
            ("secrets", "pw"): {"data": {"password": base64.b64encode(b"s3cr3t").decode()}},
            ("persistentvolumeclaims", "data"): {"metadata": {"uid": "0123456789abcdef"}}}
    fetch = lambda kind, ns, name: objs.get((kind, name))  # noqa: E731
    pod = {"metadata": {"name": "p", "namespace": "default", "labels": {"app": "x"}},
           "spec": {"volumes": [
               {"name": "cfg", "configMap": {"name": "cfg", "items": [{"key": "app.conf", "path": "conf/app.conf", "mode": 0o600}]}},
               {"name": "bin", "configMap": {"name": "cfg"}},
               {"name": "pw", "secret": {"secretName": "pw", "defaultMode": 0o400}},
               {"name": "scratch", "emptyDir": {}},
               {"name": "info", "downwardAPI": {"items": [{"path": "labels", "fieldRef": {"fieldPath": "metadata.labels"}},
                                                        {"path": "name", "fieldRef": {"fieldPath": "metadata.name"}}]}},
               {"name": "data", "persistentVolumeClaim": {"claimName": "data"}},
               {"name": "opt", "configMap": {"name": "absent", "optional": True}}]}}
    dirs = volume_dirs(pod, tmp_path / "pod", tmp_path / "node", fetch)
    assert (dirs["cfg"][0] / "conf" / "app.conf").read_text() == "x=1\n"
    assert stat.S_IMODE(os.stat(dirs["cfg"][0] / "conf" / "app.conf").st_mode) == 0o600
    assert (dirs["bin"][0] / "blob").read_bytes() == b"\x00\x01" and (dirs["bin"][0] / "other").read_text() == "y"
    assert (dirs["pw"][0] / "password").read_bytes() == b"s3cr3t"
    assert stat.S_IMODE(os.stat(dirs["pw"][0] / "password").st_mode) == 0o400
    assert (dirs["info"][0] / "labels").read_text() == 'app="x"\n' and (dirs["info"][0] / "name").read_text() == "p"
    assert dirs["data"][0] == tmp_path / "node" / "volumes" / "default_data-01234567"
    assert dirs["cfg"][1] and not dirs["scratch"][1]  # configMaps are read-only, emptyDirs are not
    m = mounts({"volumeMounts": [{"name": "scratch", "mountPath": "/work", "subPath": "a/b"},
                                 {"name": "data", "mountPath": "/data", "readOnly": True}]}, dirs)
    assert m == [(str(dirs["scratch"][0] / "a" / "b"), "/work", False), (str(dirs["data"][0]), "/data", True)]
    with pytest.raises(VolumeError, match="not found"):
        volume_dirs({"metadata": pod["metadata"], "spec": {"volumes": [{"name": "c", "configMap": {"name": "absent"}}]}},
                    tmp_path / "p2", tmp_path / "node", fetch)
    with pytest.raises(VolumeError):  # item paths cannot leave the volume
        volume_dirs({"metadata": pod["metadata"], "spec": {"volumes": [{"name": "c", "configMap": {
            "name": "cfg", "items": [{"key": "other", "path": "../../etc/x"}]}}]}}, tmp_path / "p3", tmp_path / "node", fetch)
    with pytest.raises(VolumeError):
        mounts({"volumeMounts": [{"name": "scratch", "mountPath": "/w", "subPath": "../x"}]}, dirs)


def test_projected_volumes_and_atomic_refresh(tmp_path):
    """ConfigMap/Secret/projected volumes are published through ..data; a refresh swaps a changed
    ConfigMap in at once and drops keys that are gone (the kubelet's atomic writer)."""
    import base64

    from tritonk8ssupervisor_amd.agent.volumes import refresh, volume_dirs

    objs = {("configmaps", "cfg"): {"data": {"a": "1", "b": "2"}},
            ("secrets", "default-token"): {"data": {"token": base64.b64encode(b"tok").decode()}},
            ("secrets", "pw"): {"data": {"password": base64.b64encode(b"s3").decode()}}}
    fetch = lambda kind, ns, name: objs.get((kind, name))  # noqa: E731
    pod = {"metadata": {"name": "p", "namespace": "default", "labels": {"v": "1"}}, "spec": {"volumes": [
        {"name": "cfg", "configMap": {"name": "cfg"}},
        {"name": "all", "projected": {"sources": [
            {"configMap": {"name": "cfg", "items": [{"key": "a", "path": "conf/a"}]}},
            {"secret": {"name": "pw"}},
            {"downwardAPI": {"items": [{"path": "labels", "fieldRef": {"fieldPath": "metadata.labels"}}]}},
            {"serviceAccountToken": {"path": "token", "expirationSeconds": 3600}}]}}]}}
    dirs = volume_dirs(pod, tmp_path / "pod", tmp_path / "node", fetch)
    cfg, proj = dirs["cfg"][0], dirs["all"][0]
    assert (cfg / "a").read_text() == "1" and (cfg / "a").is_symlink() and (cfg / "..data").is_symlink()
    assert (proj / "conf" / "a").read_text() == "1" and (proj / "password").read_bytes() == b"s3"
    assert (proj / "labels").read_text() == 'v="1"\n' and (proj / "token").read_bytes() == b"tok"
    assert refresh(pod, tmp_path / "pod", fetch) == []  # nothing changed: nothing rewritten
    old = os.readlink(cfg / "..data")
    objs[("configmaps", "cfg")] = {"data": {"a": "10", "c": "3"}}
    pod["metadata"]["labels"] = {"v": "2"}
    assert sorted(refresh(pod, tmp_path / "pod", fetch)) == ["all", "cfg"]
    assert (cfg / "a").read_text() == "10" and (cfg / "c").read_text() == "3" and not (cfg / "b").exists()
    assert os.readlink(cfg / "..data") != old and not (cfg / old).exists()  # the old generation is gone
    assert (proj / "conf" / "a").read_text() == "10" and (proj / "labels").read_text() == 'v="2"\n'
    del objs[("configmaps", "cfg")]  # a deleted source leaves the volume as it was
    assert refresh(pod, tmp_path / "pod", fetch) == [] and (cfg / "a").read_text() == "10"


def test_metrics_api_and_hpa(cp):
    import asyncio

    cp.create("1a1", "deployments", "default", {"metadata": {"name": "web"}, "spec": {
        "replicas": 2, "selector": {"matchLabels": {"app": "web"}},
        "template": {"metadata": {"labels": {"app": "web"}}, "spec": {"containers": [
            {"name": "c", "command": ["true"], "resources": {"requests": {"cpu": "500m"}}}]}}}})
    for n in _pods(cp, "web-"):
        cp.store.patch("pods", _key("1a1", "default", n), lambda o: o["status"].update(phase="Running"))

    def usage(cores):
        cp._ingest_metrics("1a1", "kubenode1", {"timestamp": "2026-01-01T00:00:00Z", "node": {
            "cpu_cores": 3.0, "memory_bytes": 2 ** 30}, "pods": {
            f"default/{n}": [{"name": "c", "cpu_cores": cores, "memory_bytes": 2 ** 20}] for n in _pods(cp, "web-")}})

    usage(0.5)  # 100 % of the request
    req = type("R", (), {"q": lambda self, k, d=None: None})()
    cp._pid = lambda pid, r: "1a1"
    lst = asyncio.run(cp.h_pod_metrics(req, ns="default"))
    assert lst["kind"] == "PodMetricsList" and len(lst["items"]) == 2
    assert lst["items"][0]["containers"][0]["usage"] == {"cpu": "500000000n", "memory": "1024Ki"}
    nodes = asyncio.run(cp.h_node_metrics(req))
    assert nodes["items"][0]["usage"]["cpu"] == "3000000000n"
    cp.create("1a1", "horizontalpodautoscalers", "default", {"metadata": {"name": "web"}, "spec": {
        "scaleTargetRef": {"apiVersion": "apps/v1", "kind": "Deployment", "name": "web"},
        "minReplicas": 1, "maxReplicas": 3,
        "metrics": [{"type": "Resource", "resource": {"name": "cpu", "target": {"type": "Utilization",
                                                                               "averageUtilization": 50}}}]}})
    cp._ctl_hpas("1a1", now=1000.0)
    d = cp.store.get("deployments", _key("1a1", "default", "web"))
    assert d["spec"]["replicas"] == 3  # 2 x 100/50 = 4, capped at maxReplicas
    hpa = cp.store.get("horizontalpodautoscalers", _key("1a1", "default", "web"))
    assert hpa["status"]["desiredReplicas"] == 3 and hpa["status"]["currentMetrics"][0]["resource"]["current"][
        "averageUtilization"] == 100
    # low use: the scale-down waits out the stabilization window (300 s by default)
    for n in _pods(cp, "web-"):
        cp.store.patch("pods", _key("1a1", "default", n), lambda o: o["status"].update(phase="Running"))
    usage(0.05)
    cp._ctl_hpas("1a1", now=1100.0)
    assert cp.store.get("deployments", _key("1a1", "default", "web"))["spec"]["replicas"] == 3
    cp._ctl_hpas("1a1", now=1500.0)
    assert cp.store.get("deployments", _key("1a1", "default", "web"))["spec"]["replicas"] == 1
    assert any(e["reason"] == "SuccessfulRescale" for e in cp.store.list("events"))
    with pytest.raises(HttpError):
        cp.create("1a1", "horizontalpodautoscalers", "default", {"metadata": {"name": "bad"}, "spec": {
            "scaleTargetRef": {"kind": "Deployment", "name": "web"}, "minReplicas": 5, "maxReplicas": 2}})


def test_hpa_on_gpu_utilisation(cp):
    """An MI355X-aware HorizontalPodAutoscaler: resource amd.com/gpu, the pods' GPU busy %."""
    cp.create("1a1", "deployments", "default", {"metadata": {"name": "infer"}, "spec": {
        "replicas": 2, "selector": {"matchLabels": {"app": "infer"}},
        "template": {"metadata": {"labels": {"app": "infer"}}, "spec": {"containers": [
            {"name": "c", "command": ["true"], "resources": {"limits": {"amd.com/gpu": "1"}}}]}}}})
    for n in _pods(cp, "infer-"):
        cp.store.patch("pods", _key("1a1", "default", n), lambda o: o["status"].update(phase="Running"))
    cp.create("1a1", "horizontalpodautoscalers", "default", {"metadata": {"name": "infer"}, "spec": {
        "scaleTargetRef": {"kind": "Deployment", "name": "infer"}, "maxReplicas": 8,
        "metrics": [{"type": "Resource", "resource": {"name": "amd.com/gpu", "target": {"type": "Utilization",
                                                                                       "averageUtilization": 60}}}]}})
    cp._ctl_hpas("1a1", now=10.0)
    hpa = cp.store.get("horizontalpodautoscalers", _key("1a1", "default", "infer"))
    assert hpa["status"]["conditions"][-1]["reason"] == "FailedGetResourceMetric"  # no samples yet
    cp._ingest_metrics("1a1", "kubenode1", {"pods": {f"default/{n}": [{"name": "c", "cpu_cores": 0.1, "memory_bytes": 0,
                                                                       "gpu_pct": 90.0, "gpus": 1}]
                                                     for n in _pods(cp, "infer-")}})
    cp._ctl_hpas("1a1", now=20.0)
    assert cp.store.get("deployments", _key("1a1", "default", "infer"))["spec"]["replicas"] == 3  # ceil(2 x 90/60)


def test_deployment_revisions_as_replicasets(cp):
    """Every template a Deployment has had is a ReplicaSet <name>-<hash> with a revision; going
    back to an old template makes it the newest revision; deleting the Deployment removes them."""
    tmpl = {"metadata": {"labels": {"app": "web"}}, "spec": {"containers": [{"name": "c", "command": ["sleep", "1"]}]}}
    cp.create("1a1", "deployments", "default", {"metadata": {"name": "web"}, "spec": {
        "replicas": 2, "selector": {"matchLabels": {"app": "web"}}, "template": json.loads(json.dumps(tmpl))}})

    def rss():
        return {o["metadata"]["name"]: o for o in cp.store.list("replicasets")}

    def rev(o):
        return int(o["metadata"]["annotations"]["deployment.kubernetes.io/revision"])

    first = rss()
    assert len(first) == 1
    (n1, rs1), = first.items()
    assert rev(rs1) == 1 and rs1["status"]["replicas"] == 2 and rs1["metadata"]["ownerReferences"][0]["kind"] == "Deployment"
    assert cp.store.get("deployments", _key("1a1", "default", "web"))["metadata"]["annotations"][
        "deployment.kubernetes.io/revision"] == "1"
    assert len(_pods(cp, "web-")) == 2  # the ReplicaSet controller does not run a Deployment's pods again

    def set_cmd(cmd):
        body = json.loads(json.dumps(cp._strip(cp.store.get("deployments", _key("1a1", "default", "web")))))
        body["spec"]["template"]["spec"]["containers"][0]["command"] = cmd
        cp.replace("1a1", "deployments", "default", "web", body)
        for n in _pods(cp, "web-"):
            cp.store.patch("pods", _key("1a1", "default", n), lambda o: o["status"].update(phase="Running"))
        cp.reconcile()

    set_cmd(["sleep", "2"])
    assert len(rss()) == 2 and max(rev(o) for o in rss().values()) == 2
    set_cmd(["sleep", "1"])  # back to the first template: its ReplicaSet is revision 3 now
    assert rev(rss()[n1]) == 3 and len(rss()) == 2
    import asyncio

    from tritonk8ssupervisor_amd.controlplane.httpserver import Request

    cp._auth = lambda req, proj: None
    cp._pid = lambda pid, req: "1a1"
    asyncio.run(cp._deleter("deployments")(Request("DELETE", "/x", {}, {}, b""), ns="default", name="web"))
    assert rss() == {} and _pods(cp, "web-") == []


def test_endpoints_follow_ready_pods_and_leases_are_plain_objects(cp):
    cp.create("1a1", "services", "default", {"metadata": {"name": "web"}, "spec": {
        "selector": {"app": "web"}, "ports": [{"name": "http", "port": 80, "targetPort": "http"}]}})
    for n in ("a", "b"):
        cp.create("1a1", "pods", "default", {"metadata": {"name": n, "labels": {"app": "web"}}, "spec": {
            "containers": [{"name": "c", "command": ["true"], "ports": [{"name": "http", "containerPort": 8080}]}]}})
    assert cp.store.get("endpoints", _key("1a1", "default", "web"))["subsets"] == []
    cp.store.patch("pods", _key("1a1", "default", "a"), lambda o: o["status"].update(phase="Running", podIP="127.128.0.2"))
    cp.store.patch("pods", _key("1a1", "default", "b"), lambda o: o["status"].update(
        phase="Running", podIP="127.128.0.3", conditions=[{"type": "Ready", "status": "False"}]))
    cp.reconcile()
    sub = cp.store.get("endpoints", _key("1a1", "default", "web"))["subsets"][0]
    assert [a["ip"] for a in sub["addresses"]] == ["127.128.0.2"] and sub["addresses"][0]["targetRef"]["name"] == "a"
    assert [a["ip"] for a in sub["notReadyAddresses"]] == ["127.128.0.3"]
    assert sub["ports"] == [{"name": "http", "port": 8080, "protocol": "TCP"}]
    import asyncio

    from tritonk8ssupervisor_amd.controlplane.httpserver import Request

    cp._auth = lambda req, proj: None
    cp._pid = lambda pid, req: "1a1"
    asyncio.run(cp._deleter("services")(Request("DELETE", "/x", {}, {}, b""), ns="default", name="web"))
    assert cp.store.get("endpoints", _key("1a1", "default", "web")) is None
    lease = cp.create("1a1", "leases", "default", {"apiVersion": "coordination.k8s.io/v1", "kind": "Lease",
                                                   "metadata": {"name": "leader"}, "spec": {"holderIdentity": "op-1"}})
    assert lease["kind"] == "Lease" and lease["spec"]["holderIdentity"] == "op-1"


def _nodes(cp, n=3, gpus=0):
    for i in range(1, n + 1):
        cp.store.put("nodes", _key("1a1", f"kubenode{i}"), {"_project": "1a1", "metadata": {
            "name": f"kubenode{i}", "labels": {"kubernetes.io/hostname": f"kubenode{i}", "zone": "a" if i < 3 else "b"}},
            "spec": {}, "status": {"allocatable": {"amd.com/gpu": str(gpus)}, "conditions": [
                {"type": "Ready", "status": "True"}, {"type": "AMDGPUValidated", "status": "True"}]}})


def _node_of(cp, name):
    return cp.store.get("pods", _key("1a1", "default", name))["spec"].get("nodeName")


def test_taints_tolerations_and_node_affinity(cp):
    _nodes(cp)
    cp.store.patch("nodes", _key("1a1", "kubenode1"), lambda o: o["spec"].update(
        taints=[{"key": "dedicated", "value": "train", "effect": "NoSchedule"}]))
    cp.store.patch("nodes", _key("1a1", "kubenode2"), lambda o: o["spec"].update(
        taints=[{"key": "maint", "effect": "NoSchedule"}]))
    pod = lambda name, **spec: {"metadata": {"name": name}, "spec": {"containers": [{"name": "c", "command": ["true"]}], **spec}}
    cp.create("1a1", "pods", "default", pod("plain"))
    assert _node_of(cp, "plain") == "kubenode3"  # the only untainted node
    cp.create("1a1", "pods", "default", pod("trainer", tolerations=[{"key": "dedicated", "operator": "Equal",
                                                                      "value": "train", "effect": "NoSchedule"}],
                                            affinity={"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {
                                                "nodeSelectorTerms": [{"matchExpressions": [{"key": "zone", "operator": "In",
                                                                                             "values": ["a"]}]}]}}}))
    assert _node_of(cp, "trainer") == "kubenode1"  # zone a, and kubenode2's taint is not tolerated
    cp.create("1a1", "pods", "default", pod("nowhere", affinity={"nodeAffinity": {
        "requiredDuringSchedulingIgnoredDuringExecution": {"nodeSelectorTerms": [{"matchFields": [
            {"key": "metadata.name", "operator": "In", "values": ["kubenode2"]}]}]}}}))
    p = cp.store.get("pods", _key("1a1", "default", "nowhere"))
    assert not p["spec"].get("nodeName") and "untolerated taint" in p["status"]["conditions"][0]["message"]
    cp.create("1a1", "pods", "default", pod("anything", tolerations=[{"operator": "Exists"}], affinity={"nodeAffinity": {
        "requiredDuringSchedulingIgnoredDuringExecution": {"nodeSelectorTerms": [{"matchFields": [
            {"key": "metadata.name", "operator": "In", "values": ["kubenode2"]}]}]}}}))
    assert _node_of(cp, "anything") == "kubenode2"


def test_pod_anti_affinity_spreads_ranks_one_per_node(cp):
    _nodes(cp)
    cp.create("1a1", "statefulsets", "default", _sts(4, podManagementPolicy="Parallel", template={
        "metadata": {"labels": {"app": "web"}},
        "spec": {"containers": [{"name": "c", "command": ["sleep", "60"]}],
                 "affinity": {"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
                     {"labelSelector": {"matchLabels": {"app": "web"}}, "topologyKey": "kubernetes.io/hostname"}]}}}}))
    placed = [_node_of(cp, f"web-{i}") for i in range(4)]
    assert sorted(n for n in placed if n) == ["kubenode1", "kubenode2", "kubenode3"] and placed.count(None) == 1
    # co-location: a pod that wants to be next to web-0
    cp.create("1a1", "pods", "default", {"metadata": {"name": "sidecar"}, "spec": {
        "containers": [{"name": "c", "command": ["true"]}],
        "affinity": {"podAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
            {"labelSelector": {"matchExpressions": [{"key": "statefulset.kubernetes.io/pod-name", "operator": "In",
                                                     "values": ["web-0"]}]}, "topologyKey": "kubernetes.io/hostname"}]}}}})
    assert _node_of(cp, "sidecar") == _node_of(cp, "web-0")


def test_resource_quota_caps_a_namespaces_gpus(cp):
    _nodes(cp, 2, gpus=4)
    cp.create("1a1", "resourcequotas", "team", {"metadata": {"name": "gpus"}, "spec": {"hard": {
        "requests.amd.com/gpu": "3", "pods": "4", "requests.cpu": "2"}}})
    pod = lambda name, gpus=0, cpu=None: {"metadata": {"name": name}, "spec": {"containers": [{
        "name": "c", "command": ["true"], "resources": {"limits": {"amd.com/gpu": str(gpus), **({"cpu": cpu} if cpu else {})}}}]}}
    cp.create("1a1", "pods", "team", pod("a", 2))
    with pytest.raises(HttpError) as e:
        cp.create("1a1", "pods", "team", pod("b", 2))
    assert e.value.status == 403 and "exceeded quota: gpus" in e.value.message and "requests.amd.com/gpu" in e.value.message
    cp.create("1a1", "pods", "team", pod("c", 1, cpu="1500m"))
    with pytest.raises(HttpError) as e:
        cp.create("1a1", "pods", "team", pod("d", 0, cpu="1"))  # cpu: 1.5 + 1 > 2
    assert "requests.cpu" in e.value.message
    cp.create("1a1", "pods", "other", pod("free", 4))  # other namespaces are not limited
    st = cp.store.get("resourcequotas", _key("1a1", "team", "gpus"))["status"]
    assert st["used"] == {"requests.amd.com/gpu": "3", "pods": "2", "requests.cpu": "1.5"}
    # a finished pod no longer counts
    cp.store.patch("pods", _key("1a1", "team", "a"), lambda o: o["status"].update(phase="Succeeded"))
    cp.create("1a1", "pods", "team", pod("b", 2))


def test_quota_holds_back_controller_pods_until_it_allows_them(cp):
    _nodes(cp, 1, gpus=8)
    cp.create("1a1", "resourcequotas", "default", {"metadata": {"name": "gpus"}, "spec": {"hard": {"requests.amd.com/gpu": "2"}}})
    cp.create("1a1", "deployments", "default", {"metadata": {"name": "inf"}, "spec": {
        "replicas": 3, "selector": {"matchLabels": {"app": "inf"}},
        "template": {"metadata": {"labels": {"app": "inf"}}, "spec": {"containers": [
            {"name": "c", "command": ["true"], "resources": {"limits": {"amd.com/gpu": "1"}}}]}}}})
    pods = [cp.store.get("pods", _key("1a1", "default", n)) for n in _pods(cp, "inf-")]
    assert len(pods) == 3
    bound = [p for p in pods if p["spec"].get("nodeName")]
    held = [p for p in pods if not p["spec"].get("nodeName")]
    assert len(bound) == 2 and len(held) == 1 and held[0]["status"]["conditions"][0]["reason"] == "ExceededQuota"
    assert any(e["reason"] == "FailedCreate" for e in cp.store.list("events"))
    # raising the quota lets the held pod through
    body = json.loads(json.dumps(cp._strip(cp.store.get("resourcequotas", _key("1a1", "default", "gpus")))))
    body["spec"]["hard"]["requests.amd.com/gpu"] = "3"
    cp.replace("1a1", "resourcequotas", "default", "gpus", body)
    assert cp.store.get("pods", _key("1a1", "default", held[0]["metadata"]["name"]))["spec"].get("nodeName") == "kubenode1"
    assert cp.store.get("resourcequotas", _key("1a1", "default", "gpus"))["status"]["used"] == {"requests.amd.com/gpu": "3"}


def test_lost_node_taints_and_evicts_its_pods(cp):
    """SURVEY §5.3 failure recovery: a node whose agent goes silent gets the unreachable taints;
    after the pods' toleration their controller re-creates them on the nodes that are left."""
    from tritonk8ssupervisor_amd.controlplane.objects import UNREACHABLE, _set_ready

    _nodes(cp, 2)
    cp.create("1a1", "deployments", "default", {"metadata": {"name": "srv"}, "spec": {
        "replicas": 1, "selector": {"matchLabels": {"app": "srv"}}, "template": {
            "metadata": {"labels": {"app": "srv"}}, "spec": {"containers": [{"name": "c", "command": ["sleep", "60"]}]}}}})
    (first,) = _pods(cp, "srv")
    node = _node_of(cp, first)
    stay = lambda name, **tol: {"metadata": {"name": name}, "spec": {
        "containers": [{"name": "c", "command": ["true"]}], "nodeName": node,
        "tolerations": [{"key": UNREACHABLE, "operator": "Exists", "effect": "NoExecute", **tol}]}}
    cp.create("1a1", "pods", "default", stay("forever"))
    cp.create("1a1", "pods", "default", stay("patient", tolerationSeconds=3600))
    cp._node_lost(_key("1a1", node), "lease expired")
    n = cp.store.get("nodes", _key("1a1", node))
    assert {t["effect"] for t in n["spec"]["taints"] if t["key"] == UNREACHABLE} == {"NoSchedule", "NoExecute"}
    assert not cp._taint_manager()  # the default 300 s toleration has not run out
    cp.pod_eviction_timeout = 0
    assert cp._taint_manager()
    cp.reconcile()
    left = _pods(cp)
    assert first not in left and {"forever", "patient"} <= set(left)
    (again,) = _pods(cp, "srv")
    assert _node_of(cp, again) not in (None, node)  # NoSchedule keeps the replacement off the lost node
    ev = [e for e in cp.store.list("events") if e.get("reason") == "TaintManagerEviction"]
    assert ev and ev[0]["involvedObject"]["name"] == first
    # the next heartbeat lifts the taints
    cp.store.patch("nodes", _key("1a1", node), _set_ready)
    assert not cp.store.get("nodes", _key("1a1", node))["spec"]["taints"]
    # a user's NoExecute taint evicts what does not tolerate it at once
    other = _node_of(cp, again)
    cp.store.patch("nodes", _key("1a1", other), lambda o: o["spec"].update(taints=[{"key": "drain", "effect": "NoExecute"}]))
    assert cp._taint_manager()
    assert again not in _pods(cp)


def _job(**spec):
    return {"metadata": {"name": "train"}, "spec": {"completions": 2, "parallelism": 2, "template": {
        "spec": {"restartPolicy": "Never", "containers": [{"name": "c", "command": ["sleep", "60"]}]}}, **spec}}


def _age(cp, kind, name, field, seconds, cond=None):
    """Move a job's timestamp ``seconds`` into the past."""
    import time as _time

    past = _time.strftime("%Y-%m-%dT%H:%M:%SZ", _time.gmtime(_time.time() - seconds))

    def fn(o):
        if cond:
            next(c for c in o["status"]["conditions"] if c["type"] == cond)[field] = past
        else:
            o["status"][field] = past
    cp.store.patch(kind, _key("1a1", "default", name), fn)


def test_job_suspend_resume_deadline_and_ttl(cp):
    cp.create("1a1", "jobs", "default", _job(suspend=True))
    j = cp.store.get("jobs", _key("1a1", "default", "train"))
    assert not _pods(cp, "train") and "startTime" not in j["status"]
    assert [(c["type"], c["status"]) for c in j["status"]["conditions"]] == [("Suspended", "True")]
    body = json.loads(json.dumps(cp._strip(j)))
    body["spec"]["suspend"] = False
    cp.replace("1a1", "jobs", "default", "train", body)
    assert len(_pods(cp, "train")) == 2
    j = cp.store.get("jobs", _key("1a1", "default", "train"))
    assert j["status"]["startTime"] and j["status"]["conditions"][0]["reason"] == "JobResumed"
    # suspending a running job stops its pods
    body = json.loads(json.dumps(cp._strip(j)))
    body["spec"]["suspend"] = True
    cp.replace("1a1", "jobs", "default", "train", body)
    assert not _pods(cp, "train") and cp.store.get("jobs", _key("1a1", "default", "train"))["status"]["active"] == 0
    cp._delete_job("1a1", "default", "train")
    # activeDeadlineSeconds
    cp.create("1a1", "jobs", "default", _job(activeDeadlineSeconds=30, ttlSecondsAfterFinished=60))
    assert len(_pods(cp, "train")) == 2
    cp.reconcile()
    assert len(_pods(cp, "train")) == 2  # not yet
    _age(cp, "jobs", "train", "startTime", 31)
    cp.reconcile()
    j = cp.store.get("jobs", _key("1a1", "default", "train"))
    assert not _pods(cp, "train")
    failed = [c for c in j["status"]["conditions"] if c["type"] == "Failed"]
    assert failed and failed[0]["reason"] == "DeadlineExceeded"
    # ttlSecondsAfterFinished deletes the finished job
    cp.reconcile()
    assert cp.store.get("jobs", _key("1a1", "default", "train")) is not None
    _age(cp, "jobs", "train", "lastTransitionTime", 61, cond="Failed")
    cp.reconcile()
    assert cp.store.get("jobs", _key("1a1", "default", "train")) is None


def test_pod_disruption_budget_and_eviction(cp):
    _nodes(cp, 2)
    cp.create("1a1", "deployments", "default", {"metadata": {"name": "srv"}, "spec": {
        "replicas": 3, "selector": {"matchLabels": {"app": "srv"}}, "template": {
            "metadata": {"labels": {"app": "srv"}}, "spec": {"containers": [{"name": "c", "command": ["sleep", "60"]}]}}}})
    for n in _pods(cp, "srv"):
        _run(cp, n)
    with pytest.raises(HttpError) as e:
        cp.create("1a1", "poddisruptionbudgets", "default", {"metadata": {"name": "bad"}, "spec": {
            "minAvailable": 1, "maxUnavailable": 1, "selector": {"matchLabels": {"app": "srv"}}}})
    assert e.value.status == 422
    cp.create("1a1", "poddisruptionbudgets", "default", {"metadata": {"name": "srv"}, "spec": {
        "minAvailable": "60%", "selector": {"matchLabels": {"app": "srv"}}}})
    st = cp.store.get("poddisruptionbudgets", _key("1a1", "default", "srv"))["status"]
    assert (st["expectedPods"], st["currentHealthy"], st["desiredHealthy"], st["disruptionsAllowed"]) == (3, 3, 2, 1)
    first, second, _third = _pods(cp, "srv")
    cp.evict("1a1", "default", first)
    assert first not in _pods(cp)
    with pytest.raises(HttpError) as e:  # the replacement is not Running yet: 2 healthy, 2 needed
        cp.evict("1a1", "default", second)
    assert e.value.status == 429 and "disruption budget" in e.value.message
    assert e.value.body["details"]["causes"][0]["reason"] == "DisruptionBudget"
    # a pending pod may always go
    (pending,) = [n for n in _pods(cp, "srv") if n not in (second, _third)]
    cp.evict("1a1", "default", pending)
    for n in _pods(cp, "srv"):
        _run(cp, n)
    cp.evict("1a1", "default", second)  # healthy again: 3 of 3
    st = cp.store.get("poddisruptionbudgets", _key("1a1", "default", "srv"))["status"]
    assert st["disruptionsAllowed"] == 0 and st["conditions"][0]["reason"] == "InsufficientPods"
    assert any(ev.get("reason") == "Evicted" for ev in cp.store.list("events"))
    # maxUnavailable 0: nothing may be evicted
    cp.replace("1a1", "poddisruptionbudgets", "default", "srv", {"metadata": {"name": "srv"}, "spec": {
        "maxUnavailable": 0, "selector": {"matchLabels": {"app": "srv"}}}})
    for n in _pods(cp, "srv"):
        _run(cp, n)
    with pytest.raises(HttpError):
        cp.evict("1a1", "default", _pods(cp, "srv")[0])
    d = cp.store.get("deployments", _key("1a1", "default", "srv"))["status"]
    assert {c["type"]: c["status"] for c in d["conditions"]} == {"Available": "True", "Progressing": "True"}


def test_priority_classes_and_preemption(cp):
    from tritonk8ssupervisor_amd.controlplane.objects import GPU

    _nodes(cp, 2, gpus=2)
    with pytest.raises(HttpError) as e:
        cp.create("1a1", "priorityclasses", "", {"metadata": {"name": "system-mine"}, "value": 5})
    assert e.value.status == 422
    cp.create("1a1", "priorityclasses", "", {"metadata": {"name": "low"}, "value": 10, "globalDefault": True})
    cp.create("1a1", "priorityclasses", "", {"metadata": {"name": "prod"}, "value": 1000})
    cp.create("1a1", "priorityclasses", "", {"metadata": {"name": "polite"}, "value": 1000, "preemptionPolicy": "Never"})
    with pytest.raises(HttpError):  # only one default
        cp.create("1a1", "priorityclasses", "", {"metadata": {"name": "other"}, "value": 1, "globalDefault": True})
    gpu_pod = lambda name, gpus, pc=None: {"metadata": {"name": name}, "spec": {
        **({"priorityClassName": pc} if pc else {}),
        "containers": [{"name": "c", "command": ["sleep", "60"], "resources": {"limits": {GPU: str(gpus)}}}]}}
    with pytest.raises(HttpError) as e:
        cp.create("1a1", "pods", "default", gpu_pod("x", 1, "nope"))
    assert e.value.status == 403 and "no PriorityClass" in e.value.message
    # a best-effort sweep fills all four GPUs (the default class)
    cp.create("1a1", "deployments", "default", {"metadata": {"name": "sweep"}, "spec": {
        "replicas": 4, "selector": {"matchLabels": {"app": "sweep"}}, "template": {
            "metadata": {"labels": {"app": "sweep"}}, "spec": {"containers": [{"name": "c", "command": ["sleep", "60"],
                                                                              "resources": {"limits": {GPU: "1"}}}]}}}})
    sweep = _pods(cp, "sweep")
    assert all(_node_of(cp, n) for n in sweep)
    assert cp.store.get("pods", _key("1a1", "default", sweep[0]))["spec"]["priority"] == 10
    # a polite high-priority pod waits
    cp.create("1a1", "pods", "default", gpu_pod("polite", 2, "polite"))
    assert _node_of(cp, "polite") is None
    cp.store.delete("pods", _key("1a1", "default", "polite"))
    # a production job takes a whole node: two sweep pods on one node are preempted
    cp.create("1a1", "pods", "default", gpu_pod("train", 2, "prod"))
    node = _node_of(cp, "train")
    assert node is not None
    p = cp.store.get("pods", _key("1a1", "default", "train"))
    assert p["spec"]["priority"] == 1000 and p["status"]["nominatedNodeName"] == node
    gone = [n for n in sweep if n not in _pods(cp)]
    assert len(gone) == 2
    assert len([e for e in cp.store.list("events") if e.get("reason") == "Preempted"]) == 2
    # the sweep's replacements wait: lower priority cannot preempt the job back
    new = [n for n in _pods(cp, "sweep") if n not in sweep]
    assert len(new) == 2 and all(_node_of(cp, n) is None for n in new)
    # the pod's priority comes from its class, not from the client
    with pytest.raises(HttpError):
        cp.create("1a1", "pods", "default", {**gpu_pod("cheat", 0, "low"), "spec": {
            **gpu_pod("cheat", 0, "low")["spec"], "priority": 999999}})


def test_limit_ranges_default_and_bound_containers(cp):
    _nodes(cp, 1, gpus=8)
    cp.create("1a1", "limitranges", "team", {"metadata": {"name": "lr"}, "spec": {"limits": [
        {"type": "Container", "default": {"cpu": "1", "memory": "1Gi"}, "defaultRequest": {"cpu": "500m"},
         "max": {"cpu": "4"}, "min": {"cpu": "100m"}, "maxLimitRequestRatio": {"cpu": "4"}},
        {"type": "Pod", "max": {"amd.com/gpu": "4"}}]}})
    pod = lambda name, res=None, n=1: {"metadata": {"name": name}, "spec": {"containers": [
        {"name": f"c{i}", "command": ["true"], **({"resources": res} if res else {})} for i in range(n)]}}
    p = cp.create("1a1", "pods", "team", pod("plain"))
    r = p["spec"]["containers"][0]["resources"]
    assert r == {"limits": {"cpu": "1", "memory": "1Gi"}, "requests": {"cpu": "500m", "memory": "1Gi"}}
    p = cp.create("1a1", "pods", "team", pod("own", {"limits": {"cpu": "2"}}))
    assert p["spec"]["containers"][0]["resources"]["requests"]["cpu"] == "2"  # its own limit, not defaultRequest
    for name, res, n, want in (("big", {"limits": {"cpu": "8"}}, 1, "maximum cpu usage per Container is 4"),
                               ("tiny", {"requests": {"cpu": "50m"}, "limits": {"cpu": "100m"}}, 1, "minimum cpu"),
                               ("ratio", {"requests": {"cpu": "100m"}, "limits": {"cpu": "1"}}, 1, "ratio"),
                               ("gpus", {"limits": {"amd.com/gpu": "3"}}, 2, "maximum amd.com/gpu usage per Pod is 4"),
                               ("nolimit", None, 1, None)):
        if want is None:  # (the defaults make this one fine)
            cp.create("1a1", "pods", "team", pod(name, res, n))
            continue
        with pytest.raises(HttpError) as e:
            cp.create("1a1", "pods", "team", pod(name, res, n))
        assert e.value.status == 403 and want in e.value.message, e.value.message
    cp.create("1a1", "pods", "other", pod("free", {"limits": {"cpu": "64"}}))  # other namespaces: no LimitRange
    # a controller's pod gets the defaults too
    cp.create("1a1", "jobs", "team", {"metadata": {"name": "j"}, "spec": {"template": {"spec": {
        "restartPolicy": "Never", "containers": [{"name": "c", "command": ["true"]}]}}}})
    (jp,) = [o for o in cp.store.list("pods") if o["metadata"]["name"].startswith("j-")]
    assert jp["spec"]["containers"][0]["resources"]["limits"]["cpu"] == "1"


def test_job_pod_failure_policy(cp):
    pol = {"rules": [{"action": "FailJob", "onExitCodes": {"containerName": "c", "operator": "In", "values": [42]}},
                     {"action": "Ignore", "onExitCodes": {"operator": "In", "values": [137]}}]}
    cp.create("1a1", "jobs", "default", {"metadata": {"name": "t"}, "spec": {"backoffLimit": 0, "podFailurePolicy": pol,
        "template": {"spec": {"restartPolicy": "Never", "containers": [{"name": "c", "command": ["true"]}]}}}})

    def fail(name, code):
        cp.store.patch("pods", _key("1a1", "default", name), lambda o: o["status"].update(phase="Failed", containerStatuses=[
            {"name": "c", "state": {"terminated": {"exitCode": code}}}]))
        cp.reconcile()

    (first,) = _pods(cp, "t-")
    fail(first, 137)  # a SIGKILL (node pressure, preemption): ignored, not counted, replaced
    j = cp.store.get("jobs", _key("1a1", "default", "t"))
    assert j["status"]["failed"] == 0 and not any(c["type"] == "Failed" for c in j["status"]["conditions"])
    (second,) = [n for n in _pods(cp, "t-") if n != first]
    fail(second, 42)  # the program's "bad config" code: the Job fails at once
    j = cp.store.get("jobs", _key("1a1", "default", "t"))
    failed = [c for c in j["status"]["conditions"] if c["type"] == "Failed"]
    assert failed and failed[0]["reason"] == "PodFailurePolicy" and "exit code 42" in failed[0]["message"]


def test_graceful_pod_deletion_and_pod_gc(cp):
    """A running pod on a node with a live agent goes Terminating (deletionTimestamp) and keeps its
    GPUs; its controller replaces it at once; the pod GC force-deletes it if no agent confirms."""
    import time as _time

    from tritonk8ssupervisor_amd.controlplane.objects import GPU

    _nodes(cp, 1, gpus=1)
    cp.leases[_key("1a1", "kubenode1")] = _time.monotonic()
    cp.create("1a1", "deployments", "default", {"metadata": {"name": "g"}, "spec": {
        "replicas": 1, "selector": {"matchLabels": {"app": "g"}}, "template": {
            "metadata": {"labels": {"app": "g"}}, "spec": {"terminationGracePeriodSeconds": 5, "containers": [
                {"name": "c", "command": ["sleep", "60"], "resources": {"limits": {GPU: "1"}}}]}}}})
    (old,) = _pods(cp, "g")
    _run(cp, old)
    cp._delete_pod("1a1", "default", old)
    p = cp.store.get("pods", _key("1a1", "default", old))
    assert p["metadata"]["deletionTimestamp"] and p["metadata"]["deletionGracePeriodSeconds"] == 5
    cp.reconcile()
    new = [n for n in _pods(cp, "g") if n != old]
    assert len(new) == 1 and _node_of(cp, new[0]) is None  # replaced, but the GPU is still held
    assert not cp._pod_gc()  # within its grace period (+15 s)
    cp.store.patch("pods", _key("1a1", "default", old), lambda o: o["metadata"].__setitem__(
        "deletionTimestamp", _time.strftime("%Y-%m-%dT%H:%M:%SZ", _time.gmtime(_time.time() - 20))))
    assert cp._pod_gc()
    cp.reconcile()
    assert old not in _pods(cp) and _node_of(cp, new[0]) == "kubenode1"
    # a pod that is not running (or on a node without a live agent) goes at once
    cp._delete_pod("1a1", "default", new[0])
    assert new[0] not in _pods(cp)


def test_pod_security_standards_unit():
    from tritonk8ssupervisor_amd.controlplane.podsecurity import violations

    good = {"spec": {"securityContext": {"runAsNonRoot": True, "seccompProfile": {"type": "RuntimeDefault"}},
                     "containers": [{"name": "c", "securityContext": {
                         "allowPrivilegeEscalation": False, "capabilities": {"drop": ["ALL"]}}}],
                     "volumes": [{"name": "v", "emptyDir": {}}]}}
    assert violations(good, "restricted") == [] and violations(good, "baseline") == []
    bad = {"spec": {"containers": [{"name": "c", "securityContext": {"privileged": True, "capabilities": {"add": ["SYS_ADMIN"]}},
                                    "ports": [{"containerPort": 80, "hostPort": 80}]}]}}
    v = violations(bad, "baseline")
    assert any("privileged" in x for x in v) and any("SYS_ADMIN" in x for x in v) and any("hostPort" in x for x in v)
    assert violations(bad, "privileged") == []
    assert any("runAsNonRoot" in x for x in violations({"spec": {"containers": [{"name": "c"}]}}, "restricted"))


def test_evicted_pod_carries_a_disruption_target(cp):
    import time as _time

    _nodes(cp, 1)
    cp.leases[_key("1a1", "kubenode1")] = _time.monotonic()
    cp.create("1a1", "pods", "default", {"metadata": {"name": "p"}, "spec": {"containers": [{"name": "c", "command": ["x"]}]}})
    cp.store.patch("pods", _key("1a1", "default", "p"), lambda o: o["status"].update(phase="Running"))
    cp.evict("1a1", "default", "p")
    p = cp.store.get("pods", _key("1a1", "default", "p"))
    dt = [c for c in p["status"]["conditions"] if c["type"] == "DisruptionTarget"]
    assert p["metadata"]["deletionTimestamp"] and dt and dt[0]["reason"] == "EvictionByEvictionAPI"


def test_lease_loop_forgives_its_own_stalls(cp):
    """A stalled event loop (a slow webhook) must not mark heartbeating nodes lost."""
    import asyncio
    import time as _time

    _nodes(cp, 1)
    key = _key("1a1", "kubenode1")

    async def run():
        cp.leases[key] = _time.monotonic()
        task = asyncio.ensure_future(cp.lease_loop())
        await asyncio.sleep(0.3)
        _time.sleep(cp.node_grace + 1)  # the loop is blocked longer than the grace period
        cp.leases[key] = cp.leases[key]  # (no heartbeat got through meanwhile)
        await asyncio.sleep(0.6)
        task.cancel()

    asyncio.run(run())
    n = cp.store.get("nodes", key)
    assert [c["status"] for c in n["status"]["conditions"] if c["type"] == "Ready"] == ["True"]


def test_topology_spread_constraints(cp):
    _nodes(cp, 3)  # zone a: kubenode1, kubenode2; zone b: kubenode3
    spread = [{"maxSkew": 1, "topologyKey": "zone", "whenUnsatisfiable": "DoNotSchedule",
               "labelSelector": {"matchLabels": {"app": "web"}}}]
    cp.create("1a1", "deployments", "default", {"metadata": {"name": "web"}, "spec": {
        "replicas": 4, "selector": {"matchLabels": {"app": "web"}}, "template": {
            "metadata": {"labels": {"app": "web"}}, "spec": {"topologySpreadConstraints": spread,
                                                              "containers": [{"name": "c", "command": ["x"]}]}}}})
    zones = {}
    for n in _pods(cp, "web"):
        nn = _node_of(cp, n)
        zones[nn] = zones.get(nn, 0) + 1
    per_zone = {"a": zones.get("kubenode1", 0) + zones.get("kubenode2", 0), "b": zones.get("kubenode3", 0)}
    assert per_zone == {"a": 2, "b": 2}  # skew <= 1 across the two zones
    # ScheduleAnyway only prefers: hostname spread over three nodes
    cp.create("1a1", "deployments", "default", {"metadata": {"name": "soft"}, "spec": {
        "replicas": 3, "selector": {"matchLabels": {"app": "soft"}}, "template": {
            "metadata": {"labels": {"app": "soft"}}, "spec": {"topologySpreadConstraints": [
                {"maxSkew": 1, "topologyKey": "kubernetes.io/hostname", "whenUnsatisfiable": "ScheduleAnyway",
                 "labelSelector": {"matchLabels": {"app": "soft"}}}], "containers": [{"name": "c", "command": ["x"]}]}}}})
    assert sorted(_node_of(cp, n) for n in _pods(cp, "soft")) == ["kubenode1", "kubenode2", "kubenode3"]


def test_persistent_volumes_and_storage_class(cp):
    _nodes(cp, 2)
    cp.create("1a1", "persistentvolumeclaims", "default", {"metadata": {"name": "data"}, "spec": {
        "resources": {"requests": {"storage": "10Gi"}}}})
    sc = cp.store.get("storageclasses", _key("1a1", "", "tk8s-local"))
    assert sc["volumeBindingMode"] == "WaitForFirstConsumer"
    pvc = cp.store.get("persistentvolumeclaims", _key("1a1", "default", "data"))
    pv = cp.store.get("persistentvolumes", _key("1a1", "", pvc["spec"]["volumeName"]))
    assert pv["spec"]["claimRef"]["name"] == "data" and pv["spec"]["capacity"]["storage"] == "10Gi"
    assert "nodeAffinity" not in pv["spec"]
    cp.create("1a1", "pods", "default", {"metadata": {"name": "user"}, "spec": {
        "containers": [{"name": "c", "command": ["x"]}], "volumes": [{"name": "d", "persistentVolumeClaim": {"claimName": "data"}}]}})
    node = _node_of(cp, "user")
    pv = cp.store.get("persistentvolumes", _key("1a1", "", pvc["spec"]["volumeName"]))
    assert pv["spec"]["nodeAffinity"]["required"]["nodeSelectorTerms"][0]["matchExpressions"][0]["values"] == [node]
    cp._remove("1a1", "persistentvolumeclaims", "default", "data")
    assert cp.store.get("persistentvolumes", _key("1a1", "", pvc["spec"]["volumeName"])) is None


def test_scheduler_fits_cpu_and_memory_requests(cp):
    _nodes(cp, 2)
    for i in (1, 2):
        cp.store.patch("nodes", _key("1a1", f"kubenode{i}"), lambda o: o["status"]["allocatable"].update(
            cpu="2", memory="4Gi", pods="110"))
    pod = lambda name, cpu, mem="1Gi": {"metadata": {"name": name}, "spec": {"containers": [
        {"name": "c", "command": ["x"], "resources": {"requests": {"cpu": cpu, "memory": mem}}}]}}
    cp.create("1a1", "pods", "default", pod("a", "1500m"))
    cp.create("1a1", "pods", "default", pod("b", "1500m"))
    assert {_node_of(cp, "a"), _node_of(cp, "b")} == {"kubenode1", "kubenode2"}  # one per node: 3 CPUs do not fit 2
    cp.create("1a1", "pods", "default", pod("c", "1"))
    p = cp.store.get("pods", _key("1a1", "default", "c"))
    assert p["spec"].get("nodeName") is None and "Insufficient cpu" in p["status"]["conditions"][0]["message"]
    cp.create("1a1", "pods", "default", pod("d", "100m", "8Gi"))
    assert "Insufficient memory" in cp.store.get("pods", _key("1a1", "default", "d"))["status"]["conditions"][0]["message"]
    cp.create("1a1", "pods", "default", pod("e", "100m"))  # small enough for either node
    assert _node_of(cp, "e") is not None


def test_repeated_events_are_aggregated(cp):
    import time as _time

    for _ in range(50):  # a controller failing the same way on every pass
        cp._event("1a1", "default", {"kind": "Job", "name": "j"}, "FailedCreate", "no room", "Warning")
    evs = [e for e in cp.store.list("events") if e["reason"] == "FailedCreate"]
    assert len(evs) == 1 and evs[0]["count"] == 1
    _time.sleep(1.05)
    cp._event("1a1", "default", {"kind": "Job", "name": "j"}, "FailedCreate", "no room", "Warning")
    evs = [e for e in cp.store.list("events") if e["reason"] == "FailedCreate"]
    assert len(evs) == 1 and evs[0]["count"] == 2
    cp._event("1a1", "default", {"kind": "Job", "name": "j"}, "FailedCreate", "other reason", "Warning")
    assert len([e for e in cp.store.list("events") if e["reason"] == "FailedCreate"]) == 2


def test_ingress_classes(cp):
    cp.create("1a1", "services", "default", {"metadata": {"name": "web"}, "spec": {"ports": [{"port": 80}]}})
    ing = lambda name, **spec: {"metadata": {"name": name}, "spec": {**spec, "rules": [{"host": f"{name}.local", "http": {
        "paths": [{"path": "/", "pathType": "Prefix", "backend": {"service": {"name": "web", "port": {"number": 80}}}}]}}]}}
    cp.create("1a1", "ingresses", "default", ing("plain"))
    cp.create("1a1", "ingresses", "default", ing("mine", ingressClassName="tk8s"))
    cp.create("1a1", "ingresses", "default", ing("theirs", ingressClassName="nginx"))
    hosts = {r[0] for r in cp._ingress_routes()}
    assert hosts == {"plain.local", "mine.local"}
    ic = cp.store.get("ingressclasses", _key("1a1", "", "tk8s"))
    assert ic["metadata"]["annotations"]["ingressclass.kubernetes.io/is-default-class"] == "true"


def test_hpa_rate_limit_policies():
    from tritonk8ssupervisor_amd.controlplane.metrics_api import _rate_limit

    assert _rate_limit({}, 2, 20) == 6  # default up: max(+100 % = 4, +4 pods = 6)
    assert _rate_limit({}, 10, 1) == 1  # default down: up to 100 %
    beh = {"scaleUp": {"policies": [{"type": "Pods", "value": 1, "periodSeconds": 60}]},
           "scaleDown": {"policies": [{"type": "Percent", "value": 50, "periodSeconds": 60}]}}
    assert _rate_limit(beh, 3, 10) == 4 and _rate_limit(beh, 10, 1) == 5
    assert _rate_limit({"scaleDown": {"selectPolicy": "Disabled"}}, 10, 1) == 10
    two = {"scaleUp": {"selectPolicy": "Min", "policies": [{"type": "Pods", "value": 2}, {"type": "Percent", "value": 10}]}}
    assert _rate_limit(two, 10, 30) == 11  # the smaller of +2 and +10 %


def test_hpa_rate_limit_counts_each_policys_period():
    """a policy's budget is per periodSeconds, not per reconcile -- two steps inside
    one window add up to what the policy allows, and the budget comes back when it ends."""
    from tritonk8ssupervisor_amd.controlplane.metrics_api import _rate_limit

    beh = {"scaleUp": {"policies": [{"type": "Pods", "value": 1, "periodSeconds": 60}]},
           "scaleDown": {"policies": [{"type": "Percent", "value": 50, "periodSeconds": 120}]}}
    assert _rate_limit(beh, 4, 10, [(0.0, 1)], now=15.0) == 4  # 3 -> 4 at t=0 spent the minute
    assert _rate_limit(beh, 4, 10, [(0.0, 1)], now=61.0) == 5  # a new window
    # down: 50 % of the 10 replicas at the window's start, whatever steps it took to get there
    assert _rate_limit(beh, 7, 1, [(0.0, -3)], now=30.0) == 5
    assert _rate_limit(beh, 5, 1, [(0.0, -3), (30.0, -2)], now=60.0) == 5
    assert _rate_limit(beh, 5, 1, [(0.0, -3), (30.0, -2)], now=125.0) == 3  # 50 % of 7 (the t=0 step aged out)
    # the default scale-up policy (100 % or 4 pods per 15 s): 2 -> 6 -> hold -> 6 -> 12
    assert _rate_limit({}, 6, 40, [(0.0, 4)], now=5.0) == 6
    assert _rate_limit({}, 6, 40, [(0.0, 4)], now=16.0) == 12


def test_hpa_controller_honours_period_seconds(cp):
    """The controller records its own scale events: with 1 pod per 60 s, reconciles 15 s apart
    move the target by one replica per minute, not one per reconcile."""
    cp.create("1a1", "deployments", "default", {"metadata": {"name": "web"}, "spec": {
        "replicas": 1, "selector": {"matchLabels": {"app": "web"}},
        "template": {"metadata": {"labels": {"app": "web"}}, "spec": {"containers": [{
            "name": "c", "command": ["x"], "resources": {"requests": {"cpu": "100m"}}}]}}}})
    cp.create("1a1", "horizontalpodautoscalers", "default", {"metadata": {"name": "web"}, "spec": {
        "scaleTargetRef": {"apiVersion": "apps/v1", "kind": "Deployment", "name": "web"},
        "minReplicas": 1, "maxReplicas": 10,
        "metrics": [{"type": "Resource", "resource": {"name": "cpu", "target": {"type": "Utilization",
                                                                                "averageUtilization": 50}}}],
        "behavior": {"scaleUp": {"policies": [{"type": "Pods", "value": 1, "periodSeconds": 60}]}}}})
    seen = []
    for t in (1000.0, 1015.0, 1030.0, 1061.0):
        for n in _pods(cp, "web-"):
            cp.store.patch("pods", _key("1a1", "default", n), lambda o: o["status"].update(phase="Running"))
        cp._ingest_metrics("1a1", "kubenode1", {"pods": {f"default/{n}": [{"name": "c", "cpu_cores": 0.5, "memory_bytes": 0}]
                                                         for n in _pods(cp, "web-")}})
        cp._ctl_hpas("1a1", now=t)
        seen.append(cp.store.get("deployments", _key("1a1", "default", "web"))["spec"]["replicas"])
    assert seen == [2, 2, 2, 3], seen


def test_daemonset_rolling_update(cp):
    _nodes(cp, 3)
    cp.create("1a1", "daemonsets", "default", {"metadata": {"name": "mon"}, "spec": {
        "selector": {"matchLabels": {"app": "mon"}}, "template": {"metadata": {"labels": {"app": "mon"}},
                                                                  "spec": {"containers": [{"name": "c", "command": ["v1"]}]}}}})
    names = _pods(cp, "mon")
    assert len(names) == 3
    for n in names:
        cp.store.patch("pods", _key("1a1", "default", n), lambda o: o["status"].update(phase="Running"))
    body = json.loads(json.dumps(cp._strip(cp.store.get("daemonsets", _key("1a1", "default", "mon")))))
    body["spec"]["template"]["spec"]["containers"][0]["command"] = ["v2"]
    cp.replace("1a1", "daemonsets", "default", "mon", body)
    cmds = lambda: sorted(cp.store.get("pods", _key("1a1", "default", n))["spec"]["containers"][0]["command"][0]
                          for n in _pods(cp, "mon"))
    assert cmds() == ["v1", "v1", "v2"]  # one node at a time (maxUnavailable 1)
    for _ in range(3):
        for n in _pods(cp, "mon"):
            cp.store.patch("pods", _key("1a1", "default", n), lambda o: o["status"].update(phase="Running"))
        cp.reconcile()
    assert cmds() == ["v2", "v2", "v2"]
    assert cp.store.get("daemonsets", _key("1a1", "default", "mon"))["status"]["updatedNumberScheduled"] == 3
