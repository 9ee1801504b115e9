"""The everyday kubectl verbs of cli/kubectl_more.py against a live control plane: run, set,
autoscale, patch, replace, edit, diff, events, explain, api-resources/-versions, auth can-i,
config, rollout pause/resume. Parity with a real kubectl binary is unpinned (none is installed)."""
import json
import sys

import pytest

from test_k8s_wire import DEPLOY, kube  # noqa: F401  (kube is a fixture)


@pytest.fixture
def kc(kube, tmp_path, capsys):
    from tritonk8ssupervisor_amd.cli import kubectl

    pid = kube.prefix.split("/")[3]
    cfg = tmp_path / "kubeconfig.json"
    cfg.write_text(json.dumps(kube.get(f"/env/{pid}/kubernetes/kubectl", query={"format": "json"})))

    def run(*a):
        rc = kubectl.main(["--kubeconfig", str(cfg), *a], workdir=str(tmp_path))
        out = capsys.readouterr()
        return rc, out.out, out.err
    run.kube, run.tmp = kube, tmp_path
    return run


def test_run_set_patch_and_autoscale(kc):
    rc, out, _ = kc("run", "dbg", "--image=python", "--env=A=1", "--limits=amd.com/gpu=1", "--restart=Never",
                    "--dry-run=client", "-o", "yaml", "--", "sleep", "5")
    assert rc == 0 and "amd.com/gpu: '1'" in out and "run: dbg" in out and "- sleep" in out
    assert kc("run", "dbg", "--image=python", "--", "sleep", "5")[:2] == (0, "pod/dbg created\n")
    pod = kc.kube.get(kc.kube.k8s("/api/v1/namespaces/default/pods/dbg"))
    assert pod["spec"]["containers"][0]["args"] == ["sleep", "5"] and pod["metadata"]["labels"] == {"run": "dbg"}
    man = kc.tmp / "web.json"
    man.write_text(json.dumps(DEPLOY))
    assert kc("apply", "-f", str(man))[0] == 0
    cname = DEPLOY["spec"]["template"]["spec"]["containers"][0]["name"]
    assert kc("set", "image", "deployment/web", f"{cname}=nginx:1.27")[0] == 0
    assert kc("set", "env", "deploy/web", "MODE=fast")[0] == 0
    assert kc("set", "resources", "deploy", "web", "--limits=cpu=2")[0] == 0
    d = kc.kube.get(kc.kube.k8s("/apis/apps/v1/namespaces/default/deployments/web"))
    c = d["spec"]["template"]["spec"]["containers"][0]
    assert c["image"] == "nginx:1.27" and {"name": "MODE", "value": "fast"} in c["env"] and c["resources"]["limits"]["cpu"] == "2"
    with pytest.raises(SystemExit, match="unable to find container"):
        kc("set", "image", "deploy/web", "nope=x")
    rc, out, _ = kc("patch", "deployment", "web", "-p", '{"spec":{"replicas":3}}')
    assert rc == 0 and "patched" in out
    rc, out, _ = kc("patch", "deploy", "web", "--type", "json", "-p", '[{"op":"replace","path":"/spec/replicas","value":2}]')
    assert rc == 0
    assert kc.kube.get(kc.kube.k8s("/apis/apps/v1/namespaces/default/deployments/web"))["spec"]["replicas"] == 2
    assert kc("autoscale", "deployment", "web", "--min=1", "--max=4", "--cpu-percent=50")[0] == 0
    hpa = kc.kube.get(kc.kube.k8s("/apis/autoscaling/v2/namespaces/default/horizontalpodautoscalers/web"))
    assert hpa["spec"]["maxReplicas"] == 4 and hpa["spec"]["metrics"][0]["resource"]["target"]["averageUtilization"] == 50


def test_diff_replace_edit_and_pause(kc, monkeypatch):
    man = kc.tmp / "web.json"
    man.write_text(json.dumps(DEPLOY))
    rc, out, _ = kc("diff", "-f", str(man))
    assert rc == 1 and "+kind: Deployment" in out  # not there yet: all added
    assert kc("apply", "-f", str(man))[0] == 0
    assert kc("diff", "-f", str(man))[:2] == (0, "")
    man.write_text(json.dumps({**DEPLOY, "spec": {**DEPLOY["spec"], "replicas": 5}}))
    rc, out, _ = kc("diff", "-f", str(man))
    assert rc == 1 and "+  replicas: 5" in out
    assert kc("replace", "-f", str(man))[0] == 0
    assert kc.kube.get(kc.kube.k8s("/apis/apps/v1/namespaces/default/deployments/web"))["spec"]["replicas"] == 5
    # edit through a scripted "editor"
    script = kc.tmp / "ed.py"
    script.write_text("import sys,re\np=sys.argv[1]\ns=open(p).read()\nopen(p,'w').write(s.replace('replicas: 5','replicas: 4'))\n")
    monkeypatch.setenv("KUBE_EDITOR", f"{sys.executable} {script}")
    rc, out, _ = kc("edit", "deployment/web")
    assert rc == 0 and "edited" in out
    assert kc.kube.get(kc.kube.k8s("/apis/apps/v1/namespaces/default/deployments/web"))["spec"]["replicas"] == 4
    monkeypatch.setenv("KUBE_EDITOR", "true")
    assert "no changes" in kc("edit", "deployment/web")[1]
    # rollout pause holds a template change back; resume rolls it out
    assert kc("rollout", "pause", "deploy/web")[1] == "deployment.apps/web paused\n"
    d0 = kc.kube.get(kc.kube.k8s("/apis/apps/v1/namespaces/default/deployments/web"))
    hashes = lambda: {p["metadata"]["labels"].get("pod-template-hash") for p in kc.kube.get(
        kc.kube.k8s("/api/v1/namespaces/default/pods"), query={"labelSelector": "app=web"})["items"]}
    before = hashes()
    cname = d0["spec"]["template"]["spec"]["containers"][0]["name"]
    assert kc("set", "image", "deploy/web", f"{cname}=nginx:2")[0] == 0
    assert hashes() == before
    cond = {c["type"]: c["reason"] for c in kc.kube.get(
        kc.kube.k8s("/apis/apps/v1/namespaces/default/deployments/web"))["status"]["conditions"]}
    assert cond["Progressing"] == "DeploymentPaused"
    assert kc("rollout", "resume", "deploy/web")[0] == 0
    assert hashes() != before


def test_discovery_auth_events_explain_and_config(kc):
    rc, out, _ = kc("api-resources")
    assert rc == 0 and any(l.split()[:1] == ["poddisruptionbudgets"] for l in out.splitlines())
    rc, out, _ = kc("api-resources", "--namespaced=false", "-o", "name")
    assert "nodes" in out.split() and "pods" not in out.split()
    rc, out, _ = kc("api-versions")
    assert "apps/v1" in out.split() and "policy/v1" in out.split()
    assert kc("auth", "can-i", "create", "deployments")[:2] == (0, "yes\n")
    rc, out, _ = kc("explain", "deployment")
    assert rc == 0 and "KIND:       Deployment" in out and "spec\t<object>" in out
    rc, out, _ = kc("explain", "pods.metadata")
    assert rc == 0 and "FIELD: metadata" in out
    assert kc("run", "ev", "--image=python", "--", "true")[0] == 0
    rc, out, _ = kc("events", "--for", "pod/ev")
    assert rc == 0 and out.startswith("LAST SEEN")
    rc, out, _ = kc("config", "view")
    assert rc == 0 and "REDACTED" in out
    assert kc("config", "get-contexts")[0] == 0


def test_get_output_formats_sort_and_watch(kc):
    import threading
    import time as _time

    for n, r in (("b", 3), ("a", 1), ("c", 2)):
        kc.kube.post(kc.kube.k8s("/api/v1/namespaces/default/configmaps"), {
            "apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": n, "labels": {"rank": str(r)}}, "data": {"r": str(r)}})
    rc, out, _ = kc("get", "cm", "-o", "name")
    assert rc == 0 and {"configmap/a", "configmap/b", "configmap/c"} <= set(out.split())
    rc, out, _ = kc("get", "cm", "-l", "rank", "--sort-by=.data.r", "-o", "jsonpath={.items[*].metadata.name}")
    assert out.strip() == "a c b"
    rc, out, _ = kc("get", "cm", "a", "-o", "jsonpath={.metadata.name}={.data.r}")
    assert out.strip() == "a=1"
    rc, out, _ = kc("get", "cm", "-l", "rank", "-o", "custom-columns=NAME:.metadata.name,RANK:.metadata.labels.rank",
                    "--sort-by=.metadata.name")
    lines = out.split("\n")
    assert lines[0].split() == ["NAME", "RANK"] and lines[1].split() == ["a", "1"]
    # -w: rows as the objects change, until --timeout
    def later():
        _time.sleep(0.5)
        kc.kube.post(kc.kube.k8s("/api/v1/namespaces/default/configmaps"), {
            "apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "late"}, "data": {}})
    threading.Thread(target=later, daemon=True).start()
    rc, out, _ = kc("get", "cm", "-w", "--timeout=2s")
    assert rc == 0 and any(l.split()[:1] == ["late"] for l in out.splitlines()[-3:])


def test_describe_node_and_pod(kc):
    rc, out, _ = kc("describe", "node", "kubenode1")
    assert rc == 0 and "Taints:       <none>" in out and "Allocated resources:" in out and "amd.com/gpu: 0 of" in out
    assert kc("taint", "nodes", "kubenode1", "gpu=mi355x:NoSchedule")[0] == 0
    assert "gpu=mi355x:NoSchedule" in kc("describe", "no/kubenode1")[1]
    kc("run", "d", "--image=python", "--", "sleep", "5")
    rc, out, _ = kc("describe", "pod/d")
    assert rc == 0 and "Name:         d" in out and "Status:" in out


def test_create_job_from_a_cronjob(kc):
    kc.kube.post(kc.kube.k8s("/apis/batch/v1/namespaces/default/cronjobs"), {
        "apiVersion": "batch/v1", "kind": "CronJob", "metadata": {"name": "nightly"},
        "spec": {"schedule": "0 3 * * *", "jobTemplate": {"metadata": {"labels": {"team": "ml"}}, "spec": {"template": {
            "spec": {"restartPolicy": "Never", "containers": [{"name": "c", "command": ["true"]}]}}}}}})
    rc, out, _ = kc("create", "job", "now", "--from=cronjob/nightly")
    assert rc == 0 and out == "job.batch/now created\n"
    j = kc.kube.get(kc.kube.k8s("/apis/batch/v1/namespaces/default/jobs/now"))
    assert j["metadata"]["labels"]["team"] == "ml"
    assert j["metadata"]["annotations"]["cronjob.kubernetes.io/instantiate"] == "manual"
    rc, out, _ = kc("create", "job", "once", "--image=python", "--", "echo", "hi")
    assert rc == 0 and kc.kube.get(kc.kube.k8s("/apis/batch/v1/namespaces/default/jobs/once"))["spec"]["template"][
        "spec"]["containers"][0]["command"] == ["echo", "hi"]


def test_get_all(kc):
    kc("run", "solo", "--image=python", "--", "sleep", "5")
    kc.kube.post(kc.kube.k8s("/api/v1/namespaces/default/services"), {
        "apiVersion": "v1", "kind": "Service", "metadata": {"name": "front"}, "spec": {"ports": [{"port": 80}]}})
    rc, out, _ = kc("get", "all")
    assert rc == 0 and "pod/solo" in out and "service/front" in out
