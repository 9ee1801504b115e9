"""kustomize.py: a base + overlay build (generators with hashed names and rewritten references,
prefix/suffix, namespace, labels, annotations, images, replicas, strategic-merge and JSON 6902
patches), and ``kubectl apply -k`` / ``kubectl kustomize`` against a live control plane. Parity of
the generated-name hash with the kustomize binary is unpinned (none is installed)."""
import json

import pytest
import yaml

from tritonk8ssupervisor_amd import kustomize

from test_k8s_wire import kube  # noqa: F401  (kube is a fixture)

DEPLOY = {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": "web", "labels": {"app": "web"}},
          "spec": {"replicas": 1, "selector": {"matchLabels": {"app": "web"}}, "template": {
              "metadata": {"labels": {"app": "web"}},
              "spec": {"containers": [{"name": "web", "image": "nginx:1.25", "command": ["sleep", "60"],
                                       "envFrom": [{"configMapRef": {"name": "settings"}}],
                                       "env": [{"name": "PW", "valueFrom": {"secretKeyRef": {"name": "creds", "key": "pw"}}}]}],
                       "volumes": [{"name": "cfg", "configMap": {"name": "settings"}}]}}}}
SVC = {"apiVersion": "v1", "kind": "Service", "metadata": {"name": "web"},
       "spec": {"selector": {"app": "web"}, "ports": [{"port": 80}]}}


def _tree(tmp_path):
    base = tmp_path / "base"
    base.mkdir()
    (base / "deploy.yaml").write_text(yaml.safe_dump(DEPLOY))
    (base / "svc.yaml").write_text(yaml.safe_dump(SVC))
    (base / "app.env").write_text("MODE=base\nLEVEL=1\n")
    (base / "kustomization.yaml").write_text(yaml.safe_dump({
        "resources": ["deploy.yaml", "svc.yaml"],
        "configMapGenerator": [{"name": "settings", "envs": ["app.env"]}],
        "secretGenerator": [{"name": "creds", "literals": ["pw=s3cret"]}]}))
    prod = tmp_path / "prod"
    prod.mkdir()
    (prod / "more.yaml").write_text(yaml.safe_dump({"spec": {"template": {"spec": {"containers": [
        {"name": "web", "resources": {"limits": {"amd.com/gpu": "1"}}}]}}}, "kind": "Deployment",
        "apiVersion": "apps/v1", "metadata": {"name": "web"}}))
    (prod / "kustomization.yaml").write_text(yaml.safe_dump({
        "resources": ["../base"], "namespace": "prod", "namePrefix": "p-",
        "commonLabels": {"env": "prod"}, "commonAnnotations": {"team": "ml"},
        "images": [{"name": "nginx", "newTag": "1.27"}], "replicas": [{"name": "web", "count": 3}],
        "configMapGenerator": [{"name": "settings", "behavior": "merge", "literals": ["MODE=prod"]}],
        "patches": [{"path": "more.yaml"},
                    {"target": {"kind": "Service", "name": "web"}, "patch": yaml.safe_dump(
                        [{"op": "add", "path": "/spec/type", "value": "NodePort"}])}]}))
    return base, prod


def test_base_and_overlay_build(tmp_path):
    base, prod = _tree(tmp_path)
    objs = {(o["kind"], o["metadata"]["name"]): o for o in kustomize.build(base)}
    cm = next(o for (k, n), o in objs.items() if k == "ConfigMap")
    assert cm["metadata"]["name"].startswith("settings-") and cm["data"] == {"MODE": "base", "LEVEL": "1"}
    dep = objs[("Deployment", "web")]
    c = dep["spec"]["template"]["spec"]["containers"][0]
    assert c["envFrom"][0]["configMapRef"]["name"] == cm["metadata"]["name"]  # references follow the hash
    sec = next(o for (k, n), o in objs.items() if k == "Secret")
    assert c["env"][0]["valueFrom"]["secretKeyRef"]["name"] == sec["metadata"]["name"]
    objs = {(o["kind"], o["metadata"]["name"].split("-")[0] if o["kind"] in ("ConfigMap", "Secret") else
             o["metadata"]["name"]): o for o in kustomize.build(prod)}
    dep, svc, cm = objs[("Deployment", "p-web")], objs[("Service", "p-web")], objs[("ConfigMap", "p")]
    assert cm["data"] == {"MODE": "prod", "LEVEL": "1"} and cm["metadata"]["name"].startswith("p-settings-")
    assert all(o["metadata"]["namespace"] == "prod" for o in objs.values())
    assert dep["spec"]["replicas"] == 3 and dep["metadata"]["labels"]["env"] == "prod"
    assert dep["spec"]["selector"]["matchLabels"] == {"app": "web", "env": "prod"}
    assert dep["spec"]["template"]["metadata"]["labels"]["env"] == "prod"
    assert dep["spec"]["template"]["metadata"]["annotations"]["team"] == "ml"
    c = dep["spec"]["template"]["spec"]["containers"][0]
    assert c["image"] == "nginx:1.27" and c["resources"]["limits"]["amd.com/gpu"] == "1"
    assert c["envFrom"][0]["configMapRef"]["name"] == cm["metadata"]["name"]
    assert dep["spec"]["template"]["spec"]["volumes"][0]["configMap"]["name"] == cm["metadata"]["name"]
    assert svc["spec"]["type"] == "NodePort" and svc["spec"]["selector"] == {"app": "web", "env": "prod"}
    # a content change changes the generated name (a rolling update of the pods using it)
    old = cm["metadata"]["name"]
    (base / "app.env").write_text("MODE=base\nLEVEL=2\n")
    new = next(o for o in kustomize.build(prod) if o["kind"] == "ConfigMap")["metadata"]["name"]
    assert new != old
    with pytest.raises(kustomize.KustomizeError):
        kustomize.build(tmp_path / "nowhere")


def test_kubectl_apply_k_and_kustomize(kube, tmp_path, capsys):
    from tritonk8ssupervisor_amd.cli import kubectl

    base, _prod = _tree(tmp_path)
    pid = kube.prefix.split("/")[3]
    cfg = tmp_path / "kubeconfig.json"
    cfg.write_text(json.dumps(kube.get(f"/env/{pid}/kubernetes/kubectl", query={"format": "json"})))
    kc = lambda *a: kubectl.main(["--kubeconfig", str(cfg), *a], workdir=str(tmp_path))
    assert kc("kustomize", str(base)) == 0
    docs = [d for d in yaml.safe_load_all(capsys.readouterr().out) if d]
    assert {d["kind"] for d in docs} == {"Deployment", "Service", "ConfigMap", "Secret"}
    assert kc("apply", "-k", str(base)) == 0
    out = capsys.readouterr().out
    assert "deployment/web" in out and "configmap/settings-" in out
    dep = kube.get(kube.k8s("/apis/apps/v1/namespaces/default/deployments/web"))
    name = dep["spec"]["template"]["spec"]["containers"][0]["envFrom"][0]["configMapRef"]["name"]
    assert kube.get(kube.k8s(f"/api/v1/namespaces/default/configmaps/{name}"))["data"]["MODE"] == "base"
    assert kc("delete", "-k", str(base)) == 0
    assert "4 object(s) deleted" in capsys.readouterr().out
