"""What a stock kubectl needs beyond CRUD (controlplane/k8s_openapi.py, controlplane/ssa.py):
OpenAPI v3 documents (so ``kubectl apply`` validates without ``--validate=false``), server-side
field validation, ``dryRun=All``, managed fields and server-side apply.

No kubectl binary is installed here: the tests replay, request by request, what kubectl sends
and reads -- the OpenAPI v3 root, the group-version document, the PATCH operation's
``x-kubernetes-group-version-kind`` and its ``fieldValidation`` query parameter (the check
kubectl's query-param verifier makes), then ``PATCH application/apply-patch+yaml`` with
``fieldManager``/``force``. Parity with a real kubectl binary is unpinned."""
import http.client
import json

import pytest

from tritonk8ssupervisor_amd.controlplane import k8s_openapi, k8s_wire, ssa

from test_k8s_wire import DEPLOY, _raw, kube  # noqa: F401  (kube is a fixture)

APPLY = k8s_wire.APPLY_PATCH
DPATH = "/apis/apps/v1/namespaces/default/deployments"


def _abs(k, path, accept="application/json"):
    """GET a server-relative URL as client-go does for OpenAPI (no kubeconfig path prefix)."""
    conn = http.client.HTTPConnection(k.host, k.port, timeout=10)
    conn.request("GET", path, headers={"Accept": accept, "Authorization": f"Bearer {k.token}"})
    r = conn.getresponse()
    out = r.status, dict(r.getheaders()), r.read()
    conn.close()
    return out[0], out[1], json.loads(out[2]) if out[2] else None


def _supports_field_validation(doc: dict, gvk: dict) -> bool:
    """kubectl's OpenAPI v3 query-param check: the PATCH operation of this GVK lists the
    ``fieldValidation`` query parameter."""
    for item in doc["paths"].values():
        op = item.get("patch")
        if op and op.get(k8s_openapi.GVK) == gvk:
            return any(p["name"] == "fieldValidation" and p["in"] == "query" for p in op.get("parameters", []))
    raise AssertionError(f"no PATCH operation for {gvk}")


def test_openapi_v3_lets_kubectl_validate_on_the_server(kube):
    st, _, root = _raw(kube, "GET", "/openapi/v3")
    assert st == 200 and set(root["paths"]) == {k8s_openapi.gv_key(g, v) for g, v in k8s_openapi._gvs()}
    assert {"api/v1", "apis/apps/v1", "apis/batch/v1"} <= set(root["paths"])
    for key, ref in root["paths"].items():
        url = ref["serverRelativeURL"]
        # client-go replaces the server URL's path with this one, so it carries the project prefix
        assert url.startswith(f"{kube.prefix}/openapi/v3/{key}?hash="), url
        st, headers, doc = _abs(kube, url)
        assert st == 200 and doc["openapi"].startswith("3.") and "immutable" in headers.get("Cache-Control", "")
        for plural, (g, v, kind, *_r) in k8s_wire.RESOURCES.items():
            if k8s_openapi.gv_key(g, v) != key:
                continue
            assert _supports_field_validation(doc, {"group": g, "version": v, "kind": kind}), kind
            schema = doc["components"]["schemas"][k8s_openapi._schema_name(g, v, kind)]
            assert schema[k8s_openapi.GVK] == [{"group": g, "version": v, "kind": kind}]
    # no strategic-merge-patch in the PATCH bodies: kubectl keeps its compiled-in merge keys
    _, _, apps = _abs(kube, root["paths"]["apis/apps/v1"]["serverRelativeURL"])
    patch = apps["paths"]["/apis/apps/v1/namespaces/{namespace}/deployments/{name}"]["patch"]
    assert k8s_wire.STRATEGIC_PATCH not in patch["requestBody"]["content"] and APPLY in patch["requestBody"]["content"]
    # the bare API (no project prefix) points at bare URLs
    st, _, bare = _abs(kube, "/openapi/v3")
    assert st == 200 and bare["paths"]["api/v1"]["serverRelativeURL"].startswith("/openapi/v3/api/v1?hash=")
    assert _raw(kube, "GET", "/openapi/v3/apis/nope/v9")[0] == 404


def test_field_validation_strict_warn_ignore(kube):
    bad = json.loads(json.dumps(DEPLOY))
    bad["specc"] = {}
    bad["metadata"]["labelz"] = {"a": "b"}
    st, _, body = _raw(kube, "POST", DPATH + "?fieldValidation=Strict", bad)
    assert st == 400 and 'unknown field "specc"' in body["message"] and "metadata.labelz" in body["message"], body
    conn = http.client.HTTPConnection(kube.host, kube.port, timeout=10)
    conn.request("POST", kube.k8s(DPATH + "?fieldValidation=Warn"), body=json.dumps(bad).encode(),
                 headers={"Content-Type": "application/json", "Authorization": f"Bearer {kube.token}"})
    r = conn.getresponse()
    r.read()
    assert r.status == 201 and 'unknown field \\"specc\\"' not in (r.getheader("Warning") or "x")
    assert "specc" in r.getheader("Warning"), r.getheaders()
    conn.close()
    # a well-formed object passes Strict
    good = json.loads(json.dumps(DEPLOY))
    good["metadata"]["name"] = "web2"
    assert _raw(kube, "POST", DPATH + "?fieldValidation=Strict", good)[0] == 201


def test_dry_run_writes_nothing(kube):
    st, _, d = _raw(kube, "POST", DPATH + "?dryRun=All", DEPLOY)
    assert st == 201 and d["metadata"]["name"] == "web"
    assert _raw(kube, "GET", DPATH + "/web")[0] == 404
    assert _raw(kube, "POST", DPATH, DEPLOY)[0] == 201
    st, _, d = _raw(kube, "PATCH", DPATH + "/web?dryRun=All", {"spec": {"replicas": 7}}, ctype=k8s_wire.MERGE_PATCH)
    assert st == 200 and d["spec"]["replicas"] == 7
    assert _raw(kube, "GET", DPATH + "/web")[2]["spec"]["replicas"] == 1
    assert _raw(kube, "DELETE", DPATH + "/web?dryRun=All")[0] == 200
    assert _raw(kube, "GET", DPATH + "/web")[0] == 200
    assert _raw(kube, "POST", DPATH + "?dryRun=Some", DEPLOY)[0] == 400


def _apply(k, obj, manager="kubectl", force=False, name="web", raw_body=None):
    q = f"?fieldManager={manager}" + ("&force=true" if force else "")
    if raw_body is not None:
        conn = http.client.HTTPConnection(k.host, k.port, timeout=10)
        conn.request("PATCH", k.k8s(f"{DPATH}/{name}{q}"), body=raw_body.encode(),
                     headers={"Content-Type": APPLY, "Authorization": f"Bearer {k.token}"})
        r = conn.getresponse()
        out = r.status, json.loads(r.read())
        conn.close()
        return out
    st, _, body = _raw(k, "PATCH", f"{DPATH}/{name}{q}", obj, ctype=APPLY)
    return st, body


def _owners(obj: dict) -> dict[str, set]:
    return {f'{e["manager"]}/{e["operation"]}' + (f'/{e["subresource"]}' if e.get("subresource") else ""):
            {ssa.dotted(p) for p in ssa.from_fieldsv1(e["fieldsV1"])} for e in obj["metadata"].get("managedFields", [])}


def test_server_side_apply(kube):
    cfg = json.loads(json.dumps(DEPLOY))
    cfg["metadata"]["labels"] = {"app": "web", "tier": "front"}
    st, d = _apply(kube, cfg)
    assert st == 201, d
    own = _owners(d)
    assert ".spec.replicas" in own["kubectl/Apply"] and ".metadata.labels.tier" in own["kubectl/Apply"]
    assert '.spec.template.spec.containers[{"name":"a"}].env[{"name":"Y"}].value' in own["kubectl/Apply"]
    # another manager setting the same field to another value: a conflict naming the owner
    st, body = _apply(kube, {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": "web"},
                             "spec": {"replicas": 3}}, manager="hpa")
    assert st == 409 and body["reason"] == "Conflict", body
    assert body["details"]["causes"] == [{"type": "FieldManagerConflict", "message": 'conflict with "kubectl" using apps/v1',
                                         "field": ".spec.replicas"}]
    # ... the same value: shared ownership, no conflict
    st, d = _apply(kube, {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": "web"},
                          "spec": {"replicas": 1}}, manager="hpa")
    assert st == 200 and ".spec.replicas" in _owners(d)["hpa/Apply"] and ".spec.replicas" in _owners(d)["kubectl/Apply"]
    # force takes it over
    st, d = _apply(kube, {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": "web"},
                          "spec": {"replicas": 4}}, manager="hpa", force=True)
    assert st == 200 and d["spec"]["replicas"] == 4 and ".spec.replicas" not in _owners(d)["kubectl/Apply"]
    # kubectl re-applies without replicas, env Y and label tier: its fields go, hpa's stay
    cfg2 = json.loads(json.dumps(cfg))
    del cfg2["spec"]["replicas"]
    cfg2["metadata"]["labels"] = {"app": "web"}
    cfg2["spec"]["template"]["spec"]["containers"][0]["env"] = [{"name": "X", "value": "1"}]
    st, d = _apply(kube, cfg2)
    assert st == 200, d
    assert d["spec"]["replicas"] == 4 and "tier" not in d["metadata"]["labels"]
    assert d["spec"]["template"]["spec"]["containers"][0]["env"] == [{"name": "X", "value": "1"}]
    live = _raw(kube, "GET", DPATH + "/web")[2]
    assert live["spec"]["template"]["spec"]["containers"][0]["env"] == [{"name": "X", "value": "1"}]
    assert live["metadata"]["generation"] >= 2


def test_apply_conflicts_with_an_update_and_checks_its_request(kube):
    cfg = json.loads(json.dumps(DEPLOY))
    assert _apply(kube, cfg)[0] == 201
    # kubectl scale: an Update through the scale subresource by its own manager
    st, _, _b = _raw(kube, "PATCH", DPATH + "/web/scale?fieldManager=kubectl-scale", {"spec": {"replicas": 5}},
                     ctype=k8s_wire.MERGE_PATCH)
    assert st == 200
    d = _raw(kube, "GET", DPATH + "/web")[2]
    assert _owners(d)["kubectl-scale/Update/scale"] == {".spec.replicas"}
    st, body = _apply(kube, cfg)  # replicas 1 again: conflicts with the scaler
    assert st == 409 and 'conflict with "kubectl-scale"' in body["message"], body
    # a YAML body works as well; requests without fieldManager or for another name do not
    yml = "apiVersion: apps/v1\nkind: Deployment\nmetadata:\n  name: web\nspec:\n  paused: true\n"
    st, d = _apply(kube, None, manager="yaml-user", raw_body=yml)
    assert st == 200 and d["spec"]["paused"] is True
    assert _raw(kube, "PATCH", DPATH + "/web", cfg, ctype=APPLY)[0] == 400
    assert _apply(kube, cfg, name="other")[0] == 400
    wrong = dict(cfg, kind="Job")
    assert _apply(kube, wrong)[0] == 400
    # clients cannot rewrite managedFields through a plain update
    d = _raw(kube, "GET", DPATH + "/web")[2]
    d["metadata"]["managedFields"] = []
    st, _, out = _raw(kube, "PUT", DPATH + "/web", d)
    assert st == 200 and "kubectl-scale/Update/scale" in _owners(out)


def test_managed_field_paths_unit():
    obj = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "p", "labels": {"a": "1"}},
           "spec": {"containers": [{"name": "c", "image": "i", "args": ["x", "y"],
                                   "ports": [{"containerPort": 80}]}]}, "status": {"phase": "Running"}}
    paths = ssa.field_paths(obj)
    assert ("f:metadata", "f:labels", "f:a") in paths
    assert ("f:spec", "f:containers", 'k:{"name":"c"}', ".") in paths
    assert ("f:spec", "f:containers", 'k:{"name":"c"}', "f:args") in paths  # atomic list: one leaf
    assert ("f:spec", "f:containers", 'k:{"name":"c"}', "f:ports", 'k:{"containerPort":80}', "f:containerPort") in paths
    assert not any(p[0] in ("f:status", "f:apiVersion") for p in paths)
    assert ssa.from_fieldsv1(ssa.to_fieldsv1(paths)) == paths
    assert ssa.get(obj, ("f:spec", "f:containers", 'k:{"name":"c"}', "f:image")) == "i"
    ssa.remove(obj, ("f:spec", "f:containers", 'k:{"name":"c"}', "."))
    assert obj["spec"]["containers"] == []


@pytest.mark.parametrize("mode,body,bad", [
    ("Strict", {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "x"}, "data": {}, "spec": {}}, ['"spec"']),
    ("Ignore", {"kind": "ConfigMap", "bogus": 1}, []),
    (None, {"kind": "ConfigMap", "bogus": 1}, []),
])
def test_check_fields_unit(mode, body, bad):
    out = k8s_openapi.check_fields("configmaps", body, mode)
    assert all(any(b in o for o in out) for b in bad) and (bool(out) == bool(bad))


def test_bundled_kubectl_server_side_apply(kube, tmp_path, capsys):
    """./kubectl apply --server-side [--force-conflicts] [--dry-run=server]; -o yaml hides managedFields
    unless --show-managed-fields."""
    from tritonk8ssupervisor_amd.cli import kubectl

    pid = kube.prefix.split("/")[3]
    cfg = tmp_path / "kubeconfig.json"
    cfg.write_text(json.dumps(kube.get(f"/env/{pid}/kubernetes/kubectl", query={"format": "json"})))
    man = tmp_path / "web.json"
    man.write_text(json.dumps(DEPLOY))
    kc = lambda *a: kubectl.main(["--kubeconfig", str(cfg), *a], workdir=str(tmp_path))
    assert kc("apply", "--server-side", "--dry-run", "server", "-f", str(man)) == 0
    assert "serverside-applied (server dry run)" in capsys.readouterr().out
    assert _raw(kube, "GET", DPATH + "/web")[0] == 404
    assert kc("apply", "--server-side", "-f", str(man)) == 0
    assert "deployment/web serverside-applied" in capsys.readouterr().out
    other = dict(DEPLOY, spec={**DEPLOY["spec"], "replicas": 2})
    man.write_text(json.dumps(other))
    assert kc("apply", "--server-side", "--field-manager", "ci", "-f", str(man)) == 1
    assert 'conflict with "kubectl"' in capsys.readouterr().err
    assert kc("apply", "--server-side", "--field-manager", "ci", "--force-conflicts", "-f", str(man)) == 0
    capsys.readouterr()
    assert kc("get", "deploy", "web", "-o", "json") == 0
    out = json.loads(capsys.readouterr().out)
    assert out["spec"]["replicas"] == 2 and "managedFields" not in out["metadata"]
    assert kc("get", "deploy", "web", "-o", "json", "--show-managed-fields") == 0
    managers = {e["manager"] for e in json.loads(capsys.readouterr().out)["metadata"]["managedFields"]}
    assert managers == {"kubectl", "ci"}


def test_bundled_kubectl_custom_resources(kube, tmp_path, capsys):
    """./kubectl apply of a CRD and its objects, then get/delete them by plural or short name."""
    from tritonk8ssupervisor_amd.cli import kubectl

    pid = kube.prefix.split("/")[3]
    cfg = tmp_path / "kubeconfig.json"
    cfg.write_text(json.dumps(kube.get(f"/env/{pid}/kubernetes/kubectl", query={"format": "json"})))
    kc = lambda *a: kubectl.main(["--kubeconfig", str(cfg), *a], workdir=str(tmp_path))
    crd = {"apiVersion": "apiextensions.k8s.io/v1", "kind": "CustomResourceDefinition",
           "metadata": {"name": "gpuquotas.tk8s.example.com"},
           "spec": {"group": "tk8s.example.com", "scope": "Namespaced",
                    "names": {"plural": "gpuquotas", "singular": "gpuquota", "kind": "GpuQuota", "shortNames": ["gq"]},
                    "versions": [{"name": "v1alpha1", "served": True, "storage": True}]}}
    (tmp_path / "crd.json").write_text(json.dumps(crd))
    assert kc("apply", "-f", str(tmp_path / "crd.json")) == 0
    (tmp_path / "q.json").write_text(json.dumps({"apiVersion": "tk8s.example.com/v1alpha1", "kind": "GpuQuota",
                                                 "metadata": {"name": "team-a"}, "spec": {"gpus": 4}}))
    assert kc("apply", "-f", str(tmp_path / "q.json")) == 0
    capsys.readouterr()
    assert kc("get", "gq") == 0 and "team-a" in capsys.readouterr().out
    assert kc("get", "gpuquota", "team-a", "-o", "json") == 0
    assert json.loads(capsys.readouterr().out)["spec"]["gpus"] == 4
    assert kc("get", "crds") == 0 and "gpuquotas.tk8s.example.com" in capsys.readouterr().out
    assert kc("delete", "gpuquotas", "team-a") == 0
