"""The control plane speaks the Kubernetes wire conventions a stock client relies on
(controlplane/k8s_wire.py): discovery, typed lists, Status errors, field selectors, the three
patch types, server-side Tables and the chunked watch stream.

No kubectl / client-go / kubernetes Python client is installed here, so these tests play the
client's part at the HTTP level, request by request, the way kubectl issues them (discovery
first, then e.g. GET -> 404 -> POST -> PATCH application/strategic-merge-patch+json for
``kubectl apply``). Parity with a real kubectl binary is unpinned."""
import http.client
import json
import threading
import time

import pytest

from tritonk8ssupervisor_amd.controlplane import k8s_wire
from tritonk8ssupervisor_amd.controlplane.client import client_from_kubeconfig

from test_controlplane import _env, _join, _start, _stop


@pytest.fixture
def kube(tmp_path):
    p, c = _start(tmp_path)
    proj = _env(c)
    _join(c, proj["id"], "kubenode1", ngpu=2)
    k = client_from_kubeconfig(c.get(f"/env/{proj['id']}/kubernetes/kubectl", query={"format": "json"}))
    yield k
    _stop(p)


def _raw(k, method, path, body=None, ctype="application/json", accept="application/json", timeout=10):
    conn = http.client.HTTPConnection(k.host, k.port, timeout=timeout)
    headers = {"Accept": accept, "Authorization": f"Bearer {k.token}"}
    data = None
    if body is not None:
        data = json.dumps(body).encode()
        headers["Content-Type"] = ctype
    conn.request(method, k.k8s(path), body=data, headers=headers)
    r = conn.getresponse()
    out = r.status, r.getheader("Content-Type"), r.read()
    conn.close()
    return out[0], out[1], (json.loads(out[2]) if out[2] and "json" in (out[1] or "") else out[2])


# ---- discovery ------------------------------------------------------------------------------
def test_discovery_documents(kube):
    st, _, v = _raw(kube, "GET", "/api")
    assert st == 200 and v["kind"] == "APIVersions" and v["versions"] == ["v1"]
    _, _, groups = _raw(kube, "GET", "/apis")
    names = {g["name"]: g["preferredVersion"]["groupVersion"] for g in groups["groups"]}
    # every served group, each at its one version (the list grows with the kinds served)
    assert {"apps": "apps/v1", "batch": "batch/v1", "networking.k8s.io": "networking.k8s.io/v1",
            "autoscaling": "autoscaling/v2", "metrics.k8s.io": "metrics.k8s.io/v1beta1",
            "rbac.authorization.k8s.io": "rbac.authorization.k8s.io/v1"}.items() <= names.items()
    assert set(names) == {g for g, _v in k8s_wire._groups()}
    _, _, core = _raw(kube, "GET", "/api/v1")
    res = {r["name"]: r for r in core["resources"]}
    assert core["kind"] == "APIResourceList" and core["groupVersion"] == "v1"
    assert res["pods"]["kind"] == "Pod" and res["pods"]["namespaced"] and "po" in res["pods"]["shortNames"]
    assert not res["nodes"]["namespaced"] and "watch" in res["nodes"]["verbs"] and "pods/log" in res
    _, _, apps = _raw(kube, "GET", "/apis/apps/v1")
    scale = next(r for r in apps["resources"] if r["name"] == "deployments/scale")
    assert scale["kind"] == "Scale" and scale["group"] == "autoscaling"
    assert _raw(kube, "GET", "/apis/nope/v1")[0] == 404
    _, _, grp = _raw(kube, "GET", "/apis/batch")
    assert grp["kind"] == "APIGroup" and grp["preferredVersion"]["version"] == "v1"


# ---- typed objects, lists and Status errors --------------------------------------------------
def test_typed_lists_and_objects(kube):
    cm = {"metadata": {"name": "a"}, "data": {"k": "v"}}
    _raw(kube, "POST", "/api/v1/namespaces/default/configmaps", cm)
    _, _, lst = _raw(kube, "GET", "/api/v1/namespaces/default/configmaps")
    assert lst["kind"] == "ConfigMapList" and lst["apiVersion"] == "v1" and lst["metadata"]["resourceVersion"]
    assert lst["items"][0]["kind"] == "ConfigMap" and lst["items"][0]["apiVersion"] == "v1"
    _, _, nodes = _raw(kube, "GET", "/api/v1/nodes")
    assert nodes["kind"] == "NodeList" and nodes["items"][0]["kind"] == "Node"
    _, _, deps = _raw(kube, "GET", "/apis/apps/v1/deployments")
    assert deps["kind"] == "DeploymentList" and deps["apiVersion"] == "apps/v1"
    _, _, ns = _raw(kube, "GET", "/api/v1/namespaces")
    assert ns["kind"] == "NamespaceList" and all(i["kind"] == "Namespace" for i in ns["items"])


def test_errors_are_kubernetes_status_objects(kube):
    st, _, body = _raw(kube, "GET", "/api/v1/namespaces/default/pods/missing")
    assert st == 404 and body["kind"] == "Status" and body["reason"] == "NotFound" and body["code"] == 404
    cm = {"metadata": {"name": "dup"}, "data": {}}
    _raw(kube, "POST", "/api/v1/namespaces/default/configmaps", cm)
    st, _, body = _raw(kube, "POST", "/api/v1/namespaces/default/configmaps", cm)
    assert st == 409 and body["reason"] == "AlreadyExists"
    stale = dict(cm, metadata={"name": "dup", "resourceVersion": "1"})
    st, _, body = _raw(kube, "PUT", "/api/v1/namespaces/default/configmaps/dup", stale)
    assert st == 409 and body["reason"] == "Conflict"
    st, _, body = _raw(kube, "POST", "/api/v1/namespaces/default/pods", {"metadata": {"name": "x"}, "spec": {}})
    assert st == 422 and body["reason"] == "Invalid"


# ---- selectors and tables -------------------------------------------------------------------
def test_field_selectors(kube):
    for n in ("one", "two"):
        _raw(kube, "POST", "/api/v1/namespaces/default/configmaps", {"metadata": {"name": n}, "data": {}})
    _, _, one = _raw(kube, "GET", "/api/v1/namespaces/default/configmaps?fieldSelector=metadata.name%3Done")
    assert [i["metadata"]["name"] for i in one["items"]] == ["one"]
    _, _, rest = _raw(kube, "GET", "/api/v1/namespaces/default/configmaps?fieldSelector=metadata.name!%3Done")
    assert [i["metadata"]["name"] for i in rest["items"]] == ["two"]
    _, _, nodes = _raw(kube, "GET", "/api/v1/nodes?fieldSelector=metadata.name%3Dkubenode1")
    assert len(nodes["items"]) == 1


def test_server_side_table_for_kubectl_get(kube):
    acc = "application/json;as=Table;v=v1;g=meta.k8s.io,application/json;as=Table;v=v1beta1;g=meta.k8s.io,application/json"
    _, _, t = _raw(kube, "GET", "/api/v1/nodes", accept=acc)
    assert t["kind"] == "Table" and t["apiVersion"] == "meta.k8s.io/v1"
    cols = [c["name"] for c in t["columnDefinitions"]]
    assert cols[:2] == ["Name", "Status"] and "GPU" in cols
    row = t["rows"][0]
    assert row["cells"][0] == "kubenode1" and row["cells"][cols.index("GPU")] == "2/2"
    assert row["object"]["kind"] == "PartialObjectMetadata" and row["object"]["metadata"]["name"] == "kubenode1"
    _, _, t = _raw(kube, "GET", "/api/v1/namespaces", accept=acc)
    assert t["kind"] == "Table" and any(r["cells"][0] == "default" for r in t["rows"])


# ---- patches --------------------------------------------------------------------------------
DEPLOY = {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": "web"},
          "spec": {"replicas": 1, "selector": {"matchLabels": {"app": "web"}},
                   "template": {"metadata": {"labels": {"app": "web"}},
                                "spec": {"containers": [
                                    {"name": "a", "image": "img:1", "command": ["sleep", "60"],
                                     "env": [{"name": "X", "value": "1"}, {"name": "Y", "value": "2"}]},
                                    {"name": "b", "image": "side:1", "command": ["sleep", "60"]}]}}}}


def test_kubectl_apply_flow_with_a_strategic_merge_patch(kube):
    """kubectl apply: GET (404) -> POST with last-applied; change -> PATCH strategic-merge-patch."""
    path = "/apis/apps/v1/namespaces/default/deployments/web"
    assert _raw(kube, "GET", path)[0] == 404
    st, _, created = _raw(kube, "POST", "/apis/apps/v1/namespaces/default/deployments", DEPLOY)
    assert st == 201 and created["kind"] == "Deployment"
    patch = {"metadata": {"annotations": {"kubectl.kubernetes.io/last-applied-configuration": "{}"}},
             "spec": {"template": {"spec": {
                 "$setElementOrder/containers": [{"name": "a"}, {"name": "b"}],
                 "containers": [{"name": "a", "image": "img:2",
                                 "$setElementOrder/env": [{"name": "X"}, {"name": "Y"}],
                                 "env": [{"name": "Y", "value": "3"}]}]}}}}
    st, _, d = _raw(kube, "PATCH", path, patch, ctype=k8s_wire.STRATEGIC_PATCH)
    assert st == 200, d
    a, b = d["spec"]["template"]["spec"]["containers"]
    assert a["image"] == "img:2" and a["command"] == ["sleep", "60"]          # merged by name, not replaced
    assert a["env"] == [{"name": "X", "value": "1"}, {"name": "Y", "value": "3"}]
    assert b == DEPLOY["spec"]["template"]["spec"]["containers"][1]
    assert "$setElementOrder" not in json.dumps(d)  # directives are applied, never stored
    assert d["metadata"]["generation"] == 2
    # $patch: delete removes one element of a merge-keyed list
    st, _, d = _raw(kube, "PATCH", path, {"spec": {"template": {"spec": {"containers": [{"name": "b", "$patch": "delete"}]}}}},
                    ctype=k8s_wire.STRATEGIC_PATCH)
    assert [c["name"] for c in d["spec"]["template"]["spec"]["containers"]] == ["a"]


def test_json_patch_and_merge_patch(kube):
    _raw(kube, "POST", "/apis/apps/v1/namespaces/default/deployments", DEPLOY)
    path = "/apis/apps/v1/namespaces/default/deployments/web"
    st, _, d = _raw(kube, "PATCH", path, [{"op": "replace", "path": "/spec/replicas", "value": 3},
                                          {"op": "add", "path": "/metadata/labels/tier", "value": "front"}],
                    ctype=k8s_wire.JSON_PATCH)
    assert st == 200 and d["spec"]["replicas"] == 3 and d["metadata"]["labels"]["tier"] == "front"
    st, _, body = _raw(kube, "PATCH", path, [{"op": "test", "path": "/spec/replicas", "value": 9}],
                       ctype=k8s_wire.JSON_PATCH)
    assert st == 422 and body["reason"] == "Invalid"
    st, _, d = _raw(kube, "PATCH", path, {"spec": {"replicas": 2}}, ctype=k8s_wire.MERGE_PATCH)
    assert st == 200 and d["spec"]["replicas"] == 2
    # server-side apply needs a field manager (tests/test_k8s_ssa.py covers apply itself)
    assert _raw(kube, "PATCH", path, {"spec": {}}, ctype=k8s_wire.APPLY_PATCH)[0] == 400


def test_strategic_merge_directives_unit():
    cur = {"spec": {"ports": [{"port": 80, "name": "http"}, {"port": 443, "name": "https"}],
                    "finalizers": ["a"], "keep": 1, "drop": 2}}
    out = k8s_wire.strategic_merge(cur, {"spec": {"ports": [{"port": 443, "targetPort": 8443}],
                                                  "finalizers": ["b"], "drop": None}})
    assert out["spec"]["ports"] == [{"port": 80, "name": "http"}, {"port": 443, "name": "https", "targetPort": 8443}]
    assert out["spec"]["finalizers"] == ["a", "b"] and "drop" not in out["spec"]
    assert k8s_wire.strategic_merge(cur, {"spec": {"$patch": "replace", "x": 1}}) == {"spec": {"x": 1}}
    assert k8s_wire.strategic_merge(cur, {"spec": {"$retainKeys": ["keep"], "keep": 5}}) == {"spec": {"keep": 5}}
    out = k8s_wire.strategic_merge(cur, {"spec": {"$deleteFromPrimitiveList/finalizers": ["a"]}})
    assert out["spec"]["finalizers"] == []
    with pytest.raises(k8s_wire.PatchError):
        k8s_wire.json_patch({"a": 1}, [{"op": "remove", "path": "/b"}])
    assert k8s_wire.json_patch({"a": [1, 2]}, [{"op": "add", "path": "/a/-", "value": 3},
                                               {"op": "move", "from": "/a/0", "path": "/b"}]) == {"a": [2, 3], "b": 1}


# ---- watch stream ---------------------------------------------------------------------------
def _stream(k, path, timeout=10):
    conn = http.client.HTTPConnection(k.host, k.port, timeout=timeout)
    conn.request("GET", k.k8s(path), headers={"Accept": "application/json", "Authorization": f"Bearer {k.token}"})
    r = conn.getresponse()
    return conn, r


def test_watch_is_a_chunked_stream_of_events(kube):
    _raw(kube, "POST", "/api/v1/namespaces/default/configmaps", {"metadata": {"name": "before"}, "data": {}})
    conn, r = _stream(kube, "/api/v1/namespaces/default/configmaps?watch=true&timeoutSeconds=3")
    assert r.status == 200 and r.getheader("Transfer-Encoding") == "chunked"
    first = json.loads(r.readline())
    assert first["type"] == "ADDED" and first["object"]["metadata"]["name"] == "before"
    assert first["object"]["kind"] == "ConfigMap"

    def later():
        time.sleep(0.2)
        _raw(kube, "POST", "/api/v1/namespaces/default/configmaps", {"metadata": {"name": "after"}, "data": {}})
        _raw(kube, "DELETE", "/api/v1/namespaces/default/configmaps/before")

    threading.Thread(target=later).start()
    ev = [json.loads(r.readline()) for _ in range(2)]
    assert [(e["type"], e["object"]["metadata"]["name"]) for e in ev] == [("ADDED", "after"), ("DELETED", "before")]
    t = time.monotonic()
    assert r.read() == b""  # the stream ends at timeoutSeconds (chunked terminator)
    assert time.monotonic() - t < 5
    conn.close()


def test_watch_from_a_resource_version_and_with_a_field_selector(kube):
    _, _, cm = _raw(kube, "POST", "/api/v1/namespaces/default/configmaps", {"metadata": {"name": "w"}, "data": {}})
    rv = cm["metadata"]["resourceVersion"]
    _raw(kube, "POST", "/api/v1/namespaces/default/configmaps", {"metadata": {"name": "other"}, "data": {}})
    _raw(kube, "PATCH", "/api/v1/namespaces/default/configmaps/w", {"data": {"k": "v"}}, ctype=k8s_wire.MERGE_PATCH)
    conn, r = _stream(kube, f"/api/v1/namespaces/default/configmaps?watch=true&resourceVersion={rv}"
                            "&fieldSelector=metadata.name%3Dw&timeoutSeconds=1")
    ev = [json.loads(ln) for ln in r.read().splitlines() if ln.strip()]
    assert [(e["type"], e["object"]["data"]) for e in ev] == [("MODIFIED", {"k": "v"})]
    conn.close()
    conn, r = _stream(kube, "/api/v1/namespaces/default/configmaps?watch=true&resourceVersion=abc&timeoutSeconds=1")
    e = json.loads(r.readline())
    assert e["type"] == "ERROR" and e["object"]["code"] == 400
    conn.close()


def test_tk8s_clients_keep_the_batch_long_poll(kube):
    rv = int(kube.get(kube.k8s("/api/v1/namespaces/default/configmaps"))["metadata"]["resourceVersion"])
    threading.Timer(0.2, lambda: _raw(kube, "POST", "/api/v1/namespaces/default/configmaps",
                                      {"metadata": {"name": "lp"}, "data": {}})).start()
    new_rv, events = kube.watch(kube.k8s("/api/v1/namespaces/default/configmaps"), rv, timeout=5)
    assert new_rv > rv and [e["object"]["metadata"]["name"] for e in events] == ["lp"]


def test_json_patch_rejects_out_of_range_and_malformed_indices():
    """RFC 6902 4.1 -- an add index past the end (or negative, or with a leading zero)
    is an error, not an append."""
    with pytest.raises(k8s_wire.PatchError, match="out of bounds"):
        k8s_wire.json_patch({"a": [1]}, [{"op": "add", "path": "/a/5", "value": 2}])
    for bad in ("-1", "01", "x"):
        with pytest.raises(k8s_wire.PatchError, match="invalid array index"):
            k8s_wire.json_patch({"a": [1]}, [{"op": "add", "path": f"/a/{bad}", "value": 2}])
    assert k8s_wire.json_patch({"a": [1]}, [{"op": "add", "path": "/a/1", "value": 2}]) == {"a": [1, 2]}
    assert k8s_wire.json_patch({"a": [1]}, [{"op": "add", "path": "/a/0", "value": 0}]) == {"a": [0, 1]}


def test_scale_subresource_answers_4xx_to_a_non_object_body(kube):
    """a JSON-patch list sent to deployments/scale is applied as a patch (kubectl patch
    --type json), and a body that is not an object is a 422 -- never a 500."""
    _raw(kube, "POST", "/apis/apps/v1/namespaces/default/deployments", DEPLOY)
    path = "/apis/apps/v1/namespaces/default/deployments/web/scale"
    st, _, d = _raw(kube, "PATCH", path, [{"op": "replace", "path": "/spec/replicas", "value": 4}],
                    ctype=k8s_wire.JSON_PATCH)
    assert st == 200 and d["spec"]["replicas"] == 4
    st, _, _ = _raw(kube, "PUT", path, [1, 2, 3])
    assert st == 422


def test_fabric_only_annotations_cannot_be_added_by_update(kube):
    """the gpu-visibility / gpu-scope admission holds for PUT, merge, JSON and strategic
    patches, not only for create -- and a client cannot write the scheduler's host claims."""
    pod = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "sneaky", "namespace": "kube-system",
                                                          "ownerReferences": [{"kind": "Job", "name": "x", "uid": "1"}]},
           "spec": {"containers": [{"name": "c", "command": ["sleep", "1"]}]}}
    st, _, _ = _raw(kube, "POST", "/api/v1/namespaces/kube-system/pods", pod)
    assert st == 201
    path = "/api/v1/namespaces/kube-system/pods/sneaky"
    for body, ctype in (({"metadata": {"annotations": {"tk8s.amd.com/gpu-visibility": "node"}}}, k8s_wire.MERGE_PATCH),
                        ({"metadata": {"annotations": {"tk8s.amd.com/gpu-scope": "host"}}}, k8s_wire.STRATEGIC_PATCH),
                        ([{"op": "add", "path": "/metadata/annotations/tk8s.amd.com~1gpu-visibility", "value": "node"}],
                         k8s_wire.JSON_PATCH),
                        ({"metadata": {"annotations": {"tk8s.amd.com/host-claims": "{}"}}}, k8s_wire.MERGE_PATCH)):
        st, _, err = _raw(kube, "PATCH", path, body, ctype=ctype)
        assert st == 403, (body, st, err)
    st, _, cur = _raw(kube, "GET", path)
    cur["metadata"]["annotations"]["tk8s.amd.com/gpu-visibility"] = "node"
    assert _raw(kube, "PUT", path, cur)[0] == 403
    # a DaemonSet / Deployment may not carry them in its template, whatever the verb
    st, _, _ = _raw(kube, "POST", "/apis/apps/v1/namespaces/default/deployments", DEPLOY)
    st, _, d = _raw(kube, "PATCH", "/apis/apps/v1/namespaces/default/deployments/web",
                    {"spec": {"template": {"metadata": {"annotations": {"tk8s.amd.com/gpu-scope": "host"}}}}},
                    ctype=k8s_wire.MERGE_PATCH)
    assert st == 403


def test_events_select_by_uid_as_kubectl_describe_does(kube):
    pod = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "ev"},
           "spec": {"containers": [{"name": "c", "image": "x", "command": ["true"]}]}}
    st, _, p = _raw(kube, "POST", "/api/v1/namespaces/default/pods", pod)
    assert st == 201
    sel = f"involvedObject.kind=Pod,involvedObject.name=ev,involvedObject.namespace=default,involvedObject.uid={p['metadata']['uid']}"
    _, _, evs = _raw(kube, "GET", "/api/v1/namespaces/default/events?fieldSelector=" + sel.replace(",", "%2C"))
    assert any(e["reason"] == "Scheduled" for e in evs["items"]), evs
    e = evs["items"][0]
    assert e["involvedObject"]["apiVersion"] == "v1" and e["lastTimestamp"] and e["source"]["component"]


def test_namespaces_create_get_label_and_cascade_delete(kube):
    st, _, ns = _raw(kube, "POST", "/api/v1/namespaces", {"apiVersion": "v1", "kind": "Namespace",
                                                          "metadata": {"name": "team-a"}})
    assert st == 201 and ns["metadata"]["labels"]["kubernetes.io/metadata.name"] == "team-a"
    assert _raw(kube, "POST", "/api/v1/namespaces", {"metadata": {"name": "team-a"}})[0] == 409
    assert _raw(kube, "POST", "/api/v1/namespaces", {"metadata": {"name": "Bad_Name"}})[0] == 422
    assert _raw(kube, "GET", "/api/v1/namespaces/team-a")[0] == 200
    assert _raw(kube, "GET", "/api/v1/namespaces/kube-system")[0] == 200  # built in
    assert _raw(kube, "GET", "/api/v1/namespaces/nope")[0] == 404
    st, _, ns = _raw(kube, "PATCH", "/api/v1/namespaces/team-a", {"metadata": {"labels": {"tier": "gpu"}}},
                     ctype=k8s_wire.MERGE_PATCH)
    assert st == 200 and ns["metadata"]["labels"]["tier"] == "gpu"
    cm = {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "c"}, "data": {"a": "1"}}
    assert _raw(kube, "POST", "/api/v1/namespaces/team-a/configmaps", cm)[0] == 201
    names = [n["metadata"]["name"] for n in _raw(kube, "GET", "/api/v1/namespaces")[2]["items"]]
    assert "team-a" in names and "default" in names
    st, _, gone = _raw(kube, "DELETE", "/api/v1/namespaces/team-a")
    assert st == 200 and gone["status"]["phase"] == "Terminating"
    assert _raw(kube, "GET", "/api/v1/namespaces/team-a/configmaps/c")[0] == 404  # its objects went with it
    assert _raw(kube, "GET", "/api/v1/namespaces/team-a")[0] == 404
    assert _raw(kube, "DELETE", "/api/v1/namespaces/default")[0] == 403


def test_service_accounts_and_rbac(kube):
    import base64

    def as_(tok, method, path, body=None):
        conn = http.client.HTTPConnection(kube.host, kube.port, timeout=10)
        headers = {"Content-Type": "application/json", **({"Authorization": f"Bearer {tok}"} if tok else {})}
        conn.request(method, kube.k8s(path), body=json.dumps(body).encode() if body is not None else None, headers=headers)
        r = conn.getresponse()
        out = r.status, r.read()
        conn.close()
        return out[0], json.loads(out[1]) if out[1] else None

    assert _raw(kube, "POST", "/api/v1/namespaces/default/serviceaccounts", {"metadata": {"name": "bot"}})[0] == 201
    sa = _raw(kube, "GET", "/api/v1/namespaces/default/serviceaccounts/bot")[2]
    assert sa["secrets"] == [{"name": "bot-token"}]
    assert _raw(kube, "GET", "/api/v1/namespaces/default/serviceaccounts/default")[0] == 200  # every namespace has one
    sec = _raw(kube, "GET", "/api/v1/namespaces/default/secrets/bot-token")[2]
    assert sec["type"] == "kubernetes.io/service-account-token"
    tok = base64.b64decode(sec["data"]["token"]).decode()
    st, body = as_(tok, "GET", "/api/v1/namespaces/default/pods")
    assert st == 403 and 'User "system:serviceaccount:default:bot" cannot list resource "pods"' in body["message"]
    assert as_(tok, "GET", "/apis/apps/v1")[0] == 200  # discovery is open
    # view in its namespace: read workloads, not secrets, no writes
    assert _raw(kube, "POST", "/apis/rbac.authorization.k8s.io/v1/namespaces/default/rolebindings", {
        "metadata": {"name": "bot-view"}, "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole",
                                                     "name": "view"},
        "subjects": [{"kind": "ServiceAccount", "name": "bot", "namespace": "default"}]})[0] == 201
    assert as_(tok, "GET", "/api/v1/namespaces/default/pods")[0] == 200
    assert as_(tok, "GET", "/api/v1/namespaces/kube-system/pods")[0] == 403  # a RoleBinding is namespaced
    assert as_(tok, "GET", "/api/v1/namespaces/default/secrets")[0] == 403
    cm = {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "bot-cm"}, "data": {}}
    assert as_(tok, "POST", "/api/v1/namespaces/default/configmaps", cm)[0] == 403
    # a Role with a resourceName, then edit cluster-wide
    assert _raw(kube, "POST", "/apis/rbac.authorization.k8s.io/v1/namespaces/default/roles", {
        "metadata": {"name": "one-secret"}, "rules": [{"apiGroups": [""], "resources": ["secrets"], "verbs": ["get"],
                                                      "resourceNames": ["bot-token"]}]})[0] == 201
    assert _raw(kube, "POST", "/apis/rbac.authorization.k8s.io/v1/namespaces/default/rolebindings", {
        "metadata": {"name": "bot-secret"}, "roleRef": {"kind": "Role", "name": "one-secret"},
        "subjects": [{"kind": "ServiceAccount", "name": "bot", "namespace": "default"}]})[0] == 201
    assert as_(tok, "GET", "/api/v1/namespaces/default/secrets/bot-token")[0] == 200
    assert as_(tok, "GET", "/api/v1/namespaces/default/secrets/default-token")[0] == 403
    st, _ = _raw(kube, "POST", "/apis/rbac.authorization.k8s.io/v1/clusterrolebindings", {
        "metadata": {"name": "bot-edit"}, "roleRef": {"kind": "ClusterRole", "name": "edit"},
        "subjects": [{"kind": "ServiceAccount", "name": "bot", "namespace": "default"}]})[:2]
    assert st == 201
    assert as_(tok, "POST", "/api/v1/namespaces/default/configmaps", cm)[0] == 201
    assert as_(tok, "GET", "/api/v1/namespaces/kube-system/pods")[0] == 200
    assert as_(tok, "POST", "/apis/rbac.authorization.k8s.io/v1/clusterrolebindings", {"metadata": {"name": "x"}})[0] == 403
    names = [o["metadata"]["name"] for o in _raw(kube, "GET", "/apis/rbac.authorization.k8s.io/v1/clusterroles")[2]["items"]]
    assert {"cluster-admin", "admin", "edit", "view"} <= set(names)
    # anonymous: discovery only (controlplane/authn.py) -- no object, log or write
    assert as_(None, "GET", "/api/v1")[0] == 200
    for path in ("/api/v1/namespaces/default/pods", "/api/v1/namespaces/default/configmaps",
                 "/api/v1/namespaces/default/secrets", "/api/v1/nodes"):
        assert as_(None, "GET", path)[0] == 401, path
    assert as_(None, "POST", "/api/v1/namespaces/default/configmaps", cm)[0] == 401


def test_self_subject_access_review(kube):
    """kubectl auth can-i: the admin may, a fresh ServiceAccount may not until bound."""
    import base64

    def review(tok, verb, resource, ns="default"):
        conn = http.client.HTTPConnection(kube.host, kube.port, timeout=10)
        conn.request("POST", kube.k8s("/apis/authorization.k8s.io/v1/selfsubjectaccessreviews"), body=json.dumps({
            "apiVersion": "authorization.k8s.io/v1", "kind": "SelfSubjectAccessReview",
            "spec": {"resourceAttributes": {"namespace": ns, "verb": verb, "resource": resource}}}).encode(),
            headers={"Content-Type": "application/json", "Authorization": f"Bearer {tok}"})
        r = conn.getresponse()
        out = json.loads(r.read())
        conn.close()
        return out["status"]["allowed"]

    assert review(kube.token, "delete", "nodes")
    _raw(kube, "POST", "/api/v1/namespaces/default/serviceaccounts", {"metadata": {"name": "asker"}})
    tok = base64.b64decode(_raw(kube, "GET", "/api/v1/namespaces/default/secrets/asker-token")[2]["data"]["token"]).decode()
    assert not review(tok, "list", "pods")
    _raw(kube, "POST", "/apis/rbac.authorization.k8s.io/v1/namespaces/default/rolebindings", {
        "metadata": {"name": "asker"}, "roleRef": {"kind": "ClusterRole", "name": "view"},
        "subjects": [{"kind": "ServiceAccount", "name": "asker", "namespace": "default"}]})
    assert review(tok, "list", "pods") and not review(tok, "create", "pods") and not review(tok, "list", "pods", "other")


def test_custom_resource_definitions(kube):
    crd = {"apiVersion": "apiextensions.k8s.io/v1", "kind": "CustomResourceDefinition",
           "metadata": {"name": "trainingjobs.mi355x.example.com"},
           "spec": {"group": "mi355x.example.com", "scope": "Namespaced",
                    "names": {"plural": "trainingjobs", "singular": "trainingjob", "kind": "TrainingJob",
                              "shortNames": ["tj"]},
                    "versions": [{"name": "v1", "served": True, "storage": True, "subresources": {"status": {}},
                                  "schema": {"openAPIV3Schema": {"type": "object", "x-kubernetes-preserve-unknown-fields": True}}}]}}
    bad = json.loads(json.dumps(crd))
    bad["metadata"]["name"] = "wrong"
    assert _raw(kube, "POST", "/apis/apiextensions.k8s.io/v1/customresourcedefinitions", bad)[0] == 422
    st, _, c = _raw(kube, "POST", "/apis/apiextensions.k8s.io/v1/customresourcedefinitions", crd)
    assert st == 201 and {x["type"] for x in c["status"]["conditions"]} == {"NamesAccepted", "Established"}
    groups = {g["name"] for g in _raw(kube, "GET", "/apis")[2]["groups"]}
    assert "mi355x.example.com" in groups
    res = _raw(kube, "GET", "/apis/mi355x.example.com/v1")[2]["resources"]
    assert {r["name"] for r in res} == {"trainingjobs", "trainingjobs/status"} and res[0]["shortNames"] == ["tj"]
    base = "/apis/mi355x.example.com/v1/namespaces/default/trainingjobs"
    tj = {"apiVersion": "mi355x.example.com/v1", "kind": "TrainingJob", "metadata": {"name": "llama"},
          "spec": {"gpus": 8, "model": "llama"}}
    st, _, o = _raw(kube, "POST", base, tj)
    assert st == 201 and o["kind"] == "TrainingJob" and o["metadata"]["uid"]
    assert _raw(kube, "GET", base + "/llama")[2]["spec"]["gpus"] == 8
    lst = _raw(kube, "GET", base)[2]
    assert lst["kind"] == "TrainingJobList" and lst["apiVersion"] == "mi355x.example.com/v1" and len(lst["items"]) == 1
    assert len(_raw(kube, "GET", "/apis/mi355x.example.com/v1/trainingjobs")[2]["items"]) == 1  # all namespaces
    st, _, o = _raw(kube, "PATCH", base + "/llama", {"spec": {"gpus": 16}}, ctype=k8s_wire.MERGE_PATCH)
    assert st == 200 and o["spec"]["gpus"] == 16
    st, _, o = _raw(kube, "PUT", base + "/llama/status", {"status": {"phase": "Running"}})
    assert st == 200 and o["status"] == {"phase": "Running"} and o["spec"]["gpus"] == 16
    st, _, o = _raw(kube, "PATCH", base + "/llama?fieldManager=op", {"apiVersion": "mi355x.example.com/v1",
                    "kind": "TrainingJob", "metadata": {"name": "llama"}, "spec": {"priority": 1}},
                    ctype=k8s_wire.APPLY_PATCH)
    assert st == 200 and o["spec"]["priority"] == 1  # server-side apply works on custom resources too
    assert _raw(kube, "GET", "/apis/mi355x.example.com/v2/namespaces/default/trainingjobs")[0] == 404
    assert _raw(kube, "GET", "/apis/nope.example.com/v1/namespaces/default/things")[0] == 404
    # deleting the CRD deletes its objects and its API
    assert _raw(kube, "DELETE", "/apis/apiextensions.k8s.io/v1/customresourcedefinitions/trainingjobs.mi355x.example.com")[0] == 200
    assert _raw(kube, "GET", base)[0] == 404
    _raw(kube, "POST", "/apis/apiextensions.k8s.io/v1/customresourcedefinitions", crd)
    assert _raw(kube, "GET", base)[2]["items"] == []


def test_eviction_api_and_kubectl_drain_wait(kube, tmp_path, capsys):
    """POST pods/<name>/eviction answers 429 while a PodDisruptionBudget allows no disruption;
    ./kubectl drain evicts through it and retries; ./kubectl wait --for=condition/delete/jsonpath."""
    from tritonk8ssupervisor_amd.cli import kubectl
    from test_controlplane import Client

    pid = kube.prefix.split("/")[3]
    cfg = tmp_path / "kubeconfig.json"
    cfg.write_text(json.dumps(kube.get(f"/env/{pid}/kubernetes/kubectl", query={"format": "json"})))
    kc = lambda *a: kubectl.main(["--kubeconfig", str(cfg), *a], workdir=str(tmp_path))
    # the fixture's node, and its node token to post pod status as its agent would
    ctl = Client(kube.base, token=kube.token)
    from test_controlplane import _join

    nc, _reg = _join(ctl, pid, "kubenode2", ngpu=0)
    for i in range(2):
        kube.post(kube.k8s("/api/v1/namespaces/default/pods"), {"metadata": {"name": f"p{i}", "labels": {"app": "x"}},
                                                                 "spec": {"nodeName": "kubenode2", "containers": [
                                                                     {"name": "c", "command": ["sleep", "60"]}]}})
        nc.put(nc.k8s(f"/api/v1/namespaces/default/pods/p{i}/status"), {"status": {"phase": "Running"}})
    assert kc("wait", "pod/p0", "pod/p1", "--for=condition=Ready", "--timeout=5s") == 0
    assert "pod/p0 condition met" in capsys.readouterr().out
    assert kc("wait", "pod", "-l", "app=x", "--for=jsonpath={.status.phase}=Running", "--timeout=5s") == 0
    assert kc("wait", "pod/p0", "--for=jsonpath={.status.phase}=Failed", "--timeout=0.5s") == 1
    assert "timed out waiting" in capsys.readouterr().err
    kube.post(kube.k8s("/apis/policy/v1/namespaces/default/poddisruptionbudgets"), {
        "apiVersion": "policy/v1", "kind": "PodDisruptionBudget", "metadata": {"name": "x"},
        "spec": {"minAvailable": 2, "selector": {"matchLabels": {"app": "x"}}}})
    code, _ct, body = _raw(kube, "POST", "/api/v1/namespaces/default/pods/p0/eviction",
                           {"apiVersion": "policy/v1", "kind": "Eviction", "metadata": {"name": "p0"}})
    assert code == 429 and body["reason"] == "TooManyRequests"
    assert kc("drain", "kubenode2", "--ignore-daemonsets", "--timeout=2s") == 1
    err = capsys.readouterr().err
    assert "disruption budget" in err and "global timeout" in err
    assert kube.get(kube.k8s("/api/v1/nodes/kubenode2"))["spec"]["unschedulable"] is True
    # relax the budget: the drain goes through
    kube.request("PATCH", kube.k8s("/apis/policy/v1/namespaces/default/poddisruptionbudgets/x"),
                 body={"spec": {"minAvailable": 0}}, content_type="application/merge-patch+json")
    assert kc("drain", "kubenode2", "--timeout=5s") == 0
    out = capsys.readouterr().out
    assert "evicting pod default/p0" in out and "node/kubenode2 drained" in out
    assert kc("wait", "pod/p0", "--for=delete", "--timeout=5s") == 0
    assert "pod/p0 deleted" in capsys.readouterr().out
    assert kc("get", "pdb") == 0
    out = capsys.readouterr().out
    assert "ALLOWED DISRUPTIONS" in out and out.splitlines()[1].split()[:3] == ["x", "0", "N/A"]


def test_finalizers_and_propagation_policies(kube):
    """DELETE of an object with finalizers only marks it (deletionTimestamp); removing the last
    finalizer completes the deletion; propagationPolicy=Orphan keeps what the owner owned."""
    cm = "/api/v1/namespaces/default/configmaps"
    code, _, _ = _raw(kube, "POST", cm, {"apiVersion": "v1", "kind": "ConfigMap",
                                         "metadata": {"name": "held", "finalizers": ["example.com/cleanup"]}, "data": {}})
    assert code == 201
    code, _, body = _raw(kube, "DELETE", cm + "/held")
    assert code == 200 and body["metadata"]["deletionTimestamp"] and body["kind"] == "ConfigMap"
    assert _raw(kube, "GET", cm + "/held")[0] == 200  # still there, being deleted
    code, _, body = _raw(kube, "PATCH", cm + "/held", {"metadata": {"finalizers": ["example.com/cleanup", "more"]}},
                         ctype="application/merge-patch+json")
    assert code == 422 and "no new finalizers" in body["message"]
    code, _, body = _raw(kube, "PATCH", cm + "/held", {"metadata": {"labels": {"x": "y"}, "deletionTimestamp": None}},
                         ctype="application/merge-patch+json")
    assert code == 200 and body["metadata"]["deletionTimestamp"]  # a client cannot undo the deletion
    code, _, _ = _raw(kube, "PATCH", cm + "/held", {"metadata": {"finalizers": None}}, ctype="application/merge-patch+json")
    assert code == 200 and _raw(kube, "GET", cm + "/held")[0] == 404
    # Orphan: the Deployment goes, its pods stay without the ownerReference
    dep = "/apis/apps/v1/namespaces/default/deployments"
    assert _raw(kube, "POST", dep, DEPLOY)[0] == 201
    pods = _raw(kube, "GET", "/api/v1/namespaces/default/pods", None)[2]["items"]
    mine = [p["metadata"]["name"] for p in pods if any(r.get("kind") == "Deployment" for r in p["metadata"].get("ownerReferences", []))]
    assert mine
    code, _, _ = _raw(kube, "DELETE", dep + "/web?propagationPolicy=Orphan")
    assert code == 200
    left = {p["metadata"]["name"]: p for p in _raw(kube, "GET", "/api/v1/namespaces/default/pods")[2]["items"]}
    assert set(mine) <= set(left) and all(not left[n]["metadata"].get("ownerReferences") for n in mine)
    assert _raw(kube, "DELETE", dep + "/web?propagationPolicy=Sideways")[0] in (400, 404)


def test_admission_webhooks(kube):
    """A mutating webhook's JSONPatch lands on the object, a validating webhook's denial refuses
    the request; failurePolicy decides about an unreachable webhook (webhooks.py)."""
    import base64
    from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

    seen = []

    class Hook(BaseHTTPRequestHandler):
        def log_message(self, *a):
            pass

        def do_POST(self):
            review = json.loads(self.rfile.read(int(self.headers["Content-Length"])))
            req = review["request"]
            seen.append((self.path, req["operation"], req["kind"]["kind"], req["userInfo"]["username"]))
            resp = {"uid": req["uid"], "allowed": True}
            if self.path == "/mutate":
                patch = [{"op": "add", "path": "/metadata/labels/injected", "value": "yes"}]
                resp.update(patchType="JSONPatch", patch=base64.b64encode(json.dumps(patch).encode()).decode())
            elif self.path == "/validate" and "forbidden" in ((req.get("object") or {}).get("data") or {}):
                resp.update(allowed=False, status={"code": 422, "message": "key 'forbidden' is not allowed"})
            out = json.dumps({"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview", "response": resp}).encode()
            self.send_response(200)
            self.send_header("Content-Type", "application/json")
            self.send_header("Content-Length", str(len(out)))
            self.end_headers()
            self.wfile.write(out)

    srv = ThreadingHTTPServer(("127.0.0.1", 0), Hook)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    base = f"http://127.0.0.1:{srv.server_address[1]}"
    try:
        rule = lambda res, ops=("CREATE", "UPDATE"): {"operations": list(ops), "apiGroups": [""], "apiVersions": ["v1"],
                                                      "resources": [res]}
        assert _raw(kube, "POST", "/apis/admissionregistration.k8s.io/v1/mutatingwebhookconfigurations", {
            "apiVersion": "admissionregistration.k8s.io/v1", "kind": "MutatingWebhookConfiguration",
            "metadata": {"name": "inject"}, "webhooks": [{
                "name": "inject.example.com", "clientConfig": {"url": base + "/mutate"}, "rules": [rule("configmaps")],
                "objectSelector": {"matchExpressions": [{"key": "skip", "operator": "DoesNotExist"}]},
                "sideEffects": "None", "admissionReviewVersions": ["v1"]}]})[0] == 201
        assert _raw(kube, "POST", "/apis/admissionregistration.k8s.io/v1/validatingwebhookconfigurations", {
            "apiVersion": "admissionregistration.k8s.io/v1", "kind": "ValidatingWebhookConfiguration",
            "metadata": {"name": "policy"}, "webhooks": [{
                "name": "policy.example.com", "clientConfig": {"url": base + "/validate"},
                "rules": [rule("configmaps", ("CREATE", "UPDATE", "DELETE"))], "sideEffects": "None",
                "admissionReviewVersions": ["v1"]},
                {"name": "gone.example.com", "clientConfig": {"url": "http://127.0.0.1:9/x"}, "failurePolicy": "Ignore",
                 "rules": [rule("configmaps")], "sideEffects": "None", "admissionReviewVersions": ["v1"]}]})[0] == 201
        cm = "/api/v1/namespaces/default/configmaps"
        code, _, body = _raw(kube, "POST", cm, {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "a"},
                                                "data": {"k": "v"}})
        assert code == 201 and body["metadata"]["labels"]["injected"] == "yes", body
        code, _, body = _raw(kube, "POST", cm, {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "b"},
                                                "data": {"forbidden": "1"}})
        assert code == 422 and 'admission webhook "policy.example.com" denied the request' in body["message"]
        assert _raw(kube, "GET", cm + "/b")[0] == 404
        code, _, body = _raw(kube, "POST", cm, {"apiVersion": "v1", "kind": "ConfigMap",
                                                "metadata": {"name": "c", "labels": {"skip": "1"}}, "data": {}})
        assert code == 201 and "injected" not in body["metadata"]["labels"]  # objectSelector
        code, _, body = _raw(kube, "PATCH", cm + "/a", {"data": {"forbidden": "x"}}, ctype="application/merge-patch+json")
        assert code == 422
        assert _raw(kube, "DELETE", cm + "/a")[0] == 200
        ops = [(p, op) for p, op, kind, _u in seen if kind == "ConfigMap"]
        assert ("/mutate", "CREATE") in ops and ("/validate", "UPDATE") in ops and ("/validate", "DELETE") in ops
        assert all(u == "tk8s:admin" for *_x, u in seen)
        # a webhook that cannot be reached, failurePolicy Fail (the default): the request fails
        assert _raw(kube, "POST", "/apis/admissionregistration.k8s.io/v1/validatingwebhookconfigurations", {
            "apiVersion": "admissionregistration.k8s.io/v1", "kind": "ValidatingWebhookConfiguration",
            "metadata": {"name": "strict"}, "webhooks": [{
                "name": "strict.example.com", "clientConfig": {"url": "http://127.0.0.1:9/x"}, "timeoutSeconds": 2,
                "rules": [rule("secrets")], "sideEffects": "None", "admissionReviewVersions": ["v1"]}]})[0] == 201
        code, _, body = _raw(kube, "POST", "/api/v1/namespaces/default/secrets", {
            "apiVersion": "v1", "kind": "Secret", "metadata": {"name": "s"}, "data": {}})
        assert code == 500 and "failed calling webhook" in body["message"]
        _https_webhook(kube, Hook, seen, rule)
    finally:
        srv.shutdown()


def _https_webhook(kube, handler, seen, rule):
    """The same webhook over HTTPS, verified against the configuration's caBundle."""
    import base64
    import shutil
    import ssl
    import subprocess
    import tempfile
    from http.server import ThreadingHTTPServer

    if not shutil.which("openssl"):
        return
    d = tempfile.mkdtemp()
    subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", f"{d}/k.pem", "-out",
                    f"{d}/c.pem", "-days", "1", "-subj", "/CN=127.0.0.1", "-addext", "subjectAltName=IP:127.0.0.1"],
                   check=True, capture_output=True)
    srv = ThreadingHTTPServer(("127.0.0.1", 0), handler)
    ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
    ctx.load_cert_chain(f"{d}/c.pem", f"{d}/k.pem")
    srv.socket = ctx.wrap_socket(srv.socket, server_side=True)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    try:
        ca = base64.b64encode(open(f"{d}/c.pem", "rb").read()).decode()
        assert _raw(kube, "POST", "/apis/admissionregistration.k8s.io/v1/validatingwebhookconfigurations", {
            "apiVersion": "admissionregistration.k8s.io/v1", "kind": "ValidatingWebhookConfiguration",
            "metadata": {"name": "tls"}, "webhooks": [{
                "name": "tls.example.com", "clientConfig": {"url": f"https://127.0.0.1:{srv.server_address[1]}/tls",
                                                            "caBundle": ca},
                "rules": [rule("serviceaccounts")], "sideEffects": "None", "admissionReviewVersions": ["v1"]}]})[0] == 201
        code, _, body = _raw(kube, "POST", "/api/v1/namespaces/default/serviceaccounts", {
            "apiVersion": "v1", "kind": "ServiceAccount", "metadata": {"name": "robot"}})
        assert code == 201, body
        assert any(p == "/tls" and k == "ServiceAccount" for p, _op, k, _u in seen)
    finally:
        srv.shutdown()


def test_pod_security_admission(kube):
    """Namespace labels pick the Pod Security Standard: enforce refuses, warn answers with a
    Warning header (podsecurity.py)."""
    for ns, labels in (("tenant", {"pod-security.kubernetes.io/enforce": "baseline"}),
                       ("strict", {"pod-security.kubernetes.io/warn": "restricted"})):
        assert _raw(kube, "POST", "/api/v1/namespaces", {"apiVersion": "v1", "kind": "Namespace",
                                                         "metadata": {"name": ns, "labels": labels}})[0] == 201
    pod = lambda name, **spec: {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name},
                                "spec": {"containers": [{"name": "c", "command": ["true"]}], **spec}}
    code, _, body = _raw(kube, "POST", "/api/v1/namespaces/tenant/pods", pod("dev", volumes=[
        {"name": "d", "hostPath": {"path": "/dev"}}]))
    assert code == 403 and 'violates PodSecurity "baseline:latest"' in body["message"] and "hostPath" in body["message"]
    code, _, body = _raw(kube, "POST", "/api/v1/namespaces/tenant/pods", pod("net", hostNetwork=True))
    assert code == 403 and "host namespaces" in body["message"]
    assert _raw(kube, "POST", "/api/v1/namespaces/tenant/pods", pod("ok"))[0] == 201
    conn = http.client.HTTPConnection(kube.host, kube.port, timeout=10)
    conn.request("POST", kube.k8s("/api/v1/namespaces/strict/pods"), body=json.dumps(pod("loose")),
                 headers={"Authorization": f"Bearer {kube.token}", "Content-Type": "application/json"})
    r = conn.getresponse()
    r.read()
    assert r.status == 201 and "restricted:latest" in (r.getheader("Warning") or "")
    assert "runAsNonRoot" in r.getheader("Warning")
    conn.close()
