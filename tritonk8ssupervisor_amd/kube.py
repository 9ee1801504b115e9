"""Kubernetes object helpers shared by kubectl, the playbook's tk8s_kube module and setup.

Maps kinds to API paths, loads (templated) multi-document manifests, applies/deletes objects and
waits for conditions with the control plane's long-poll watch (no sleep loops).
"""
from __future__ import annotations

import time
from pathlib import Path

from . import templating
from .controlplane.client import ApiError, Client
from .utils import yamlio

# server-side apply's content type (= controlplane/k8s_wire.APPLY_PATCH, pinned by
# tests/test_kube_helpers.py): spelled out here so setup's deploy task, on the bring-up's critical
# path, does not import the control plane's wire module (and `copy`, `weakref`) for one string
APPLY_PATCH = "application/apply-patch+yaml"

KINDS = {
    "pod": ("Pod", "/api/v1", "pods"),
    "service": ("Service", "/api/v1", "services"),
    "event": ("Event", "/api/v1", "events"),
    "daemonset": ("DaemonSet", "/apis/apps/v1", "daemonsets"),
    "deployment": ("Deployment", "/apis/apps/v1", "deployments"),
    "job": ("Job", "/apis/batch/v1", "jobs"),
    "statefulset": ("StatefulSet", "/apis/apps/v1", "statefulsets"),
    "replicaset": ("ReplicaSet", "/apis/apps/v1", "replicasets"),
    "cronjob": ("CronJob", "/apis/batch/v1", "cronjobs"),
    "horizontalpodautoscaler": ("HorizontalPodAutoscaler", "/apis/autoscaling/v2", "horizontalpodautoscalers"),
    "serviceaccount": ("ServiceAccount", "/api/v1", "serviceaccounts"),
    "role": ("Role", "/apis/rbac.authorization.k8s.io/v1", "roles"),
    "rolebinding": ("RoleBinding", "/apis/rbac.authorization.k8s.io/v1", "rolebindings"),
    "clusterrole": ("ClusterRole", "/apis/rbac.authorization.k8s.io/v1", "clusterroles"),
    "clusterrolebinding": ("ClusterRoleBinding", "/apis/rbac.authorization.k8s.io/v1", "clusterrolebindings"),
    "customresourcedefinition": ("CustomResourceDefinition", "/apis/apiextensions.k8s.io/v1", "customresourcedefinitions"),
    "configmap": ("ConfigMap", "/api/v1", "configmaps"),
    "secret": ("Secret", "/api/v1", "secrets"),
    "persistentvolumeclaim": ("PersistentVolumeClaim", "/api/v1", "persistentvolumeclaims"),
    "ingress": ("Ingress", "/apis/networking.k8s.io/v1", "ingresses"),
    "poddisruptionbudget": ("PodDisruptionBudget", "/apis/policy/v1", "poddisruptionbudgets"),
    "priorityclass": ("PriorityClass", "/apis/scheduling.k8s.io/v1", "priorityclasses"),
    "limitrange": ("LimitRange", "/api/v1", "limitranges"),
    "persistentvolume": ("PersistentVolume", "/api/v1", "persistentvolumes"),
    "storageclass": ("StorageClass", "/apis/storage.k8s.io/v1", "storageclasses"),
    "ingressclass": ("IngressClass", "/apis/networking.k8s.io/v1", "ingressclasses"),
    "resourcequota": ("ResourceQuota", "/api/v1", "resourcequotas"),
    "mutatingwebhookconfiguration": ("MutatingWebhookConfiguration", "/apis/admissionregistration.k8s.io/v1",
                                     "mutatingwebhookconfigurations"),
    "validatingwebhookconfiguration": ("ValidatingWebhookConfiguration", "/apis/admissionregistration.k8s.io/v1",
                                       "validatingwebhookconfigurations"),
}
ALIASES = {"po": "pod", "pods": "pod", "svc": "service", "services": "service", "ds": "daemonset",
           "daemonsets": "daemonset", "deploy": "deployment", "deployments": "deployment", "jobs": "job",
           "ev": "event", "events": "event", "no": "node", "nodes": "node", "cm": "configmap",
           "configmaps": "configmap", "secrets": "secret", "ing": "ingress", "ingresses": "ingress",
           "sts": "statefulset", "statefulsets": "statefulset", "rs": "replicaset", "replicasets": "replicaset",
           "cj": "cronjob", "cronjobs": "cronjob", "pvc": "persistentvolumeclaim",
           "persistentvolumeclaims": "persistentvolumeclaim", "ns": "namespace", "namespaces": "namespace",
           "hpa": "horizontalpodautoscaler", "horizontalpodautoscalers": "horizontalpodautoscaler",
           "sa": "serviceaccount", "serviceaccounts": "serviceaccount", "roles": "role", "rolebindings": "rolebinding",
           "clusterroles": "clusterrole", "clusterrolebindings": "clusterrolebinding", "crd": "customresourcedefinition",
           "crds": "customresourcedefinition", "customresourcedefinitions": "customresourcedefinition",
           "pdb": "poddisruptionbudget", "poddisruptionbudgets": "poddisruptionbudget",
           "pc": "priorityclass", "priorityclasses": "priorityclass", "limits": "limitrange",
           "limitranges": "limitrange", "quota": "resourcequota", "resourcequotas": "resourcequota",
           "pv": "persistentvolume", "persistentvolumes": "persistentvolume", "sc": "storageclass",
           "storageclasses": "storageclass", "ingressclasses": "ingressclass"}


CLUSTER_SCOPED: set[str] = {"customresourcedefinition", "priorityclass", "mutatingwebhookconfiguration",
                             "validatingwebhookconfiguration", "persistentvolume", "storageclass", "ingressclass"}  # (+ kinds learnt from discovery without a namespace)


def learn_kind(k: Client, name: str) -> str | None:
    """A kind the bundled client does not know (a CustomResourceDefinition's): find it by plural,
    singular, kind or short name in the server's discovery and remember where it lives."""
    want = name.lower()
    for g in k.get(k.k8s("/apis")).get("groups", []):
        gv = g["preferredVersion"]["groupVersion"]
        try:
            res = k.get(k.k8s(f"/apis/{gv}")).get("resources", [])
        except ApiError:
            continue
        for r in res:
            if "/" in r["name"]:
                continue
            names = {r["name"], r.get("singularName", ""), r.get("kind", "").lower(), *r.get("shortNames", [])}
            if want in names:
                key = r.get("singularName") or r["kind"].lower()
                KINDS[key] = (r["kind"], f"/apis/{gv}", r["name"])
                for n in names - {""}:
                    ALIASES.setdefault(n, key)
                if not r.get("namespaced", True):
                    CLUSTER_SCOPED.add(key)
                return key
    return None


def kind_key(kind: str) -> str:
    k = kind.lower()
    return ALIASES.get(k, k)


def collection_path(kind: str, ns: str = "default") -> str:
    k = kind_key(kind)
    if k == "node":
        return "/api/v1/nodes"
    if k == "namespace":
        return "/api/v1/namespaces"
    if k in ("clusterrole", "clusterrolebinding") or k in CLUSTER_SCOPED:  # cluster-scoped
        return f"{KINDS[k][1]}/{KINDS[k][2]}"
    if k not in KINDS:
        raise ValueError(f"unsupported kind {kind!r}")
    _, group, plural = KINDS[k]
    return f"{group}/namespaces/{ns}/{plural}"


def object_path(kind: str, name: str, ns: str = "default") -> str:
    return f"{collection_path(kind, ns)}/{name}"


def load_manifests(path: str | Path, variables: dict | None = None) -> list[dict]:
    """The objects of a manifest file (``-``: standard input, as ``kubectl apply -f -``)."""
    if str(path) == "-":
        import sys

        text = sys.stdin.read()
    else:
        text = Path(path).read_text()
    docs = [d for d in yamlio.load_all(text) if d]
    if variables:
        docs = templating.render(docs, variables)
    out = []
    for d in docs:
        if d.get("kind") == "List":
            out += d.get("items", [])
        else:
            out.append(d)
    return out


def is_subset(want, have) -> bool:
    """Does the live object already carry every field the manifest sets? (server-side defaults
    such as a Service's clusterIP or nodePorts do not count as a difference)."""
    if isinstance(want, dict):
        return isinstance(have, dict) and all(is_subset(v, have.get(k)) for k, v in want.items())
    if isinstance(want, list):
        return isinstance(have, list) and len(want) == len(have) and all(is_subset(a, b) for a, b in zip(want, have))
    return want == have or (want is not None and have is not None and str(want) == str(have))


def _ensure_namespace(k: Client, o: dict) -> dict:
    try:
        k.post(k.k8s("/api/v1/namespaces"), {"apiVersion": "v1", "kind": "Namespace", "metadata": {
            "name": o["metadata"]["name"], **{f: o["metadata"][f] for f in ("labels", "annotations") if o["metadata"].get(f)}}})
        return {"created": True, "action": "created"}
    except ApiError as e:
        if e.status != 409:
            raise
        return {"created": False, "action": "unchanged"}


def _known(k: Client, kind: str) -> None:
    if kind_key(kind) not in KINDS and kind_key(kind) not in ("node", "namespace"):
        learn_kind(k, kind)


def apply_objects(k: Client, objs: list[dict]) -> list[dict]:
    """``kubectl apply``: create, or update an existing object to the manifest (PUT with the live
    resourceVersion; status and server-allocated fields are kept by the control plane)."""
    res = []
    for o in objs:
        kind = o.get("kind", "")
        if kind.lower() == "namespace":
            res.append({"kind": kind, "name": o["metadata"]["name"], **_ensure_namespace(k, o)})
            continue
        _known(k, kind)
        ns = o.get("metadata", {}).get("namespace", "default")
        name = o["metadata"].get("name")
        try:
            k.post(k.k8s(collection_path(kind, ns)), o)
            res.append({"kind": kind, "name": name, "created": True, "action": "created"})
            continue
        except ApiError as e:
            if e.status != 409:
                raise
        path = k.k8s(object_path(kind, name, ns))
        cur = k.get(path)
        want = {key: v for key, v in o.items() if key not in ("apiVersion", "kind", "status")}
        if is_subset(want, cur):
            action = "unchanged"
        else:
            import copy

            body = copy.deepcopy(o)
            md = body.setdefault("metadata", {})
            md["resourceVersion"] = cur["metadata"]["resourceVersion"]
            for f in ("labels", "annotations"):  # apply merges map fields it does not mention
                md[f] = {**cur["metadata"].get(f, {}), **(md.get(f) or {})}
            k.put(path, body)
            action = "configured"
        res.append({"kind": kind, "name": name, "created": False, "action": action})
    return res


def server_apply_objects(k: Client, objs: list[dict], manager: str = "kubectl", force: bool = False,
                         dry_run: bool = False) -> list[dict]:
    """``kubectl apply --server-side``: one ``PATCH application/apply-patch+yaml`` per object; the
    control plane merges it and tracks field ownership (controlplane/ssa.py). A conflict with
    another manager raises ApiError 409 unless ``force`` (``--force-conflicts``)."""
    res = []
    for o in objs:
        kind = o.get("kind", "")
        if kind.lower() == "namespace":
            _ensure_namespace(k, o)
            res.append({"kind": kind, "name": o["metadata"]["name"], "action": "serverside-applied"})
            continue
        _known(k, kind)
        ns = o.get("metadata", {}).get("namespace", "default")
        name = o["metadata"]["name"]
        q = {"fieldManager": manager, "force": "true" if force else None, "dryRun": "All" if dry_run else None}
        k.request("PATCH", k.k8s(object_path(kind, name, ns)), body=o, query=q, content_type=APPLY_PATCH)
        res.append({"kind": kind, "name": name, "action": "serverside-applied"})
    return res


def delete_objects(k: Client, objs: list[dict]) -> int:
    """``kubectl delete -f``: the objects, then the manifest's namespaces (with what is left in them)."""
    n = 0
    for o in sorted(objs, key=lambda o: o.get("kind", "").lower() == "namespace"):
        kind = o.get("kind", "")
        _known(k, kind)
        ns = o.get("metadata", {}).get("namespace", "default")
        try:
            k.delete(k.k8s(object_path(kind, o["metadata"]["name"], ns)))
            n += 1
        except ApiError as e:
            if e.status != 404:
                raise
    return n


def job_state(job: dict) -> str:
    for c in job.get("status", {}).get("conditions", []):
        if c.get("type") in ("Complete", "Failed") and c.get("status") == "True":
            return c["type"]
    return "Running"


def wait_job(k: Client, name: str, ns: str = "default", timeout: float = 300.0) -> dict:
    """Block (long-poll watch) until the Job is Complete or Failed; returns the Job."""
    deadline = time.monotonic() + timeout
    path = k.k8s(collection_path("job", ns))
    rv = 0
    while True:
        job = k.get(k.k8s(object_path("job", name, ns)))
        if job_state(job) != "Running":
            return job
        left = deadline - time.monotonic()
        if left <= 0:
            raise TimeoutError(f"job {ns}/{name} not finished after {timeout}s")
        rv = max(rv, int(job["metadata"]["resourceVersion"]))
        rv, _ = k.watch(path, rv, timeout=min(left, 20.0))


def rollout_complete(d: dict) -> bool:
    st, want = d.get("status", {}), int(d["spec"].get("replicas", 1))
    return (int(st.get("observedGeneration", 0)) >= int(d["metadata"].get("generation", 1))
            and st.get("updatedReplicas", 0) == want and st.get("replicas", 0) == want
            and st.get("readyReplicas", 0) == want)


def wait_rollout(k: Client, name: str, ns: str = "default", timeout: float = 300.0, progress=None) -> dict:
    """Block (long-poll watch) until every replica of the Deployment runs the current template."""
    deadline = time.monotonic() + timeout
    path = k.k8s(collection_path("deployment", ns))
    last = None
    while True:
        d = k.get(k.k8s(object_path("deployment", name, ns)))
        if rollout_complete(d):
            return d
        st = d.get("status", {})
        msg = (st.get("updatedReplicas", 0), st.get("readyReplicas", 0), st.get("replicas", 0))
        if progress is not None and msg != last:
            progress(d)
        last = msg
        left = deadline - time.monotonic()
        if left <= 0:
            raise TimeoutError(f"deployment {ns}/{name} not rolled out after {timeout}s")
        k.watch(path, int(d["metadata"]["resourceVersion"]), timeout=min(left, 20.0))


def pods_of(k: Client, label_selector: str, ns: str = "default") -> list[dict]:
    return k.get(k.k8s(collection_path("pod", ns)), query={"labelSelector": label_selector})["items"]
