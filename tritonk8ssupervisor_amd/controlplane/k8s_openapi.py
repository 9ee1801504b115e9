"""OpenAPI v3 documents for the kinds the control plane serves (``/openapi/v3`` and
``/openapi/v3/<api/v1 | apis/G/V>``), and the server's side of ``fieldValidation``.

Why it exists: a stock ``kubectl apply/create`` validates by default. It first asks the OpenAPI v3
document of the object's group version whether the PATCH operation of that kind takes the
``fieldValidation`` query parameter; if it does, kubectl leaves validation to the server and sends
``?fieldValidation=Strict``. Without any OpenAPI document kubectl stops with "failed to download
openapi" unless the user adds ``--validate=false``. So the documents here carry what that check
reads -- per-kind paths, ``x-kubernetes-group-version-kind`` on every operation, the write
operations' query parameters -- plus a loose schema per kind (for ``kubectl explain``), and
``check_fields`` is the server-side validation those clients then rely on.

Deliberately not advertised: ``application/strategic-merge-patch+json`` in the PATCH request
bodies. kubectl would then build client-side-apply patches from these schemas, which carry no
list merge keys; without it kubectl uses its compiled-in types, whose merge keys match
``k8s_wire.MERGE_KEYS``.

Reference: the reference's users pointed any kubectl at the cluster it printed
(/root/reference/setup.sh:181-183); there is no code of the reference behind this module.
"""
from __future__ import annotations

import json

from . import k8s_wire

GVK = "x-kubernetes-group-version-kind"
_WRITE_PARAMS = ("dryRun", "fieldManager", "fieldValidation")
_DESCRIPTIONS = {
    "Pod": "A group of processes (containers) scheduled together onto a node, with their GPUs.",
    "Service": "A named, load-balanced address for the pods a selector matches.",
    "Event": "A report of something that happened to an object.",
    "ConfigMap": "Non-secret configuration data for pods.",
    "Secret": "Secret data for pods (base64 in data, plain text in stringData).",
    "Namespace": "A scope for names.",
    "Node": "A worker: its capacity (amd.com/gpu), conditions and GPU validation.",
    "DaemonSet": "One pod per matching node.",
    "Deployment": "A replicated, rolling-updated set of pods.",
    "Job": "Pods that run to completion (Indexed jobs get JOB_COMPLETION_INDEX).",
    "Ingress": "HTTP routing from the node's proxy to Services.",
    "StatefulSet": "Pods with stable names <name>-<ordinal>, their own DNS names and claims.",
    "ReplicaSet": "A number of identical pods.",
    "CronJob": "A Job on a schedule.",
    "PersistentVolumeClaim": "Node-local storage that outlives pods (class tk8s-local).",
    "HorizontalPodAutoscaler": "Scales a workload by its pods' CPU or memory use.",
    "PodDisruptionBudget": "How many of a set of pods voluntary disruptions (evictions, drains) may take down.",
    "PriorityClass": "A named pod priority; higher-priority pods schedule first and may preempt lower ones.",
}
# the top-level fields each kind's objects may have (fieldValidation=Strict rejects others)
_TOP = {"Pod": ("spec", "status"), "Service": ("spec", "status"), "Node": ("spec", "status"),
        "Namespace": ("spec", "status"), "DaemonSet": ("spec", "status"), "Deployment": ("spec", "status"),
        "Job": ("spec", "status"), "Ingress": ("spec", "status"),
        "ConfigMap": ("data", "binaryData", "immutable"),
        "ServiceAccount": ("secrets", "imagePullSecrets", "automountServiceAccountToken"),
        "Role": ("rules",), "ClusterRole": ("rules", "aggregationRule"),
        "RoleBinding": ("roleRef", "subjects"), "ClusterRoleBinding": ("roleRef", "subjects"),
        "Secret": ("data", "stringData", "type", "immutable"),
        "PriorityClass": ("value", "globalDefault", "description", "preemptionPolicy"),
        "MutatingWebhookConfiguration": ("webhooks",), "ValidatingWebhookConfiguration": ("webhooks",),
        "StorageClass": ("provisioner", "parameters", "reclaimPolicy", "volumeBindingMode", "allowVolumeExpansion",
                         "mountOptions", "allowedTopologies"),
        "Endpoints": ("subsets",),
        "Event": ("involvedObject", "reason", "message", "source", "firstTimestamp", "lastTimestamp", "count",
                  "type", "eventTime", "series", "action", "related", "reportingComponent",
                  "reportingInstance")}
OBJECT_META = ("name", "generateName", "namespace", "selfLink", "uid", "resourceVersion", "generation",
               "creationTimestamp", "deletionTimestamp", "deletionGracePeriodSeconds", "labels", "annotations",
               "ownerReferences", "finalizers", "managedFields")


def gv_key(group: str, version: str) -> str:
    return f"apis/{group}/{version}" if group else f"api/{version}"


def _gvs() -> list[tuple[str, str]]:
    """The group versions with objects (metrics.k8s.io has no writable objects: no document)."""
    out: list[tuple[str, str]] = []
    for g, v, *_ in k8s_wire.RESOURCES.values():
        if (g, v) not in out:
            out.append((g, v))
    return out


def _schema_name(group: str, version: str, kind: str) -> str:
    pkg = {"": "core", "apps": "apps", "batch": "batch", "networking.k8s.io": "networking",
           "autoscaling": "autoscaling", "rbac.authorization.k8s.io": "rbac"}.get(group, group)
    return f"io.k8s.api.{pkg}.{version}.{kind}"


def _param(name: str, desc: str, where: str = "query", required: bool = False, kind: str = "string") -> dict:
    return {"name": name, "in": where, "description": desc, "required": required, "schema": {"type": kind}}


_PARAM_DESC = {
    "dryRun": "When present, modifications are not persisted (All).",
    "fieldManager": "Name of the actor making the change (managed fields).",
    "fieldValidation": "Ignore, Warn or Strict: what to do with unknown or duplicate fields.",
    "force": "Server-side apply: take the conflicting fields from their other managers.",
}


def _op(action: str, gvk: dict, ref: str, op_id: str, writes: bool = False, patch: bool = False) -> dict:
    op = {"operationId": op_id, "x-kubernetes-action": action, GVK: dict(gvk),
          "responses": {"200": {"description": "OK", "content": {"application/json": {"schema": {"$ref": ref}}}}}}
    params = []
    if writes:
        params += [_param(n, _PARAM_DESC[n]) for n in _WRITE_PARAMS]
    if patch:
        params.append(_param("force", _PARAM_DESC["force"], kind="boolean"))
        op["requestBody"] = {"content": {t: {"schema": {"type": "object"}} for t in (
            k8s_wire.JSON_PATCH, k8s_wire.MERGE_PATCH, k8s_wire.APPLY_PATCH)}, "required": True}
    elif writes and action in ("post", "put"):
        op["requestBody"] = {"content": {"application/json": {"schema": {"$ref": ref}}}, "required": True}
    if params:
        op["parameters"] = params
    return op


def gv_document(group: str, version: str) -> dict | None:
    """The OpenAPI 3.0 document of one group version (paths + component schemas)."""
    paths: dict[str, dict] = {}
    schemas: dict[str, dict] = {}
    base = f"/apis/{group}/{version}" if group else f"/api/{version}"
    for plural, (g, v, kind, _singular, namespaced, _short, _subs) in k8s_wire.RESOURCES.items():
        if (g, v) != (group, version):
            continue
        gvk = {"group": g, "version": v, "kind": kind}
        name = _schema_name(g, v, kind)
        ref = f"#/components/schemas/{name}"
        top = {f: {"type": "object" if f in ("spec", "status", "data", "binaryData", "stringData", "involvedObject",
                                              "source", "series", "related", "roleRef", "aggregationRule") else
                   "array" if f in ("rules", "subjects", "secrets", "imagePullSecrets") else
                   "boolean" if f in ("immutable", "automountServiceAccountToken") else
                   "integer" if f == "count" else "string",
                   **({"x-kubernetes-preserve-unknown-fields": True} if f in ("spec", "status") else {})}
               for f in _TOP.get(kind, ("spec", "status"))}
        schemas[name] = {"type": "object", "description": _DESCRIPTIONS.get(kind, kind), GVK: [gvk],
                         "properties": {"apiVersion": {"type": "string"}, "kind": {"type": "string"},
                                        "metadata": {"$ref": "#/components/schemas/io.k8s.apimachinery.pkg.apis.meta.v1.ObjectMeta"},
                                        **top}}
        schemas[name + "List"] = {"type": "object", GVK: [{**gvk, "kind": kind + "List"}], "properties": {
            "apiVersion": {"type": "string"}, "kind": {"type": "string"}, "metadata": {"type": "object"},
            "items": {"type": "array", "items": {"$ref": ref}}}}
        lref = f"#/components/schemas/{name}List"
        coll = f"{base}/namespaces/{{namespace}}/{plural}" if namespaced else f"{base}/{plural}"
        ns_param = [_param("namespace", "object name and auth scope", "path", True)] if namespaced else []
        pid = f"{kind}{'Namespaced' if namespaced else ''}"
        paths[coll] = {"parameters": ns_param,
                       "get": _op("list", gvk, lref, f"list{pid}"),
                       "post": _op("post", gvk, ref, f"create{pid}", writes=True)}
        item_params = [*ns_param, _param("name", f"name of the {kind}", "path", True)]
        paths[coll + "/{name}"] = {"parameters": item_params,
                                   "get": _op("get", gvk, ref, f"read{pid}"),
                                   "put": _op("put", gvk, ref, f"replace{pid}", writes=True),
                                   "patch": _op("patch", gvk, ref, f"patch{pid}", writes=True, patch=True),
                                   "delete": _op("delete", gvk, ref, f"delete{pid}")}
        if namespaced:
            paths[f"{base}/{plural}"] = {"get": _op("list", gvk, lref, f"list{kind}ForAllNamespaces")}
    if not paths:
        return None
    schemas["io.k8s.apimachinery.pkg.apis.meta.v1.ObjectMeta"] = {
        "type": "object", "description": "Standard object metadata.",
        "properties": {f: {"type": "object" if f in ("labels", "annotations") else
                           "array" if f in ("ownerReferences", "finalizers", "managedFields") else
                           "integer" if f in ("generation", "deletionGracePeriodSeconds") else "string"}
                       for f in OBJECT_META}}
    return {"openapi": "3.0.0", "info": {"title": "tk8s", "version": "v1"}, "paths": paths,
            "components": {"schemas": schemas}}


def _hash(doc: dict) -> str:
    import hashlib  # (the control plane's start-up path imports this module)

    return hashlib.sha512(json.dumps(doc, sort_keys=True).encode()).hexdigest()[:32].upper()


_DOCS: dict[str, tuple[dict, str]] = {}


def document(key: str) -> tuple[dict, str] | None:
    """``api/v1`` / ``apis/G/V`` -> (document, its hash), built once."""
    if key not in _DOCS:
        parts = key.split("/")
        if parts[0] == "api" and len(parts) == 2:
            doc = gv_document("", parts[1])
        elif parts[0] == "apis" and len(parts) == 3:
            doc = gv_document(parts[1], parts[2])
        else:
            doc = None
        if doc is None:
            return None
        _DOCS[key] = (doc, _hash(doc))
    return _DOCS[key]


def root(prefix: str) -> dict:
    """``/openapi/v3``: each group version's document, by server-relative URL. client-go replaces
    the kubeconfig server's path with this URL, so it carries the project prefix when there is one."""
    paths = {}
    for g, v in _gvs():
        key = gv_key(g, v)
        _doc, h = document(key)
        paths[key] = {"serverRelativeURL": f"{prefix}/openapi/v3/{key}?hash={h}"}
    return {"paths": paths}


def check_fields(kind_plural: str, body: dict, mode: str | None) -> list[str]:
    """Server-side field validation of a create/update/apply body: the unknown top-level and
    ``metadata`` fields. ``mode`` Strict -> the caller answers 400 with these; Warn -> Warning
    headers; Ignore/None -> nothing is checked. Nested fields are not checked."""
    if not mode or mode.lower() == "ignore" or not isinstance(body, dict) or kind_plural not in k8s_wire.RESOURCES:
        return []
    kind = k8s_wire.RESOURCES[kind_plural][2]
    allowed = {"apiVersion", "kind", "metadata", *_TOP.get(kind, ("spec", "status"))}
    bad = [f'unknown field "{k}"' for k in body if k not in allowed]
    md = body.get("metadata")
    if isinstance(md, dict):
        bad += [f'unknown field "metadata.{k}"' for k in md if k not in OBJECT_META]
    return bad
