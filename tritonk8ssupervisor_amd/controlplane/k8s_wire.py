"""Kubernetes wire conventions of the control plane, for stock clients (kubectl, client-go, the
Python kubernetes client), not only tk8s's own:

* API discovery: ``/api`` (APIVersions), ``/apis`` (APIGroupList), ``/api/v1`` and
  ``/apis/<group>/<version>`` (APIResourceList) -- what kubectl reads before any request.
* Typed objects and lists: every object carries ``apiVersion``/``kind``, lists are
  ``<Kind>List`` of their group version.
* ``Status`` error bodies with the machine-readable ``reason`` clients branch on (NotFound,
  AlreadyExists, Conflict, Invalid, Forbidden, Expired ...).
* Field selectors (``metadata.name=x``, ``spec.nodeName=n``, ``status.phase!=Running``).
* Patch types: JSON merge patch (RFC 7386), JSON patch (RFC 6902), and the strategic merge patch
  kubectl apply/edit/patch send, with its list merge keys and ``$patch``/``$setElementOrder``
  directives.
* Server-side ``Table`` output (``Accept: application/json;as=Table;g=meta.k8s.io;v=v1``) so
  ``kubectl get`` prints real columns, GPU columns for nodes included.

The reference's cluster was a real Rancher-launched Kubernetes that any kubectl could use
(/root/reference/setup.sh:181-183 prints the kubeconfig URL for it); this module is what lets a
stock kubectl pointed at that kubeconfig work against the tk8s control plane.
"""
from __future__ import annotations

import copy
import time

# plural -> (group, version, Kind, singular, namespaced, short names, subresources)
RESOURCES: dict[str, tuple[str, str, str, str, bool, tuple[str, ...], tuple[str, ...]]] = {
    "pods": ("", "v1", "Pod", "pod", True, ("po",), ("log", "status", "exec", "portforward", "attach", "eviction")),
    "services": ("", "v1", "Service", "service", True, ("svc",), ()),
    "events": ("", "v1", "Event", "event", True, ("ev",), ()),
    "configmaps": ("", "v1", "ConfigMap", "configmap", True, ("cm",), ()),
    "secrets": ("", "v1", "Secret", "secret", True, (), ()),
    "persistentvolumeclaims": ("", "v1", "PersistentVolumeClaim", "persistentvolumeclaim", True, ("pvc",), ()),
    "persistentvolumes": ("", "v1", "PersistentVolume", "persistentvolume", False, ("pv",), ()),
    "storageclasses": ("storage.k8s.io", "v1", "StorageClass", "storageclass", False, ("sc",), ()),
    "namespaces": ("", "v1", "Namespace", "namespace", False, ("ns",), ()),
    "nodes": ("", "v1", "Node", "node", False, ("no",), ("status",)),
    "daemonsets": ("apps", "v1", "DaemonSet", "daemonset", True, ("ds",), ()),
    "deployments": ("apps", "v1", "Deployment", "deployment", True, ("deploy",), ("scale",)),
    "statefulsets": ("apps", "v1", "StatefulSet", "statefulset", True, ("sts",), ("scale",)),
    "replicasets": ("apps", "v1", "ReplicaSet", "replicaset", True, ("rs",), ("scale",)),
    "jobs": ("batch", "v1", "Job", "job", True, (), ()),
    "cronjobs": ("batch", "v1", "CronJob", "cronjob", True, ("cj",), ()),
    "horizontalpodautoscalers": ("autoscaling", "v2", "HorizontalPodAutoscaler", "horizontalpodautoscaler", True,
                                 ("hpa",), ()),
    "serviceaccounts": ("", "v1", "ServiceAccount", "serviceaccount", True, ("sa",), ()),
    "endpoints": ("", "v1", "Endpoints", "endpoints", True, ("ep",), ()),
    "resourcequotas": ("", "v1", "ResourceQuota", "resourcequota", True, ("quota",), ()),
    "limitranges": ("", "v1", "LimitRange", "limitrange", True, ("limits",), ()),
    "leases": ("coordination.k8s.io", "v1", "Lease", "lease", True, (), ()),
    "roles": ("rbac.authorization.k8s.io", "v1", "Role", "role", True, (), ()),
    "rolebindings": ("rbac.authorization.k8s.io", "v1", "RoleBinding", "rolebinding", True, (), ()),
    "clusterroles": ("rbac.authorization.k8s.io", "v1", "ClusterRole", "clusterrole", False, (), ()),
    "clusterrolebindings": ("rbac.authorization.k8s.io", "v1", "ClusterRoleBinding", "clusterrolebinding", False, (), ()),
    "customresourcedefinitions": ("apiextensions.k8s.io", "v1", "CustomResourceDefinition", "customresourcedefinition",
                                  False, ("crd", "crds"), ()),
    "ingresses": ("networking.k8s.io", "v1", "Ingress", "ingress", True, ("ing",), ()),
    "ingressclasses": ("networking.k8s.io", "v1", "IngressClass", "ingressclass", False, (), ()),
    "poddisruptionbudgets": ("policy", "v1", "PodDisruptionBudget", "poddisruptionbudget", True, ("pdb",), ("status",)),
    "priorityclasses": ("scheduling.k8s.io", "v1", "PriorityClass", "priorityclass", False, ("pc",), ()),
    "mutatingwebhookconfigurations": ("admissionregistration.k8s.io", "v1", "MutatingWebhookConfiguration",
                                      "mutatingwebhookconfiguration", False, (), ()),
    "validatingwebhookconfigurations": ("admissionregistration.k8s.io", "v1", "ValidatingWebhookConfiguration",
                                        "validatingwebhookconfiguration", False, (), ()),
}
READ_ONLY = {"namespaces": ("create", "delete", "get", "list", "patch", "watch"),
             "events": ("get", "list", "watch", "create", "delete")}
VERBS = ("create", "delete", "get", "list", "patch", "update", "watch")


def group_version(plural: str) -> str:
    g, v = RESOURCES[plural][:2]
    return f"{g}/{v}" if g else v


def type_meta() -> dict[str, tuple[str, str]]:
    """plural -> (apiVersion, Kind): what the store stamps on every object it keeps."""
    return {p: (group_version(p), r[2]) for p, r in RESOURCES.items()}


def list_kind(plural: str) -> tuple[str, str]:
    return group_version(plural), RESOURCES[plural][2] + "List"


# ---- discovery ----------------------------------------------------------------------------
def api_versions(server_address: str) -> dict:
    return {"kind": "APIVersions", "versions": ["v1"],
            "serverAddressByClientCIDRs": [{"clientCIDR": "0.0.0.0/0", "serverAddress": server_address}]}


def _groups() -> list[tuple[str, str]]:
    seen: list[tuple[str, str]] = []
    for g, v, *_ in RESOURCES.values():
        if g and (g, v) not in seen:
            seen.append((g, v))
    # served by metrics_api.py and rbac.py, not objects
    return seen + [("metrics.k8s.io", "v1beta1"), ("authorization.k8s.io", "v1")]


def api_group_list() -> dict:
    return {"kind": "APIGroupList", "apiVersion": "v1", "groups": [
        {"name": g, "versions": [{"groupVersion": f"{g}/{v}", "version": v}],
         "preferredVersion": {"groupVersion": f"{g}/{v}", "version": v}} for g, v in _groups()]}


def api_group(group: str) -> dict | None:
    for g, v in _groups():
        if g == group:
            return {"kind": "APIGroup", "apiVersion": "v1", "name": g,
                    "versions": [{"groupVersion": f"{g}/{v}", "version": v}],
                    "preferredVersion": {"groupVersion": f"{g}/{v}", "version": v}}
    return None


def api_resource_list(group: str, version: str) -> dict | None:
    res = []
    for plural, (g, v, kind, singular, namespaced, short, subs) in RESOURCES.items():
        if (g, v) != (group, version):
            continue
        r = {"name": plural, "singularName": singular, "namespaced": namespaced, "kind": kind,
             "verbs": list(READ_ONLY.get(plural, VERBS))}
        if short:
            r["shortNames"] = list(short)
        if plural in ("pods", "deployments", "daemonsets", "jobs", "services", "statefulsets", "replicasets", "cronjobs",
                      "horizontalpodautoscalers"):
            r["categories"] = ["all"]
        res.append(r)
        for s in subs:
            sub = {"name": f"{plural}/{s}", "singularName": "", "namespaced": namespaced, "kind": kind,
                   "verbs": ["get"] if s == "log" else ["create", "get"] if s in ("exec", "portforward", "attach")
                   else ["create"] if s == "eviction"
                   else ["get", "patch", "update"]}
            if s == "scale":
                sub.update(kind="Scale", group="autoscaling", version="v1")
            elif s == "eviction":
                sub.update(kind="Eviction", group="policy", version="v1")
            res.append(sub)
    if not res:
        return None
    return {"kind": "APIResourceList", "apiVersion": "v1", "groupVersion": f"{group}/{version}" if group else version,
            "resources": res}


# ---- errors -------------------------------------------------------------------------------
REASONS = {400: "BadRequest", 401: "Unauthorized", 403: "Forbidden", 404: "NotFound", 405: "MethodNotAllowed",
           409: "Conflict", 410: "Expired", 415: "UnsupportedMediaType", 422: "Invalid", 429: "TooManyRequests",
           500: "InternalError",
           503: "ServiceUnavailable", 504: "Timeout"}


def status_body(code: int, message: str, reason: str | None = None) -> dict:
    if reason is None:
        reason = REASONS.get(code, "Unknown")
        if code == 409 and "already exists" in message:
            reason = "AlreadyExists"
    return {"kind": "Status", "apiVersion": "v1", "metadata": {}, "status": "Failure", "message": message,
            "reason": reason, "code": code}


def is_k8s_path(path: str) -> bool:
    """The Kubernetes API's paths, bare or behind the Rancher project proxy prefix."""
    if path.startswith("/r/projects/"):
        parts = path.split("/", 5)  # '', r, projects, pid, kubernetes, rest
        path = "/" + parts[5] if len(parts) > 5 and parts[4] == "kubernetes" else ""
    return path == "/api" or path.startswith(("/api/", "/apis", "/openapi/"))


# ---- field selectors ----------------------------------------------------------------------
def parse_field_selector(s: str | None) -> list[tuple[str, str, str]]:
    """``a.b=x,c!=y`` -> [(a.b, '=', x), (c, '!=', y)] (``==`` is ``=``)."""
    out = []
    for part in (s or "").split(","):
        part = part.strip()
        if not part:
            continue
        if "!=" in part:
            k, v = part.split("!=", 1)
            out.append((k.strip(), "!=", v.strip()))
        elif "=" in part:
            k, v = part.split("=", 1)
            out.append((k.strip(), "=", v.strip().lstrip("=")))
    return out


def _field(obj: dict, path: str) -> str:
    cur = obj
    for p in path.split("."):
        if not isinstance(cur, dict):
            return ""
        cur = cur.get(p)
    if cur is None:
        return ""
    if isinstance(cur, bool):
        return "true" if cur else "false"
    return str(cur)


def fields_match(sel: list[tuple[str, str, str]], obj: dict) -> bool:
    for path, op, want in sel:
        have = _field(obj, path)
        if path == "metadata.namespace" and not have:
            have = "default"
        if (have == want) != (op == "="):
            return False
    return True


# ---- patches ------------------------------------------------------------------------------
MERGE_PATCH = "application/merge-patch+json"
JSON_PATCH = "application/json-patch+json"
STRATEGIC_PATCH = "application/strategic-merge-patch+json"
APPLY_PATCH = "application/apply-patch+yaml"

# list field -> merge key, for the kinds served here (k8s.io/api patchMergeKey tags)
MERGE_KEYS = {"containers": "name", "initContainers": "name", "ephemeralContainers": "name", "env": "name",
              "volumes": "name", "volumeMounts": "mountPath", "volumeDevices": "devicePath",
              "imagePullSecrets": "name", "ports": None,  # container ports: containerPort, service ports: port
              "hostAliases": "ip", "conditions": "type", "ownerReferences": "uid", "finalizers": None}


def _ports_key(items: list) -> str | None:
    for it in items:
        if isinstance(it, dict):
            if "containerPort" in it:
                return "containerPort"
            if "port" in it:
                return "port"
    return None


def strategic_merge(target, patch):
    """Strategic merge patch: maps merge key by key (``null`` deletes, ``$patch: replace|delete``),
    lists with a merge key merge element by element (``$patch: delete`` removes one element,
    ``$setElementOrder/<field>`` orders the result), other lists are replaced whole;
    ``$retainKeys`` keeps only the listed keys; ``$deleteFromPrimitiveList/<field>`` removes values."""
    if not isinstance(patch, dict):
        return copy.deepcopy(patch)
    if patch.get("$patch") == "replace":
        return {k: copy.deepcopy(v) for k, v in patch.items() if k != "$patch"}
    if patch.get("$patch") == "delete":
        return None
    out = copy.deepcopy(target) if isinstance(target, dict) else {}
    orders = {}
    for k, v in patch.items():
        if k.startswith("$setElementOrder/"):
            orders[k.split("/", 1)[1]] = v
        elif k.startswith("$deleteFromPrimitiveList/"):
            f = k.split("/", 1)[1]
            if isinstance(out.get(f), list):
                out[f] = [x for x in out[f] if x not in (v or [])]
        elif k in ("$retainKeys", "$patch"):
            continue
        elif v is None:
            out.pop(k, None)
        elif isinstance(v, list) and k in MERGE_KEYS:
            out[k] = _merge_list(out.get(k), v, MERGE_KEYS[k] or (_ports_key(v + list(out.get(k) or [])) if k == "ports" else None))
        elif isinstance(v, dict):
            merged = strategic_merge(out.get(k), v)
            if merged is None:
                out.pop(k, None)
            else:
                out[k] = merged
        else:
            out[k] = copy.deepcopy(v)
    if "$retainKeys" in patch:
        keep = set(patch["$retainKeys"] or [])
        out = {k: v for k, v in out.items() if k in keep}
    for f, order in orders.items():
        key = MERGE_KEYS.get(f) or (_ports_key(order) if f == "ports" else None)
        if key and isinstance(out.get(f), list):
            rank = {str(o.get(key)): i for i, o in enumerate(order) if isinstance(o, dict)}
            out[f] = sorted(out[f], key=lambda e: rank.get(str(e.get(key)) if isinstance(e, dict) else "", len(rank)))
    return out


def _merge_list(cur, patch: list, key: str | None) -> list:
    if not key:  # primitives (finalizers) merge as a set union, keeping order; others replace
        if all(not isinstance(x, (dict, list)) for x in patch):
            base = list(cur or [])
            return base + [x for x in patch if x not in base]
        return copy.deepcopy(patch)
    out = [copy.deepcopy(e) for e in (cur or [])]
    for el in patch:
        if not isinstance(el, dict) or key not in el:
            continue
        idx = next((i for i, e in enumerate(out) if isinstance(e, dict) and e.get(key) == el[key]), None)
        if el.get("$patch") == "delete":
            if idx is not None:
                out.pop(idx)
            continue
        if idx is None:
            out.append({k: v for k, v in copy.deepcopy(el).items() if k != "$patch"})
        else:
            out[idx] = strategic_merge(out[idx], el)
    return out


class PatchError(ValueError):
    pass


def _pointer(path: str) -> list[str]:
    if path == "":
        return []
    if not path.startswith("/"):
        raise PatchError(f"invalid JSON pointer {path!r}")
    return [p.replace("~1", "/").replace("~0", "~") for p in path[1:].split("/")]


def json_patch(doc, ops: list):
    """RFC 6902: add, remove, replace, move, copy, test."""
    if not isinstance(ops, list):
        raise PatchError("a JSON patch is a list of operations")
    doc = copy.deepcopy(doc)

    def parent(d, parts):
        for p in parts[:-1]:
            d = d[_index(p)] if isinstance(d, list) else d[p]
        return d

    def get(d, parts):
        for p in parts:
            d = d[_index(p)] if isinstance(d, list) else d[p]
        return d

    def add(d, parts, value):
        if not parts:
            return value
        par, last = parent(d, parts), parts[-1]
        if isinstance(par, list):
            if last == "-":
                par.append(value)
                return d
            idx = _index(last)
            if idx > len(par):  # RFC 6902 4.1: an index past the end is an error, not an append
                raise PatchError(f"index {last} out of bounds (array of {len(par)})")
            par.insert(idx, value)
        else:
            par[last] = value
        return d

    def _index(tok: str) -> int:
        if not tok.isdigit() or (len(tok) > 1 and tok[0] == "0"):  # RFC 6901: no sign, no leading zero
            raise PatchError(f"invalid array index {tok!r}")
        return int(tok)

    def remove(d, parts):
        par, last = parent(d, parts), parts[-1]
        if isinstance(par, list):
            return par.pop(_index(last))
        return par.pop(last)

    for i, op in enumerate(ops):
        try:
            kind, parts = op["op"], _pointer(op["path"])
            if kind == "add":
                doc = add(doc, parts, copy.deepcopy(op["value"]))
            elif kind == "remove":
                remove(doc, parts)
            elif kind == "replace":
                get(doc, parts)  # must exist
                if not parts:
                    doc = copy.deepcopy(op["value"])
                else:
                    par = parent(doc, parts)
                    par[_index(parts[-1]) if isinstance(par, list) else parts[-1]] = copy.deepcopy(op["value"])
            elif kind in ("move", "copy"):
                src = _pointer(op["from"])
                val = remove(doc, src) if kind == "move" else copy.deepcopy(get(doc, src))
                doc = add(doc, parts, val)
            elif kind == "test":
                if get(doc, parts) != op["value"]:
                    raise PatchError(f"test operation {i} failed at {op['path']}")
            else:
                raise PatchError(f"unknown operation {kind!r}")
        except (KeyError, IndexError, ValueError, TypeError) as e:
            if isinstance(e, PatchError):
                raise
            raise PatchError(f"operation {i} ({op.get('op') if isinstance(op, dict) else op!r}) failed: {e}") from e
    return doc


# ---- server-side printing (Table) ----------------------------------------------------------
def wants_table(accept: str) -> bool:
    return "as=Table" in (accept or "")


def _age(obj: dict) -> str:
    ts = (obj.get("metadata") or {}).get("creationTimestamp")
    if not ts:
        return "<unknown>"
    from calendar import timegm  # only for printing; off the control plane's start-up path

    try:
        s = max(0, int(time.time() - timegm(time.strptime(ts, "%Y-%m-%dT%H:%M:%SZ"))))
    except ValueError:
        return "<unknown>"
    for unit, n in (("d", 86400), ("h", 3600), ("m", 60)):
        if s >= n:
            return f"{s // n}{unit}"
    return f"{s}s"


def _cond(obj: dict, t: str) -> dict:
    return next((c for c in (obj.get("status") or {}).get("conditions") or [] if c.get("type") == t), {})


def _node_row(n: dict) -> list:
    ready = _cond(n, "Ready").get("status")
    st = "Ready" if ready == "True" else "NotReady"
    if (n.get("spec") or {}).get("unschedulable"):
        st += ",SchedulingDisabled"
    val = _cond(n, "AMDGPUValidated").get("status")
    s = n.get("status") or {}
    gpus = f"{(s.get('allocatable') or {}).get('amd.com/gpu', '0')}/{(s.get('capacity') or {}).get('amd.com/gpu', '0')}"
    return [n["metadata"]["name"], st, "worker", _age(n), (s.get("nodeInfo") or {}).get("kubeletVersion", ""), gpus,
            {"True": "yes", "False": "FAILED"}.get(val, "pending")]


def _pod_row(p: dict) -> list:
    cs = (p.get("status") or {}).get("containerStatuses") or []
    n = len((p.get("spec") or {}).get("containers") or [])
    ready = sum(1 for c in cs if c.get("ready"))
    restarts = sum(int(c.get("restartCount", 0)) for c in cs)
    phase = (p.get("status") or {}).get("phase", "Pending")
    if p["metadata"].get("deletionTimestamp"):
        phase = "Terminating"
    return [p["metadata"]["name"], f"{ready}/{n}", phase if phase == "Terminating" else (p.get("status") or {}).get("reason")
            or phase, restarts, _age(p),
            (p.get("status") or {}).get("podIP", "<none>"), (p.get("spec") or {}).get("nodeName", "<none>")]


def _deploy_row(d: dict) -> list:
    s, want = d.get("status") or {}, int((d.get("spec") or {}).get("replicas", 1))
    return [d["metadata"]["name"], f"{s.get('readyReplicas', 0)}/{want}", s.get("updatedReplicas", 0),
            s.get("availableReplicas", 0), _age(d)]


def _job_row(j: dict) -> list:
    s, spec = j.get("status") or {}, j.get("spec") or {}
    return [j["metadata"]["name"], f"{s.get('succeeded', 0)}/{spec.get('completions', 1)}", _age(j)]


def _svc_row(o: dict) -> list:
    spec = o.get("spec") or {}
    ports = ",".join(f"{p.get('port')}{':' + str(p['nodePort']) if p.get('nodePort') else ''}/{p.get('protocol', 'TCP')}"
                     for p in spec.get("ports") or [])
    lb = ((o.get("status") or {}).get("loadBalancer") or {}).get("ingress") or []
    return [o["metadata"]["name"], spec.get("type", "ClusterIP"), spec.get("clusterIP", ""),
            ",".join(i.get("ip", "") for i in lb) or "<none>", ports or "<none>", _age(o)]


def _sts_row(o: dict) -> list:
    s = o.get("status") or {}
    return [o["metadata"]["name"], f"{s.get('readyReplicas', 0)}/{(o.get('spec') or {}).get('replicas', 1)}", _age(o)]


def _rs_row(o: dict) -> list:
    s = o.get("status") or {}
    return [o["metadata"]["name"], (o.get("spec") or {}).get("replicas", 1), s.get("replicas", 0),
            s.get("readyReplicas", 0), _age(o)]


def _cj_row(o: dict) -> list:
    spec, s = o.get("spec") or {}, o.get("status") or {}
    return [o["metadata"]["name"], spec.get("schedule", ""), spec.get("timeZone") or "<none>",
            str(bool(spec.get("suspend", False))), len(s.get("active") or []),
            _age({"metadata": {"creationTimestamp": s["lastScheduleTime"]}}) if s.get("lastScheduleTime") else "<none>",
            _age(o)]


def _pvc_row(o: dict) -> list:
    spec, s = o.get("spec") or {}, o.get("status") or {}
    return [o["metadata"]["name"], s.get("phase", "Pending"), spec.get("volumeName", ""),
            (s.get("capacity") or {}).get("storage", ""), ",".join(_ACCESS.get(m, m) for m in spec.get("accessModes") or []),
            spec.get("storageClassName", ""), _age(o)]


_ACCESS = {"ReadWriteOnce": "RWO", "ReadOnlyMany": "ROX", "ReadWriteMany": "RWX", "ReadWriteOncePod": "RWOP"}


def _ds_row(o: dict) -> list:
    s = o.get("status") or {}
    return [o["metadata"]["name"], s.get("desiredNumberScheduled", 0), s.get("currentNumberScheduled", 0),
            s.get("numberReady", 0), _age(o)]


def _pdb_row(o: dict) -> list:
    spec, s = o.get("spec") or {}, o.get("status") or {}
    return [o["metadata"]["name"], str(spec.get("minAvailable", "N/A")), str(spec.get("maxUnavailable", "N/A")),
            s.get("disruptionsAllowed", 0), _age(o)]


_S, _I = "string", "integer"
TABLES = {
    "nodes": ([("Name", _S), ("Status", _S), ("Roles", _S), ("Age", _S), ("Version", _S), ("GPU", _S),
               ("Validated", _S)], _node_row),
    "pods": ([("Name", _S), ("Ready", _S), ("Status", _S), ("Restarts", _I), ("Age", _S), ("IP", _S), ("Node", _S)],
             _pod_row),
    "deployments": ([("Name", _S), ("Ready", _S), ("Up-to-date", _I), ("Available", _I), ("Age", _S)], _deploy_row),
    "jobs": ([("Name", _S), ("Completions", _S), ("Age", _S)], _job_row),
    "services": ([("Name", _S), ("Type", _S), ("Cluster-IP", _S), ("External-IP", _S), ("Port(s)", _S), ("Age", _S)],
                 _svc_row),
    "daemonsets": ([("Name", _S), ("Desired", _I), ("Current", _I), ("Ready", _I), ("Age", _S)], _ds_row),
    "statefulsets": ([("Name", _S), ("Ready", _S), ("Age", _S)], _sts_row),
    "persistentvolumeclaims": ([("Name", _S), ("Status", _S), ("Volume", _S), ("Capacity", _S), ("Access Modes", _S),
                                ("StorageClass", _S), ("Age", _S)], _pvc_row),
    "replicasets": ([("Name", _S), ("Desired", _I), ("Current", _I), ("Ready", _I), ("Age", _S)], _rs_row),
    "cronjobs": ([("Name", _S), ("Schedule", _S), ("Timezone", _S), ("Suspend", _S), ("Active", _I),
                  ("Last Schedule", _S), ("Age", _S)], _cj_row),
    "poddisruptionbudgets": ([("Name", _S), ("Min Available", _S), ("Max Unavailable", _S), ("Allowed Disruptions", _I),
                              ("Age", _S)], _pdb_row),
}


def table(plural: str | None, items: list[dict], resource_version: str) -> dict:
    cols, row = TABLES.get(plural or "", ([("Name", _S), ("Age", _S)], lambda o: [o["metadata"]["name"], _age(o)]))
    defs = [{"name": n, "type": t, "format": "name" if n == "Name" else "", "description": "", "priority": 0}
            for n, t in cols]
    rows = []
    for o in items:
        md = {k: v for k, v in (o.get("metadata") or {}).items() if k in ("name", "namespace", "uid", "resourceVersion",
                                                                         "creationTimestamp", "labels")}
        rows.append({"cells": row(o), "object": {"kind": "PartialObjectMetadata", "apiVersion": "meta.k8s.io/v1",
                                                 "metadata": md}})
    return {"kind": "Table", "apiVersion": "meta.k8s.io/v1", "metadata": {"resourceVersion": resource_version},
            "columnDefinitions": defs, "rows": rows}
