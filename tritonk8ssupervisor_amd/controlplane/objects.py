"""Object helpers of the control plane (split out of server.py): store keys, node conditions and
readiness, GPU counts, merge patches, template hashes, admission, label selectors.
"""
from __future__ import annotations

import copy
import json
import re

from .httpserver import HttpError
from .store import now_iso

GPU = "amd.com/gpu"
VALIDATION_LABEL = "tk8s.amd.com/validation"
TERMINAL = ("Succeeded", "Failed")
KIND_GROUPS = (("pods", "/api/v1"), ("services", "/api/v1"), ("events", "/api/v1"), ("configmaps", "/api/v1"),
               ("secrets", "/api/v1"), ("persistentvolumeclaims", "/api/v1"), ("daemonsets", "/apis/apps/v1"), ("deployments", "/apis/apps/v1"),
               ("statefulsets", "/apis/apps/v1"), ("replicasets", "/apis/apps/v1"),
               ("jobs", "/apis/batch/v1"), ("cronjobs", "/apis/batch/v1"), ("ingresses", "/apis/networking.k8s.io/v1"),
               ("horizontalpodautoscalers", "/apis/autoscaling/v2"), ("serviceaccounts", "/api/v1"),
               ("endpoints", "/api/v1"), ("leases", "/apis/coordination.k8s.io/v1"), ("resourcequotas", "/api/v1"),
               ("roles", "/apis/rbac.authorization.k8s.io/v1"), ("rolebindings", "/apis/rbac.authorization.k8s.io/v1"))
# cluster-scoped kinds served through the generic handlers (namespace "")
CLUSTER_KIND_GROUPS = (("clusterroles", "/apis/rbac.authorization.k8s.io/v1"),
                       ("clusterrolebindings", "/apis/rbac.authorization.k8s.io/v1"),
                       ("customresourcedefinitions", "/apis/apiextensions.k8s.io/v1"))


def _key(*parts: str) -> str:
    return "/".join(parts)


def _cond(obj: dict, ctype: str) -> dict | None:
    for c in obj.get("status", {}).get("conditions", []):
        if c.get("type") == ctype:
            return c
    return None


def _set_cond(obj: dict, ctype: str, status: str, reason: str = "", message: str = "") -> bool:
    conds = obj.setdefault("status", {}).setdefault("conditions", [])
    for c in conds:
        if c["type"] == ctype:
            changed = c.get("status") != status or c.get("reason") != reason
            if changed:
                c["lastTransitionTime"] = now_iso()
            c.update(status=status, reason=reason, message=message)
            return changed
    conds.append({"type": ctype, "status": status, "reason": reason, "message": message,
                  "lastTransitionTime": now_iso()})
    return True


def node_ready(n: dict) -> bool:
    c = _cond(n, "Ready")
    return bool(c and c["status"] == "True")


UNREACHABLE = "node.kubernetes.io/unreachable"


def _set_ready(node: dict, message: str = "tk8s agent heartbeating") -> bool:
    """Ready follows the heartbeat, unless the node's xGMI links failed the pre-Ready check
    (xgmi.py): then it stays NotReady with that reason while the agent is alive. A heartbeat
    also lifts the unreachable taints a lost lease put on the node (server.lease_loop)."""
    spec = node.setdefault("spec", {})
    lifted = False
    if any(t.get("key") == UNREACHABLE for t in spec.get("taints") or []):
        spec["taints"] = [t for t in spec["taints"] if t.get("key") != UNREACHABLE]
        lifted = True
    x = _cond(node, "XGMILinksHealthy")
    if x and x["status"] == "False":
        return _set_cond(node, "Ready", "False", "XGMILinkDegraded", x.get("message", "")) or lifted
    return _set_cond(node, "Ready", "True", "AgentReady", message) or lifted


def node_validated(n: dict) -> bool:
    c = _cond(n, "AMDGPUValidated")
    return bool(c and c["status"] == "True")


def pod_gpus(p: dict) -> int:
    total = 0
    for c in p.get("spec", {}).get("containers", []):
        r = c.get("resources", {})
        v = r.get("limits", {}).get(GPU, r.get("requests", {}).get(GPU, 0))
        total += int(v or 0)
    return total


def _xgmi_view(result: dict) -> dict | None:
    """The xGMI link verdict of a validation result: the host burn-in's share carries it
    (``xgmi``); a machine's own multi-GPU probe carries raw pulls, judged here."""
    if not isinstance(result, dict):
        return None
    if isinstance(result.get("xgmi"), dict):
        return result["xgmi"]
    if any(d.get("peers") for d in result.get("devices") or []):
        from .. import xgmi

        rep = xgmi.link_report(result)
        return xgmi.node_view(rep, sorted({e["src"] for e in rep["links"]} | {e["dst"] for e in rep["links"]}))
    return None


def merge_patch(target, patch):
    """RFC 7386 JSON merge patch (what kubectl's merge and strategic-merge patches reduce to here:
    maps merge key by key, ``null`` deletes, lists are replaced whole)."""
    if not isinstance(patch, dict):
        return copy.deepcopy(patch)
    out = copy.deepcopy(target) if isinstance(target, dict) else {}
    for k, v in patch.items():
        if v is None:
            out.pop(k, None)
        else:
            out[k] = merge_patch(out.get(k), v)
    return out


def template_hash(template: dict) -> str:
    """``pod-template-hash`` of a Deployment's pod template (names its ReplicaSet generation):
    CRC-32 and Adler-32 of its canonical JSON, 10 hex digits -- a name, not a security check
    (Kubernetes uses FNV-32). zlib, not hashlib: OpenSSL's binding costs the first DaemonSet
    create ~2.5 ms of imports, on the bring-up's critical path."""
    import zlib

    b = json.dumps(template, sort_keys=True, separators=(",", ":")).encode()
    return f"{zlib.crc32(b):08x}{zlib.adler32(b):08x}"[:10]


GPU_VISIBILITY = "tk8s.amd.com/gpu-visibility"
GPU_SCOPE = "tk8s.amd.com/gpu-scope"
# annotations only the cluster's own fabric Jobs may carry: the pod's runtime sees every GPU of its
# node (xGMI peer-to-peer between ranks), or one process drives GPUs of several nodes of a host
_RESERVED = ((GPU_VISIBILITY, "node"), (GPU_SCOPE, "host"))
# set by the scheduler on host-scoped pods (scheduler.py): never by a client
_SCHEDULER_OWNED = ("tk8s.amd.com/host-claims", "tk8s.amd.com/host-devices")
# an Indexed Job's pods on one host open each other's GPUs (agent.py _gather_peers): from the
# Job's template only; the GPUs each pod was given are published by its node agent (pod status)
GPU_PEERS = "tk8s.amd.com/gpu-peers"
GPU_DEVICES = "tk8s.amd.com/gpu-devices"
_AGENT_OWNED = (GPU_DEVICES, GPU_PEERS, "amd.com/gpu-ids")
# what a workload's pod template may never carry: the controllers copy template
# annotations into the pods they create, so a forged record there would reach a pod unchecked
_TEMPLATE_FORBIDDEN = (GPU_DEVICES, "amd.com/gpu-ids") + _SCHEDULER_OWNED


def strip_owned(annotations: dict) -> dict:
    """A pod template's annotations without the node's and the scheduler's own records."""
    return {k: v for k, v in annotations.items() if k not in _TEMPLATE_FORBIDDEN}


def _reserved(ann: dict) -> str | None:
    for k, v in _RESERVED:
        if ann.get(k) == v:
            return f"{k}: {v}"
    return None


_DNS_LABEL = re.compile(r"^[a-z0-9]([-a-z0-9]*[a-z0-9])?$")


def check_pod_spec_names(what: str, spec: dict) -> None:
    """Container and volume names are DNS-1123 labels, as kube-apiserver validates them: the node
    builds paths from them (a pod's volumes/<name>, rootfs-<name>), so ``../x`` must never reach
    it (a volume named ``../../..`` wrote into any directory the agent could)."""
    for field in ("initContainers", "containers", "volumes"):
        for i, x in enumerate(spec.get(field) or []):
            n = x.get("name") if isinstance(x, dict) else None
            if not isinstance(n, str) or len(n) > 63 or not _DNS_LABEL.match(n):
                raise HttpError(422, f'{what} is invalid: spec.{field}[{i}].name: Invalid value: {n!r}: a lowercase '
                                     "RFC 1123 label must consist of lower case alphanumeric characters or '-', and "
                                     "must start and end with an alphanumeric character")


def _admit_gpu_visibility(kind: str, ns: str, body: dict, cur: dict | None = None) -> None:
    """Admission for the fabric-only GPU annotations (``gpu-visibility: node``, ``gpu-scope: host``):
    only kube-system Jobs may carry them in their pod template; a pod cannot ask for them itself --
    not at create, and not later through PUT / merge / JSON / strategic patches (``cur``: the
    object being replaced; a pod may keep what its Job gave it, never add or change it). The
    agent re-checks the owner against the real Job's uid (agent.node_visibility_allowed)."""
    if kind == "pods":
        ann = (body.get("metadata") or {}).get("annotations") or {}
        old = ((cur or {}).get("metadata") or {}).get("annotations") or {}
        for k, _v in _RESERVED:
            if ann.get(k) != old.get(k) and _reserved({k: ann.get(k)}):
                raise HttpError(403, f'pods is forbidden: annotation {_reserved({k: ann.get(k)})} is reserved for '
                                     'kube-system Jobs')
        for k in _SCHEDULER_OWNED:
            if ann.get(k) != old.get(k):
                raise HttpError(403, f"pods is forbidden: annotation {k} is set by the scheduler")
        for k in _AGENT_OWNED:
            if ann.get(k) != old.get(k):
                raise HttpError(403, f"pods is forbidden: annotation {k} comes from an Indexed Job's pod template "
                                     "and the pod's node" if k == GPU_PEERS else
                                f"pods is forbidden: annotation {k} is set by the pod's node")
    elif kind in ("jobs", "daemonsets", "deployments", "statefulsets", "replicasets", "cronjobs"):
        spec = body.get("spec") or {}
        if kind == "cronjobs":
            spec = (spec.get("jobTemplate") or {}).get("spec") or {}
        ann = (spec.get("template") or {}).get("metadata", {}).get("annotations") or {}
        for k in _TEMPLATE_FORBIDDEN:
            if k in ann:
                raise HttpError(403, f"{kind} is forbidden: annotation {k} in a pod template: it is set "
                                     + ("by the scheduler" if k in _SCHEDULER_OWNED else "by the pod's node"))
        what = _reserved(ann)
        if what and (kind != "jobs" or ns != "kube-system"):
            raise HttpError(403, f"{kind} is forbidden: annotation {what} is reserved for kube-system Jobs")
        if GPU_PEERS in ann:
            if kind not in ("jobs", "cronjobs") or spec.get("completionMode") != "Indexed":
                raise HttpError(422, f"{kind} is invalid: annotation {GPU_PEERS} is for the pod template of an "
                                     "Indexed Job (completionMode: Indexed)")
            if ann[GPU_PEERS] != "job":
                raise HttpError(422, f'{kind} is invalid: annotation {GPU_PEERS}: supported value: "job"')


def _normalize_data(kind: str, body: dict) -> None:
    """ConfigMap data must be strings; Secret ``stringData`` folds into base64 ``data``."""
    import base64
    import binascii

    if kind == "configmaps":
        data = body.get("data") or {}
        if not isinstance(data, dict) or not all(isinstance(v, str) for v in data.values()):
            raise HttpError(422, "ConfigMap data must map keys to strings")
        body["data"] = data
    elif kind == "secrets":
        data = dict(body.get("data") or {})
        for k, v in (body.pop("stringData", None) or {}).items():
            data[k] = base64.b64encode(str(v).encode()).decode()
        for k, v in data.items():
            try:
                base64.b64decode(str(v), validate=True)
            except (binascii.Error, ValueError) as e:
                raise HttpError(422, f"Secret data[{k!r}] is not valid base64: {e}") from e
        body["data"] = data
        body.setdefault("type", "Opaque")


def labels_match(selector: dict | None, labels: dict | None) -> bool:
    if not selector:
        return True
    labels = labels or {}
    return all(labels.get(k) == v for k, v in selector.items())


def _parse_selector(s: str | None) -> dict | None:
    if not s:
        return None
    out = {}
    for part in s.split(","):
        if "=" in part:
            k, v = part.split("=", 1)
            out[k.strip().rstrip("=")] = v.strip()
    return out


QUOTA_BLOCKED = "tk8s.amd.com/quota-blocked"  # a controller's pod held back by a ResourceQuota


def pod_usage(pod: dict) -> dict[str, float]:
    """What a pod counts against a ResourceQuota: pods, amd.com/gpu, cpu/memory requests and limits."""
    from ..utils import quantity

    out = {"pods": 1.0, f"requests.{GPU}": float(pod_gpus(pod))}
    for c in pod.get("spec", {}).get("containers", []):
        r = c.get("resources") or {}
        for sect in ("requests", "limits"):
            for res in ("cpu", "memory"):
                v = (r.get(sect) or {}).get(res)
                if v is None and sect == "requests":  # a request defaults to the limit, as in Kubernetes
                    v = (r.get("limits") or {}).get(res)
                if v is not None:
                    out[f"{sect}.{res}"] = out.get(f"{sect}.{res}", 0.0) + quantity.parse(v)
    out[GPU] = out[f"requests.{GPU}"]
    out["cpu"], out["memory"] = out.get("requests.cpu", 0.0), out.get("requests.memory", 0.0)
    return out


def quota_excess(hard: dict, used: dict, add: dict) -> list[str]:
    """The resources a quota's ``hard`` limits that ``used`` + ``add`` would exceed."""
    from ..utils import quantity

    bad = []
    for res, lim in (hard or {}).items():
        name = "pods" if res == "count/pods" else res
        if name in add and used.get(name, 0.0) + add[name] > quantity.parse(lim) + 1e-9:
            bad.append(f"{res}: requested {_fmt(add[name])}, used {_fmt(used.get(name, 0.0))}, limited {lim}")
    return bad


def _fmt(v: float) -> str:
    return str(int(v)) if float(v).is_integer() else f"{v:g}"


def apply_limit_ranges(ranges: list[dict], pod: dict) -> list[str]:
    """LimitRange admission of a pod (in place): each ``type: Container`` item's ``default``
    (limits) and ``defaultRequest`` (requests) fill what a container leaves out -- a request
    defaults to the limit when only that is given -- then ``min``/``max`` and
    ``maxLimitRequestRatio`` are checked; ``type: Pod`` items check the containers' sums. The
    violations, as the API server words them (empty: admitted)."""
    from ..utils import quantity

    bad = []
    conts = pod.get("spec", {}).get("containers", []) + pod.get("spec", {}).get("initContainers", [])
    for lr in ranges:
        for item in (lr.get("spec") or {}).get("limits") or []:
            typ = item.get("type", "Container")
            if typ == "Container":
                for c in conts:
                    r = c.setdefault("resources", {})
                    lim, req = r.setdefault("limits", {}), r.setdefault("requests", {})
                    for res, v in list(lim.items()):  # the API's own defaulting: a request is its limit
                        req.setdefault(res, v)
                    for res, v in (item.get("default") or {}).items():
                        lim.setdefault(res, v)
                    for res, v in (item.get("defaultRequest") or {}).items():
                        req.setdefault(res, v)
                    for res, v in lim.items():  # no defaultRequest: the default limit
                        req.setdefault(res, v)
                    if not lim:
                        r.pop("limits")
                    if not req:
                        r.pop("requests")
                    for res, v in (item.get("min") or {}).items():
                        for what, d in (("request", req), ("limit", lim)):
                            if res in d and quantity.parse(d[res]) < quantity.parse(v):
                                bad.append(f"minimum {res} usage per Container is {v}, but {what} is {d[res]}")
                    for res, v in (item.get("max") or {}).items():
                        if res not in lim:
                            bad.append(f"maximum {res} usage per Container is {v}.  No limit is specified")
                        elif quantity.parse(lim[res]) > quantity.parse(v):
                            bad.append(f"maximum {res} usage per Container is {v}, but limit is {lim[res]}")
                    for res, v in (item.get("maxLimitRequestRatio") or {}).items():
                        if res in lim and res in req and quantity.parse(req[res]) > 0 and \
                                quantity.parse(lim[res]) / quantity.parse(req[res]) > float(quantity.parse(v)):
                            bad.append(f"{res} max limit to request ratio per Container is {v}, but provided ratio is "
                                       f"{quantity.parse(lim[res]) / quantity.parse(req[res]):g}")
            elif typ == "Pod":
                for res, v in (item.get("max") or {}).items():
                    tot = sum(quantity.parse(((c.get("resources") or {}).get("limits") or {}).get(res, 0)) for c in conts)
                    if tot > quantity.parse(v):
                        bad.append(f"maximum {res} usage per Pod is {v}, but limit is {_fmt(tot)}")
                for res, v in (item.get("min") or {}).items():
                    tot = sum(quantity.parse(((c.get("resources") or {}).get("requests") or {}).get(res, 0)) for c in conts)
                    if tot < quantity.parse(v):
                        bad.append(f"minimum {res} usage per Pod is {v}, but request is {_fmt(tot)}")
    return bad
