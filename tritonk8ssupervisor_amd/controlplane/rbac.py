"""ServiceAccounts and RBAC authorization (rbac.authorization.k8s.io/v1) for the Kubernetes API
subset: who a request is, and whether it may do what it asks.

Identities (``identity_of``):

* the project's API token (the kubeconfig's) -- the cluster administrator;
* a node agent's token -- ``system:node:<name>``, with the access nodes have always had here;
* a ServiceAccount token (the ``kubernetes.io/service-account-token`` Secret the control plane
  keeps for every ServiceAccount, mounted into pods) -- ``system:serviceaccount:<ns>:<name>``,
  authorized by Roles/ClusterRoles bound to it (or to ``system:serviceaccounts[:<ns>]`` /
  ``system:authenticated``) through RoleBindings/ClusterRoleBindings;
* no token -- anonymous: discovery, ``/version`` and health only (authn.PUBLIC).

Request attributes (``request_info``) follow the API server's: verb (get, list, watch, create,
update, patch, delete, deletecollection), API group, resource[/subresource], namespace, name.
Built-in ClusterRoles ``cluster-admin``, ``admin``, ``edit`` and ``view`` are created with each
project (``view``: read everything but Secrets; ``edit``: view + write workloads, config and
Secrets, no RBAC; ``admin``: edit + namespaced RBAC).
"""
from __future__ import annotations

import re
from collections import namedtuple

_PREFIX = re.compile(r"^/r/projects/[^/]+/kubernetes(?=/)")

WORKLOAD_RESOURCES = ["pods", "pods/log", "pods/exec", "pods/portforward", "pods/attach", "pods/eviction", "services",
                      "configmaps", "poddisruptionbudgets",
                      "secrets", "persistentvolumeclaims", "serviceaccounts", "events", "deployments",
                      "deployments/scale", "statefulsets", "statefulsets/scale", "replicasets", "replicasets/scale",
                      "daemonsets", "jobs", "cronjobs", "ingresses", "horizontalpodautoscalers"]
READ = ["get", "list", "watch"]
WRITE = ["create", "update", "patch", "delete", "deletecollection"]
ALL_GROUPS = ["", "apps", "batch", "networking.k8s.io", "autoscaling", "metrics.k8s.io", "policy"]

BUILTIN_CLUSTER_ROLES = {
    "cluster-admin": [{"apiGroups": ["*"], "resources": ["*"], "verbs": ["*"]}],
    "admin": [{"apiGroups": ALL_GROUPS, "resources": WORKLOAD_RESOURCES, "verbs": READ + WRITE},
              {"apiGroups": ["rbac.authorization.k8s.io"], "resources": ["roles", "rolebindings"], "verbs": READ + WRITE}],
    "edit": [{"apiGroups": ALL_GROUPS, "resources": WORKLOAD_RESOURCES, "verbs": READ + WRITE}],
    "view": [{"apiGroups": ALL_GROUPS, "resources": [r for r in WORKLOAD_RESOURCES if r not in (
        "secrets", "pods/exec", "pods/portforward", "pods/attach", "pods/eviction")] + ["namespaces", "nodes"], "verbs": READ}],
}


class RequestInfo(namedtuple("RequestInfo", "verb group resource namespace name")):
    """What a request does: verb, API group, resource ("pods", or "pods/log" for a subresource),
    namespace, name. (A named tuple: ``dataclasses`` costs the first authorised request ~1 ms of
    imports, and that request is on the bring-up's critical path.)"""

    __slots__ = ()

    def describe(self) -> str:
        where = f' in the namespace "{self.namespace}"' if self.namespace else " at the cluster scope"
        return f'cannot {self.verb} resource "{self.resource}" in API group "{self.group}"{where}'


def request_info(method: str, path: str, query: dict) -> RequestInfo | None:
    """The resource request a path is, or None for a non-resource path (discovery, OpenAPI...)."""
    path = _PREFIX.sub("", path).rstrip("/")
    parts = [p for p in path.split("/") if p]
    if not parts:
        return None
    if parts[0] == "api" and len(parts) >= 2:
        group, rest = "", parts[2:]
    elif parts[0] == "apis" and len(parts) >= 3:
        group, rest = parts[1], parts[3:]
    else:
        return None
    if not rest:
        return None  # discovery of a group version
    ns = ""
    if rest[0] == "namespaces" and len(rest) >= 3:
        ns, rest = rest[1], rest[2:]
    elif rest[0] == "namespaces":  # the namespaces resource itself
        return RequestInfo(_verb(method, len(rest) > 1, query), "", "namespaces", "", rest[1] if len(rest) > 1 else "")
    resource = rest[0]
    name = rest[1] if len(rest) > 1 else ""
    if len(rest) > 2:
        resource = f"{resource}/{rest[2]}"
    return RequestInfo(_verb(method, bool(name), query), group, resource, ns, name)


def _verb(method: str, named: bool, query: dict) -> str:
    if method in ("GET", "HEAD"):
        if query.get("watch") in ("1", "true"):
            return "watch"
        return "get" if named else "list"
    return {"POST": "create", "PUT": "update", "PATCH": "patch",
            "DELETE": "delete" if named else "deletecollection"}.get(method, method.lower())


def rule_allows(rule: dict, info: RequestInfo) -> bool:
    def has(field: str, value: str) -> bool:
        vals = rule.get(field) or []
        return "*" in vals or value in vals

    if not has("verbs", info.verb) or not has("apiGroups", info.group):
        return False
    res = rule.get("resources") or []
    base = info.resource.split("/")[0]
    if not ("*" in res or info.resource in res or (f"{base}/*" in res and "/" in info.resource)):
        return False
    names = rule.get("resourceNames") or []
    return not names or info.name in names


def subject_matches(subject: dict, ns: str, sa: str) -> bool:
    kind = subject.get("kind")
    if kind == "ServiceAccount":
        return subject.get("name") == sa and subject.get("namespace", "") == ns
    if kind == "Group":
        return subject.get("name") in ("system:authenticated", "system:serviceaccounts", f"system:serviceaccounts:{ns}")
    if kind == "User":
        return subject.get("name") == f"system:serviceaccount:{ns}:{sa}"
    return False


def allowed(roles: dict, cluster_roles: dict, bindings: list[dict], cluster_bindings: list[dict],
            ns: str, sa: str, info: RequestInfo) -> bool:
    """Is ServiceAccount ns/sa allowed ``info``? ``roles``: (namespace, name) -> rules;
    ``cluster_roles``: name -> rules; bindings with ``metadata.namespace``, ``roleRef``, ``subjects``."""
    def role_rules(ref: dict, bind_ns: str) -> list[dict]:
        if ref.get("kind") == "ClusterRole":
            return cluster_roles.get(ref.get("name"), BUILTIN_CLUSTER_ROLES.get(ref.get("name"), []))
        return roles.get((bind_ns, ref.get("name")), [])

    for b in cluster_bindings:
        if any(subject_matches(s, ns, sa) for s in b.get("subjects") or []):
            if any(rule_allows(r, info) for r in role_rules(b.get("roleRef") or {}, "")):
                return True
    if info.namespace:
        for b in bindings:
            if b["metadata"].get("namespace") != info.namespace:
                continue
            if any(subject_matches(s, ns, sa) for s in b.get("subjects") or []):
                if any(rule_allows(r, info) for r in role_rules(b.get("roleRef") or {}, info.namespace)):
                    return True
    return False
