"""Who a request is, and the limits of the identities that are not ServiceAccounts.

The reference ran Rancher 1.x with access control off: anyone who could reach ``:8080`` could
create environments, read registration URLs and fetch the kubeconfig
(ansible/roles/ranchermaster/tasks/main.yml:29-52, rancherhost/tasks/main.yml:11-24 call the API
with no credentials). Here the server is on a shared host, next to the cluster's own workloads,
so every request names a bearer token except a short public list (``PUBLIC``):

* the **server admin token** -- created with the control plane (``<state-dir>/admin-token``,
  mode 0600, or ``$TK8S_ADMIN_TOKEN``); the roles read it on the master and keep a copy in the
  workspace's ``.tk8s/`` (which the pod jail denies, agent/runtime.py). It creates environments
  and registration tokens and reads every environment's kubeconfig;
* a **project API token** (the kubeconfig's) -- the administrator of that environment;
* a **node token** (handed out at registration) -- the kubelet's powers and no more, as the
  Node authorizer + NodeRestriction admission give them (``node_allows``): reads of what nodes
  read, Secrets and ConfigMaps only when a pod bound to the node uses them, writes only to its
  own Node, Lease, exec results and the pods bound to it, Events;
* a **ServiceAccount token** -- RBAC (rbac.py). What pods get is a *bound*
  token, TokenRequest-style (``POST .../serviceaccounts/<sa>/token``, ``issue_bound_token``): an
  HMAC-signed claim set naming the pod it was made for, an audience and an expiry, valid only
  while that pod (same uid) exists -- deleting the pod revokes it. The node agent requests one per
  pod (NodeRestriction: only for pods bound to it, as their own ServiceAccount) and renews it
  before it expires. The legacy ``<sa>-token`` Secret still authenticates, for clients that
  mount it explicitly;
* none -- anonymous: health, version, discovery, the readiness dashboard, node registration
  (its token is in the URL) and nothing else (401).

Tokens resolve through one dict rebuilt only when projects, node secrets or Secrets change
(``Store.version``), not a scan of them per request.
"""
from __future__ import annotations

import base64
import os
import re
from pathlib import Path

from ..utils.fsutil import atomic_write
from ..utils.ids import token_hex
from .httpserver import HttpError, Request

ADMIN_TOKEN_FILE = "admin-token"
SIGNING_KEY_FILE = "sa-signing-key"
BOUND_PREFIX = "tk8sb."
# audiences this API server accepts in a bound token (TokenRequest's default is the first)
API_AUDIENCES = ("https://kubernetes.default.svc.cluster.local", "https://kubernetes.default.svc", "tk8s")
BOUND_TTL_MIN_S, BOUND_TTL_MAX_S, BOUND_TTL_DEFAULT_S = 600, 7 * 86400, 3600
# kinds a node reads in full, as the kubelet's system:node role does
_NODE_READABLE = frozenset({"nodes", "pods", "services", "endpoints", "endpointslices", "runtimeclasses", "csinodes"})
_NS_RE = re.compile(r"^[a-z0-9]([-a-z0-9]{0,61}[a-z0-9])?$")
# store kinds whose names and contents are credentials or other callers' data: never in the change
# feed of a node or ServiceAccount token
_PRIVATE_KINDS = frozenset({"secrets", "kv", "nodesecrets", "registrationtokens", "projects", "projecttemplates",
                            "serviceaccounts"})

# (method, path) anyone may call: liveness, version, discovery, node registration (token-gated
# by its URL), the Rancher template list, and the dashboard (it shows anonymous callers only the
# node table the readiness oracle of setup.sh:66-68 needs).
_K8S = r"(/r/projects/[^/]+/kubernetes)?"
PUBLIC = [
    ("GET", re.compile(r"^/(ping|healthz|readyz|livez)?/?$")),
    ("GET", re.compile(r"^/version/?$")),
    ("GET", re.compile(r"^/v2-beta/projectTemplates/?$")),
    ("GET", re.compile(r"^/v1/scripts/[^/]+$")),
    ("POST", re.compile(r"^/v1/scripts/[^/]+$")),
    ("GET", re.compile(r"^/r/projects/[^/]+/kubernetes-dashboard:9090/?$")),
    ("GET", re.compile(r"^" + _K8S + r"/(api|apis|api/v1|apis/[^/]+|apis/[^/]+/[^/]+|openapi/v3(/.*)?)/?$")),
    ("POST", re.compile(r"^" + _K8S + r"/apis/authorization\.k8s\.io/v1/selfsubjectaccessreviews$")),
]


def is_public(method: str, path: str) -> bool:
    m = "GET" if method == "HEAD" else method
    return any(m == pm and rx.match(path) for pm, rx in PUBLIC)


def load_admin_token(state_dir: Path | None) -> str:
    """``$TK8S_ADMIN_TOKEN``, else ``<state_dir>/admin-token`` (created 0600 on first start),
    else a fresh one for this process only."""
    env = os.environ.get("TK8S_ADMIN_TOKEN", "").strip()
    if env:
        return env
    if state_dir is None:
        return token_hex(24)
    p = Path(state_dir) / ADMIN_TOKEN_FILE
    try:
        tok = p.read_text().strip()
        if tok:
            return tok
    except OSError:
        pass
    tok = token_hex(24)
    atomic_write(p, tok + "\n", mode=0o600)
    return tok


def load_signing_key(state_dir: Path | None) -> bytes:
    """The key bound ServiceAccount tokens are signed with: ``<state_dir>/sa-signing-key`` (0600,
    made on first start, so tokens survive a control-plane restart), else one for this process."""
    if state_dir is None:
        return token_hex(32).encode()
    p = Path(state_dir) / SIGNING_KEY_FILE
    try:
        k = p.read_text().strip()
        if k:
            return k.encode()
    except OSError:
        pass
    k = token_hex(32)
    atomic_write(p, k + "\n", mode=0o600)
    return k.encode()


def _b64(b: bytes) -> str:
    return base64.urlsafe_b64encode(b).rstrip(b"=").decode()


def _unb64(s: str) -> bytes:
    return base64.urlsafe_b64decode(s + "=" * (-len(s) % 4))


def pod_job(pod: dict) -> str | None:
    """The Job that owns a pod (its controller ownerReference), if any."""
    for r in (pod.get("metadata") or {}).get("ownerReferences") or []:
        if r.get("kind") == "Job":
            return r.get("name")
    return None


def _pod_refs(pod: dict, kind: str) -> set[str]:
    """Names of the Secrets (``kind`` "secrets") or ConfigMaps a pod's kubelet must read."""
    spec = pod.get("spec") or {}
    out: set[str] = set()
    vol_key, ref_key, env_key = (("secret", "secretRef", "secretKeyRef") if kind == "secrets"
                                 else ("configMap", "configMapRef", "configMapKeyRef"))
    for v in spec.get("volumes") or []:
        src = v.get(vol_key) or {}
        name = src.get("secretName") if kind == "secrets" else src.get("name")
        if name:
            out.add(name)
        for s in (v.get("projected") or {}).get("sources") or []:
            if (s.get(vol_key) or {}).get("name"):
                out.add(s[vol_key]["name"])
    for c in (spec.get("containers") or []) + (spec.get("initContainers") or []):
        for e in c.get("envFrom") or []:
            if (e.get(ref_key) or {}).get("name"):
                out.add(e[ref_key]["name"])
        for e in c.get("env") or []:
            ref = (e.get("valueFrom") or {}).get(env_key) or {}
            if ref.get("name"):
                out.add(ref["name"])
    if kind == "secrets":
        out |= {s.get("name") for s in spec.get("imagePullSecrets") or [] if s.get("name")}
        if spec.get("automountServiceAccountToken") is not False:
            out.add(f"{spec.get('serviceAccountName') or spec.get('serviceAccount') or 'default'}-token")
    return out


class Authentication:
    # ---- tokens --------------------------------------------------------------------------
    def _tokens(self) -> dict[str, tuple]:
        """token -> ("admin", pid|None) | ("node", pid, name) | ("sa", pid, ns, name)."""
        ver = self.store.version("projects", "nodesecrets", "secrets")
        if getattr(self, "_tok_ver", None) != ver:
            idx: dict[str, tuple] = {}
            for s in self.store.list("secrets", lambda o: o.get("type") == "kubernetes.io/service-account-token"):
                t = (s.get("data") or {}).get("token")
                sa = (s["metadata"].get("annotations") or {}).get("kubernetes.io/service-account.name")
                if t and sa:
                    idx[base64.b64decode(t).decode(errors="replace")] = ("sa", s.get("_project"), s["metadata"]["namespace"], sa)
            for n in self.store.list("nodesecrets"):
                if n.get("nodeToken"):
                    idx[n["nodeToken"]] = ("node", n.get("_project"), n["metadata"]["name"])
            for p in self.store.list("projects"):
                if p.get("apiToken"):
                    idx[p["apiToken"]] = ("admin", p["id"])
            idx[self.admin_token] = ("admin", None)
            self._tok_idx, self._tok_ver = idx, ver
        return self._tok_idx

    # ---- bound ServiceAccount tokens (TokenRequest) -------------------------------------------
    def _signing_key(self) -> bytes:
        k = getattr(self, "_sa_key", None)
        if k is None:
            k = self._sa_key = load_signing_key(getattr(self, "state_dir", None))
        return k

    def issue_bound_token(self, pid: str | None, ns: str, sa: str, pod: dict | None, audiences: list[str],
                          ttl: float) -> tuple[str, float]:
        """A token for ServiceAccount ``ns/sa`` of project ``pid``, bound to ``pod`` (its name and
        uid; None: unbound, it only expires), for ``audiences``, valid ``ttl`` s (clamped to
        10 min .. 7 days). Returns (token, expiry unix time)."""
        import hashlib
        import hmac
        import json
        import time

        ttl = min(max(float(ttl), BOUND_TTL_MIN_S), BOUND_TTL_MAX_S)
        exp = time.time() + ttl
        claims = {"p": pid, "ns": ns, "sa": sa, "aud": list(audiences), "exp": round(exp, 3), "jti": token_hex(8)}
        if pod is not None:
            claims.update(pod=pod["metadata"]["name"], uid=pod["metadata"].get("uid", ""))
        body = _b64(json.dumps(claims, separators=(",", ":"), sort_keys=True).encode())
        sig = _b64(hmac.new(self._signing_key(), body.encode(), hashlib.sha256).digest())
        return f"{BOUND_PREFIX}{body}.{sig}", exp

    def _bound(self, tok: str) -> tuple | None:
        """("sa", pid, ns, sa, {"pod", "uid", "job"}) for a valid bound token: signature, expiry,
        audience, and -- when bound to a pod -- that pod still exists with the same uid."""
        import hashlib
        import hmac
        import json
        import time

        from .objects import _key

        try:
            body, sig = tok[len(BOUND_PREFIX):].split(".", 1)
            want = _b64(hmac.new(self._signing_key(), body.encode(), hashlib.sha256).digest())
            if not hmac.compare_digest(want, sig):
                return None
            c = json.loads(_unb64(body))
        except (ValueError, TypeError, UnicodeDecodeError):
            return None
        if not isinstance(c, dict) or float(c.get("exp") or 0) <= time.time():
            return None
        if not set(c.get("aud") or []) & set(API_AUDIENCES):
            return None
        bound = {"pod": None, "uid": None, "job": None}
        if c.get("pod"):
            pod = self.store.get("pods", _key(c.get("p"), c.get("ns"), c["pod"]))
            if pod is None or pod["metadata"].get("uid", "") != c.get("uid", "") or \
                    pod["metadata"].get("deletionTimestamp"):
                return None  # the pod it was made for is gone (or going): revoked
            bound = {"pod": c["pod"], "uid": c.get("uid"), "job": pod_job(pod)}
        return ("sa", c.get("p"), c.get("ns"), c.get("sa"), bound)

    def _lookup(self, tok: str | None) -> tuple | None:
        """Any token this server knows: admin, project, node, legacy ServiceAccount, or bound."""
        if not tok:
            return None
        hit = self._tokens().get(tok)
        if hit is None and tok.startswith(BOUND_PREFIX):
            hit = self._bound(tok)
        return hit

    def _identity(self, p: str | None, tok: str | None) -> str | None:
        """``admin`` (the server admin token, or project ``p``'s API token), ``node:<name>``,
        ``sa:<ns>:<name>`` -- a node or ServiceAccount of project ``p`` -- or None."""
        hit = self._lookup(tok)
        if hit is None:
            return None
        if hit[0] == "admin":
            return "admin" if hit[1] is None or p is None or hit[1] == p else None
        if p is not None and hit[1] != p:
            return None
        return f"node:{hit[2]}" if hit[0] == "node" else f"sa:{hit[2]}:{hit[3]}"

    def _server_admin(self, req: Request) -> bool:
        return bool(req.bearer) and req.bearer == self.admin_token

    def _authenticate(self, req: Request) -> None:
        """The gate in front of every route: a public path, or a token this server knows."""
        if is_public(req.method, req.path):
            return
        if self._lookup(req.bearer) is not None:
            return
        raise HttpError(401, "Unauthorized: this request needs a bearer token "
                             "(the kubeconfig's, a ServiceAccount's, a node's or the server admin token)")

    # ---- the side channels: KV, /v1/events, /v1/cluster/*, /metrics, /v2-beta/projects ------
    # In the reference every environment is its own Rancher project and hosts join it with a
    # registration token bound to its projectId (ranchermaster/tasks/main.yml:37-49,
    # rancherhost/tasks/main.yml:11-17). The control plane's own side channels keep that scope:
    # a token acts inside its environment -- and a ServiceAccount's inside its namespace -- only.
    def _caller(self, req: Request) -> tuple:
        hit = self._lookup(req.bearer)
        if hit is None:
            raise HttpError(401, "missing or invalid bearer token")
        return hit

    def _caller_project(self, req: Request, asked: str | None) -> dict:
        """The environment a side-channel request acts in: any one the server admin asks for
        (the oldest by default), otherwise the caller's own -- naming another one is 403."""
        hit = self._caller(req)
        if hit[0] == "admin" and hit[1] is None:
            return self.project(asked)
        if asked not in (None, "", "default", hit[1]):
            raise HttpError(403, f"this token belongs to environment {hit[1]}, not {asked}")
        return self.project(hit[1])

    def _require_project_admin(self, req: Request, pid: str | None = None) -> tuple:
        """The server admin token, or an environment's API token (of ``pid`` when given):
        node and ServiceAccount tokens get 403."""
        hit = self._caller(req)
        if hit[0] != "admin" or (pid is not None and hit[1] not in (None, pid)):
            raise HttpError(403, "this needs the server admin token or the environment's API token")
        return hit

    def kv_key(self, req: Request, key: str) -> str:
        """The store key of KV ``key`` for this caller: ``<project>/<namespace>/<key>``, or
        ``<project>/<namespace>/job:<job>/<key>`` in a Job's own keyspace.

        * a pod's bound token: a pod owned by a Job reaches its Job's keyspace
          only -- the RCCL unique id or torch address of ``rccl-allreduce-X`` is out of reach of
          every other pod, same namespace and ServiceAccount included; a pod no Job owns gets its
          namespace's shared keys, as a legacy ServiceAccount token does;
        * a legacy ServiceAccount token: its own environment and namespace (``?namespace=`` may only
          repeat it), so a pod reaches its own namespace's keys and nothing else;
        * a node token: none -- the keys are the workloads' rendezvous (RCCL unique ids, torch
          addresses), which no kubelet reads or writes, and the pods of one namespace run on many
          nodes, so a node could not be held to its own pods' keys by namespace;
        * an environment's API token: its environment, any namespace (``?job=`` a Job's
          keyspace); the server admin token: ``?project=`` (default: the oldest environment), any
          namespace."""
        if not key or len(key) > 512 or "\0" in key:
            raise HttpError(422, "a KV key is 1-512 characters")
        hit = self._caller(req)
        ns = req.q("namespace") or None
        if ns is not None and not _NS_RE.match(ns):
            raise HttpError(422, f"invalid namespace {ns!r}")
        job = req.q("job") or None
        if job is not None and not _NS_RE.match(job):
            raise HttpError(422, f"invalid job name {job!r}")
        if hit[0] == "sa":
            if ns not in (None, hit[2]):
                raise HttpError(403, f"a ServiceAccount of namespace {hit[2]} cannot reach the keys of {ns}")
            own = (hit[4] if len(hit) > 4 else {}).get("job")
            if job not in (None, own):
                raise HttpError(403, f"this pod's token reaches the keys of {'job ' + own if own else 'its namespace'}, "
                                     f"not of job {job}")
            return f"{hit[1]}/{hit[2]}/job:{own}/{key}" if own else f"{hit[1]}/{hit[2]}/{key}"
        ns = ns or "default"
        if hit[0] == "node":
            raise HttpError(403, f"node {hit[2]}: the KV store holds the workloads' rendezvous keys, "
                                 "which nodes have no access to")
        try:
            pid = self._caller_project(req, req.q("project"))["id"]
        except HttpError as e:
            if e.status != 404 or hit[1] is not None:
                raise
            pid = "-"  # the server admin before any environment exists
        return f"{pid}/{ns}/job:{job}/{key}" if job else f"{pid}/{ns}/{key}"

    def event_filter(self, req: Request):
        """What of the store's change feed (``/v1/events``) the caller may see: everything for the
        server admin, its environment for an API token, for a node its environment minus the
        credential-bearing kinds, for a ServiceAccount its namespace minus those."""
        hit = self._caller(req)
        if hit[0] == "admin":
            return (lambda kind, o: True) if hit[1] is None else (lambda kind, o: o.get("_project") == hit[1])
        pid = hit[1]
        if hit[0] == "node":
            return lambda kind, o: o.get("_project") == pid and kind not in _PRIVATE_KINDS
        ns = hit[2]
        return lambda kind, o: (o.get("_project") == pid and (o.get("metadata") or {}).get("namespace") == ns
                                and kind not in _PRIVATE_KINDS)

    def _require_admin(self, req: Request, pid: str | None) -> None:
        """The server admin token, or the API token of project ``pid``."""
        hit = self._lookup(req.bearer)
        if hit is None or hit[0] != "admin" or (hit[1] is not None and hit[1] != pid):
            raise HttpError(403 if hit else 401, "this needs the server admin token or the environment's API token")

    # ---- the Node authorizer + NodeRestriction ---------------------------------------------
    def node_allows(self, node: str, p: str | None, info) -> bool:
        """May node ``node`` (of project ``p``) do ``info`` (rbac.RequestInfo)?"""
        res = info.resource.split("/")[0]
        sub = info.resource.partition("/")[2]
        read = info.verb in ("get", "list", "watch")
        if res in ("secrets", "configmaps"):
            if info.verb != "get" or not info.name:
                return False
            return any(info.name in _pod_refs(o, res) for o in self._node_pods(node, p, info.namespace))
        if res == "nodes":
            if sub in ("execs",) or (not read and info.verb in ("update", "patch")):
                return info.name == node
            return read and not sub
        if res == "pods":
            if sub in ("log", "exec", "attach", "portforward", "eviction"):
                return False
            if read and not sub:
                return True
            if sub == "status" and info.verb in ("update", "patch", "get"):
                return self._bound_to(node, p, info.namespace, info.name)
            if info.verb == "delete" and not sub:
                return self._bound_to(node, p, info.namespace, info.name)
            return False
        if res == "leases":
            return read or info.name == node
        if res == "serviceaccounts" and sub == "token":
            # TokenRequest: the handler holds a node to pods bound to it, as their own
            # ServiceAccount (NodeRestriction; k8s_api.h_token_request)
            return info.verb == "create"
        if res == "events":
            return info.verb in ("create", "patch", "update") or read
        # what the kubelet's system:node role reads, and no more: no workload
        # specs, no RBAC; the objects of its own pods only (PVCs, their PVs, the Jobs that own them)
        if res in _NODE_READABLE:
            return read and not sub
        if res in ("persistentvolumeclaims", "jobs"):
            if info.verb != "get" or not info.name or sub:
                return False
            return any(info.name in self._pod_objects(o, res) for o in self._node_pods(node, p, info.namespace))
        if res == "persistentvolumes":
            if info.verb != "get" or not info.name or sub:
                return False
            return info.name in self._node_pvs(node, p)
        return False

    @staticmethod
    def _pod_objects(pod: dict, res: str) -> set[str]:
        """The PVCs a pod mounts, or the Job that owns it."""
        if res == "jobs":
            return {r.get("name") for r in pod["metadata"].get("ownerReferences") or [] if r.get("kind") == "Job"}
        return {(v.get("persistentVolumeClaim") or {}).get("claimName") for v in (pod.get("spec") or {}).get("volumes") or []
                if v.get("persistentVolumeClaim")}

    def _node_pvs(self, node: str, p: str | None) -> set[str]:
        """The PersistentVolumes bound to the claims of the node's pods."""
        from .objects import _key

        out = set()
        for o in self.store.list("pods", lambda o: o["spec"].get("nodeName") == node
                                 and (p is None or o.get("_project") == p)):
            ns = o["metadata"].get("namespace", "default")
            for claim in self._pod_objects(o, "persistentvolumeclaims"):
                pvc = self.store.get("persistentvolumeclaims", _key(o.get("_project"), ns, claim))
                if pvc and (pvc.get("spec") or {}).get("volumeName"):
                    out.add(pvc["spec"]["volumeName"])
        return out

    def _node_pods(self, node: str, p: str | None, ns: str) -> list[dict]:
        return self.store.list("pods", lambda o: o["spec"].get("nodeName") == node
                               and o["metadata"].get("namespace") == ns and (p is None or o.get("_project") == p))

    def _bound_to(self, node: str, p: str | None, ns: str, name: str) -> bool:
        from .objects import _key

        if p is None:
            return False
        o = self.store.get("pods", _key(p, ns, name))
        return o is None or o["spec"].get("nodeName") == node  # None: the handler answers 404
