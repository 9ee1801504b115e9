"""tk8s control plane: Rancher-1.x-style environment API + a Kubernetes API subset.

Replaces the `rancher/server:stable` container (ansible/roles/ranchermaster/tasks/main.yml:6-13)
and the Rancher-managed Kubernetes control plane it deployed onto the hosts (SURVEY.md §2.4
P1/P3). One process serves:

Rancher-compatible REST (what the reference's Ansible roles call):
  GET  /v2-beta/projectTemplates?name=kubernetes        ranchermaster/tasks/main.yml:29-35
  POST /v2-beta/projects              -> 201 {id}        ranchermaster/tasks/main.yml:37-49
  POST /v1/registrationtokens?projectId=ID -> 201 {links.self}   rancherhost/tasks/main.yml:11-17
  GET  /v1/registrationtokens/ID      -> {registrationUrl}        rancherhost/tasks/main.yml:19-24
  GET/POST /v1/scripts/TOKEN          agent bootstrap / node registration (rancher/agent join)
  GET  /r/projects/ENV/kubernetes-dashboard:9090/   the readiness oracle of setup.sh:66
  GET  /env/ENV/kubernetes/kubectl    kubeconfig  (setup.sh:89)
  GET  /env/ENV/infra/containers      what runs where (setup.sh:53)

Kubernetes subset under /r/projects/ENV/kubernetes and /api, /apis (default project):
  nodes (leases, Ready/NotReady), pods, daemonsets, jobs (Indexed), deployments, services,
  events; watch = long-poll batches (?watch=1&resourceVersion=N&timeoutSeconds=T).
  Extended resource ``amd.com/gpu`` is scheduled like the AMD k8s-device-plugin exposes it.

Extras: /v1/kv/KEY (rendezvous store, e.g. RCCL unique ids), /v1/cluster/wait (event-driven
readiness, replaces the unbounded 15 s polling loop of setup.sh:59-85), /metrics.

Everything runs on one asyncio loop; the store is the single source of truth.
"""
from __future__ import annotations

import argparse
import asyncio
import copy
import html
import json
import os
import secrets
import signal
import sys
import time
from pathlib import Path

from ..utils.net import host_port
from ..utils.trace import trace
from .httpserver import HttpError, HttpServer, Request, Response, Router
from .store import Store, now_iso

GPU = "amd.com/gpu"
VALIDATION_LABEL = "tk8s.amd.com/validation"
TERMINAL = ("Succeeded", "Failed")
KIND_GROUPS = (("pods", "/api/v1"), ("services", "/api/v1"), ("events", "/api/v1"), ("configmaps", "/api/v1"),
               ("secrets", "/api/v1"), ("daemonsets", "/apis/apps/v1"), ("deployments", "/apis/apps/v1"),
               ("jobs", "/apis/batch/v1"), ("ingresses", "/apis/networking.k8s.io/v1"))


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


def _set_ready(node: dict, message: str = "tk8s agent heartbeating") -> bool:
    """Ready follows the heartbeat, unless the node's xGMI links failed the pre-Ready check
    (xgmi.py): then it stays NotReady with that reason while the agent is alive."""
    x = _cond(node, "XGMILinksHealthy")
    if x and x["status"] == "False":
        return _set_cond(node, "Ready", "False", "XGMILinkDegraded", x.get("message", ""))
    return _set_cond(node, "Ready", "True", "AgentReady", message)


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
    """``pod-template-hash`` of a Deployment's pod template (names its ReplicaSet generation)."""
    import hashlib  # off the control plane's start-up path (it is on the bring-up's)

    return hashlib.sha1(json.dumps(template, sort_keys=True, separators=(",", ":")).encode()).hexdigest()[:10]


GPU_VISIBILITY = "tk8s.amd.com/gpu-visibility"


def _admit_gpu_visibility(kind: str, ns: str, body: dict) -> None:
    """Admission: ``gpu-visibility: node`` lets a pod's runtime see every GPU of its node (the RCCL
    fabric Job's ranks need it for xGMI peer-to-peer). Only kube-system Jobs may ask for it; a pod
    cannot ask for it directly (the agent re-checks: kube-system pods owned by a Job)."""
    if kind == "pods":
        ann = (body.get("metadata") or {}).get("annotations") or {}
        if ann.get(GPU_VISIBILITY) == "node":
            raise HttpError(403, f'pods is forbidden: annotation {GPU_VISIBILITY}: node is reserved for '
                                 'kube-system Jobs')
    elif kind in ("jobs", "daemonsets", "deployments"):
        ann = ((body.get("spec") or {}).get("template") or {}).get("metadata", {}).get("annotations") or {}
        if ann.get(GPU_VISIBILITY) == "node" and (kind != "jobs" or ns != "kube-system"):
            raise HttpError(403, f'{kind} is forbidden: annotation {GPU_VISIBILITY}: node is reserved for '
                                 'kube-system Jobs')


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


class ControlPlane:
    def __init__(self, host: str, port: int, state_dir: str | None = None, node_grace: float = 5.0,
                 advertise: str | None = None, dns_port: int | None = None, ingress_port: int | None = None):
        self.host, self.port = host, port
        self.advertise = advertise
        self.state_dir = Path(state_dir) if state_dir else None
        self.node_grace = node_grace
        self.store = Store()
        self.router = Router()
        self.http = HttpServer(self.router, on_error=self._log_error)
        self.leases: dict[str, float] = {}   # node key -> monotonic time of last heartbeat
        self.started = time.time()
        self._stop = None
        self._seq = 0
        self._reconciling = False
        self._again = False
        from .proxy import ServiceProxy

        from .ingress import IngressController

        self.proxy = ServiceProxy(self._endpoints, log=lambda m: self._log_error(m + "\n"))
        self.ingress = IngressController(self._ingress_routes, self._endpoints, log=lambda m: self._log_error(m + "\n"))
        self.dns_port = host_port(53) if dns_port is None else dns_port          # 0 disables
        self.ingress_port = host_port(80) if ingress_port is None else ingress_port
        self._routes()

    # ---- utilities --------------------------------------------------------------------
    def _log_error(self, text: str) -> None:
        sys.stderr.write(text)
        sys.stderr.flush()

    @property
    def base(self) -> str:
        return f"http://{self.advertise or self.host}:{self.port}"

    def _next_id(self, prefix: str) -> str:
        self._seq += 1
        return f"{prefix}{self._seq}"

    def _event(self, project: str, ns: str, involved: dict, reason: str, message: str, etype: str = "Normal") -> None:
        self._seq += 1
        name = f"{involved.get('name', 'x')}.{self._seq:x}"
        self.store.put("events", _key(project, ns, name), {
            "kind": "Event", "metadata": {"name": name, "namespace": ns}, "_project": project,
            "involvedObject": involved, "reason": reason, "message": message, "type": etype,
            "firstTimestamp": now_iso(), "count": 1,
        })
        evs = self.store.keys("events")
        if len(evs) > 5000:
            for k in evs[: len(evs) - 5000]:
                self.store.delete("events", k)

    def project(self, pid: str | None) -> dict:
        if pid in (None, "", "default"):
            projects = self.store.list("projects")
            if not projects:
                raise HttpError(404, "no project/environment exists yet")
            return sorted(projects, key=lambda p: p["created_seq"])[0]
        p = self.store.get("projects", pid)
        if p is None:
            raise HttpError(404, f"project {pid} not found")
        return p

    def _auth(self, req: Request, project: dict) -> None:
        tok = req.bearer
        if req.method in ("GET", "HEAD"):
            return
        valid = {project.get("apiToken")}
        if tok in valid:
            return
        # node tokens may update their own node / pods
        if tok and any(n.get("nodeToken") == tok for n in self.store.list("nodesecrets")):
            return
        raise HttpError(401, "missing or invalid bearer token")

    # ---- routes -----------------------------------------------------------------------
    def _routes(self) -> None:
        r = self.router
        r.add("GET", r"/(ping|healthz)?", self.h_ping)
        r.add("GET", r"/version", self.h_version)
        r.add("GET", r"/metrics", self.h_metrics)
        # Rancher-style API
        r.add("GET", r"/v2-beta/projectTemplates", self.h_templates)
        r.add("GET", r"/v2-beta/projects", self.h_projects)
        r.add("POST", r"/v2-beta/projects", self.h_project_create)
        r.add("GET", r"/v2-beta/projects/(?P<pid>[^/]+)", self.h_project_get)
        r.add("DELETE", r"/v2-beta/projects/(?P<pid>[^/]+)", self.h_project_delete)
        r.add("POST", r"/v1/registrationtokens", self.h_token_create)
        r.add("GET", r"/v1/registrationtokens/(?P<tid>[^/]+)", self.h_token_get)
        r.add("GET", r"/v1/scripts/(?P<token>[^/]+)", self.h_script)
        r.add("POST", r"/v1/scripts/(?P<token>[^/]+)", self.h_register)
        r.add("GET", r"/r/projects/(?P<pid>[^/]+)/kubernetes-dashboard:9090/?", self.h_dashboard)
        r.add("POST", r"/r/projects/(?P<pid>[^/]+)/kubernetes-dashboard:9090/api/v1/appdeployment", self.h_app_deploy)
        r.add("GET", r"/env/(?P<pid>[^/]+)/kubernetes/kubectl", self.h_kubeconfig)
        r.add("GET", r"/env/(?P<pid>[^/]+)/infra/containers", self.h_containers)
        # KV + cluster readiness
        r.add("GET", r"/v1/kv/(?P<key>.+)", self.h_kv_get)
        r.add("PUT", r"/v1/kv/(?P<key>.+)", self.h_kv_put)
        r.add("POST", r"/v1/kv/(?P<key>.+)", self.h_kv_put)
        r.add("DELETE", r"/v1/kv/(?P<key>.+)", self.h_kv_delete)
        r.add("GET", r"/v1/cluster/status", self.h_cluster_status)
        r.add("GET", r"/v1/cluster/wait", self.h_cluster_wait)
        r.add("GET", r"/v1/events", self.h_cp_events)
        # Kubernetes subset, with and without the Rancher project prefix
        for pre in (r"/r/projects/(?P<pid>[^/]+)/kubernetes", r""):
            def add(method, path, h, pre=pre):
                r.add(method, pre + path, h)
            add("GET", r"/api/v1/nodes", self.h_nodes)
            add("GET", r"/api/v1/nodes/(?P<name>[^/]+)", self.h_node_get)
            add("PUT", r"/api/v1/nodes/(?P<name>[^/]+)/status", self.h_node_status)
            add("PATCH", r"/api/v1/nodes/(?P<name>[^/]+)", self.h_node_patch)
            add("DELETE", r"/api/v1/nodes/(?P<name>[^/]+)", self.h_node_delete)
            add("GET", r"/api/v1/namespaces", self.h_namespaces)
            add("GET", r"/api/v1/pods", self.h_pods)
            for kind, grp in KIND_GROUPS:
                add("GET", grp + rf"/namespaces/(?P<ns>[^/]+)/{kind}", self._lister(kind))
                add("POST", grp + rf"/namespaces/(?P<ns>[^/]+)/{kind}", self._creator(kind))
                add("GET", grp + rf"/namespaces/(?P<ns>[^/]+)/{kind}/(?P<name>[^/]+)", self._getter(kind))
                add("PUT", grp + rf"/namespaces/(?P<ns>[^/]+)/{kind}/(?P<name>[^/]+)", self._replacer(kind, False))
                add("PATCH", grp + rf"/namespaces/(?P<ns>[^/]+)/{kind}/(?P<name>[^/]+)", self._replacer(kind, True))
                add("DELETE", grp + rf"/namespaces/(?P<ns>[^/]+)/{kind}/(?P<name>[^/]+)", self._deleter(kind))
                add("GET", grp + rf"/{kind}", self._lister(kind, all_ns=True))
            for method in ("GET", "PUT", "PATCH"):
                add(method, r"/apis/apps/v1/namespaces/(?P<ns>[^/]+)/deployments/(?P<name>[^/]+)/scale", self.h_scale)
            add("PUT", r"/api/v1/namespaces/(?P<ns>[^/]+)/pods/(?P<name>[^/]+)/status", self.h_pod_status)
            add("GET", r"/api/v1/namespaces/(?P<ns>[^/]+)/pods/(?P<name>[^/]+)/log", self.h_pod_log)
            add("POST", r"/api/v1/namespaces/(?P<ns>[^/]+)/pods/(?P<name>[^/]+)/exec", self.h_pod_exec)
            add("GET", r"/api/v1/nodes/(?P<node>[^/]+)/execs", self.h_node_execs)
            add("PUT", r"/api/v1/nodes/(?P<node>[^/]+)/execs/(?P<xid>[^/]+)", self.h_exec_result)

    # ---- misc handlers ---------------------------------------------------------------
    async def h_ping(self, req: Request, **_):
        return Response(200, "pong")

    async def h_version(self, req: Request):
        from .. import __version__

        return {"major": "1", "minor": "30", "gitVersion": f"v1.30.0-tk8s{__version__}", "platform": "linux/amd64",
                "tk8sVersion": __version__}

    async def h_metrics(self, req: Request):
        lines = []
        for p in self.store.list("projects"):
            pid = p["id"]
            s = self.summary(pid)
            lab = f'project="{pid}"'
            lines += [f"tk8s_nodes{{{lab}}} {s['nodes']}", f"tk8s_nodes_ready{{{lab}}} {s['nodes_ready']}",
                      f"tk8s_nodes_validated{{{lab}}} {s['nodes_validated']}",
                      f"tk8s_gpus_capacity{{{lab}}} {s['gpus_capacity']}",
                      f"tk8s_gpus_allocatable{{{lab}}} {s['gpus_allocatable']}",
                      f"tk8s_gpus_in_use{{{lab}}} {s['gpus_in_use']}"]
            for phase, n in s["pods_by_phase"].items():
                lines.append(f'tk8s_pods{{{lab},phase="{phase}"}} {n}')
        now = time.monotonic()
        for k, t in self.leases.items():
            lines.append(f'tk8s_node_heartbeat_age_seconds{{node="{k}"}} {now - t:.3f}')
        lines.append(f"tk8s_store_resource_version {self.store.rv}")
        return Response(200, "\n".join(lines) + "\n", content_type="text/plain; version=0.0.4")

    # ---- Rancher API -----------------------------------------------------------------
    def _ensure_templates(self) -> None:
        if not self.store.list("projecttemplates"):
            for i, (name, desc) in enumerate([("cattle", "Default Cattle template"),
                                              ("kubernetes", "Kubernetes on MI355X (tk8s control plane)")], 1):
                tid = f"1pt{i}"
                self.store.put("projecttemplates", tid, {"id": tid, "type": "projectTemplate", "name": name,
                                                          "description": desc, "isPublic": True,
                                                          "metadata": {"name": name}})

    async def h_templates(self, req: Request):
        self._ensure_templates()
        name = req.q("name")
        data = [t for t in self.store.list("projecttemplates") if name is None or t["name"] == name]
        return {"type": "collection", "resourceType": "projectTemplate", "data": data}

    async def h_projects(self, req: Request):
        return {"type": "collection", "resourceType": "project", "data": [self._public_project(p) for p in self.store.list("projects")]}

    def _public_project(self, p: dict) -> dict:
        return {k: v for k, v in p.items() if k not in ("apiToken",)}

    async def h_project_create(self, req: Request):
        self._ensure_templates()
        body = req.json()
        name = str(body.get("name") or "").strip()
        tid = body.get("projectTemplateId")
        if not name:
            raise HttpError(422, "name is required")
        tmpl = self.store.get("projecttemplates", str(tid))
        if tmpl is None:
            raise HttpError(422, f"projectTemplateId {tid!r} does not exist")
        pid = self._next_id("1a")
        self._seq += 1
        p = {"id": pid, "type": "project", "name": name, "description": body.get("description", ""),
             "projectTemplateId": tid, "orchestration": tmpl["name"], "state": "active",
             "allowSystemRole": bool(body.get("allowSystemRole", False)), "members": body.get("members", []),
             "virtualMachine": bool(body.get("virtualMachine", False)),
             "servicesPortRange": body.get("servicesPortRange"), "projectLinks": body.get("projectLinks", []),
             "created": now_iso(), "created_seq": self._seq, "apiToken": secrets.token_hex(16),
             "links": {"self": f"{self.base}/v2-beta/projects/{pid}"},
             "metadata": {"name": pid}}
        self.store.put("projects", pid, p)
        return Response(201, self._public_project(p))

    async def h_project_get(self, req: Request, pid: str):
        return self._public_project(self.project(pid))

    async def h_project_delete(self, req: Request, pid: str):
        p = self.project(pid)
        for kind in list(self.store.objs):
            for k in self.store.keys(kind):
                if k.startswith(pid + "/"):
                    self.store.delete(kind, k)
        self.store.delete("projects", p["id"])
        return {"id": pid, "state": "removed"}

    async def h_token_create(self, req: Request):
        pid = req.q("projectId") or req.json().get("projectId")
        p = self.project(pid)
        tid = self._next_id("1c")
        token = secrets.token_hex(20)
        t = {"id": tid, "type": "registrationToken", "projectId": p["id"], "token": token, "state": "active",
             "registrationUrl": f"{self.base}/v1/scripts/{token}",
             "command": f"python3 -m tritonk8ssupervisor_amd.agent --url {self.base}/v1/scripts/{token}",
             "links": {"self": f"{self.base}/v1/registrationtokens/{tid}"}, "metadata": {"name": tid}}
        self.store.put("registrationtokens", tid, t)
        return Response(201, {k: v for k, v in t.items() if k not in ("token", "registrationUrl", "command")})

    async def h_token_get(self, req: Request, tid: str):
        t = self.store.get("registrationtokens", tid)
        if t is None:
            raise HttpError(404, f"registration token {tid} not found")
        return t

    def _token(self, token: str) -> dict:
        for t in self.store.list("registrationtokens"):
            if t["token"] == token and t["state"] == "active":
                return t
        raise HttpError(403, "invalid registration token")

    async def h_script(self, req: Request, token: str):
        t = self._token(token)
        pid = t["projectId"]
        return {"projectId": pid, "apiUrl": self.base, "apiPrefix": f"/r/projects/{pid}/kubernetes",
                "heartbeatSeconds": max(0.2, self.node_grace / 5), "nodeGraceSeconds": self.node_grace}

    async def h_register(self, req: Request, token: str):
        t = self._token(token)
        pid = t["projectId"]
        body = req.json()
        name = str(body.get("name") or "").strip()
        if not name:
            raise HttpError(422, "node name is required")
        key = _key(pid, name)
        ntok = secrets.token_hex(16)
        gpus = body.get("devices", [])
        healthy = sum(1 for d in gpus if d.get("health", "Healthy") == "Healthy")
        cap = dict(body.get("capacity", {}))
        cap[GPU] = str(len(gpus))
        alloc = dict(cap)
        alloc[GPU] = str(healthy)
        old = self.store.get("nodes", key)
        cidr = (old or {}).get("spec", {}).get("podCIDR") or self._next_pod_cidr()
        node = {
            "kind": "Node", "apiVersion": "v1", "_project": pid,
            "metadata": {"name": name, "labels": {"kubernetes.io/hostname": name, "kubernetes.io/os": "linux",
                                                  **({"amd.com/gpu.family": "gfx950"} if gpus else {}),
                                                  **body.get("labels", {})},
                         "annotations": body.get("annotations", {})},
            "spec": {"unschedulable": False, "podCIDR": cidr},
            "status": {"capacity": cap, "allocatable": alloc, "devices": gpus,
                       "addresses": [{"type": "InternalIP", "address": body.get("ip", "")},
                                     {"type": "Hostname", "address": name}],
                       "nodeInfo": body.get("nodeInfo", {}), "conditions": []},
        }
        if old is not None and _cond(old, "XGMILinksHealthy"):  # a re-join keeps the link verdict
            node["status"]["conditions"].append(copy.deepcopy(_cond(old, "XGMILinksHealthy")))
        _set_ready(node, "tk8s agent registered and heartbeating")
        _set_cond(node, "AMDGPUValidated", "Unknown" if gpus else "True",
                  "Pending" if gpus else "NoGPUs", "validation pod not finished" if gpus else "")
        self.store.put("nodes", key, node)
        self.store.put("nodesecrets", key, {"metadata": {"name": name}, "nodeToken": ntok, "_project": pid})
        self.leases[key] = time.monotonic()
        self._event(pid, "default", {"kind": "Node", "name": name}, "RegisteredNode", f"Node {name} registered ({len(gpus)} GPU)")
        self.reconcile()
        trace("cp", f"node {name} registered")
        return Response(201, {"node": name, "nodeToken": ntok, "projectId": pid, "podCIDR": cidr,
                              "apiPrefix": f"/r/projects/{pid}/kubernetes",
                              "heartbeatSeconds": max(0.2, self.node_grace / 5)})

    async def h_dashboard(self, req: Request, pid: str):
        p = self.project(pid)
        s = self.summary(p["id"])
        if s["nodes_ready"] == 0:
            return Response(503, "Service Unavailable", content_type="text/plain")
        esc = html.escape
        rows = "".join(
            f"<tr><td>{esc(n['metadata']['name'])}</td><td>{'Ready' if node_ready(n) else 'NotReady'}</td>"
            f"<td>{n['status']['allocatable'].get(GPU, '0')}</td><td>{'yes' if node_validated(n) else 'no'}</td></tr>"
            for n in self.store.list("nodes", lambda n: self._in(p['id'], n)))
        deps = "".join(
            f"<tr><td>{esc(d['metadata']['namespace'])}</td><td>{esc(d['metadata']['name'])}</td>"
            f"<td>{d.get('status', {}).get('readyReplicas', 0)}/{d['spec'].get('replicas', 1)}</td>"
            f"<td>{esc(', '.join(c.get('image', '') or ' '.join(c.get('command', [])) for c in d['spec']['template']['spec']['containers']))}</td></tr>"
            for d in self.store.list("deployments", lambda o: self._in(p['id'], o)))
        svcs = "".join(
            f"<tr><td>{esc(o['metadata']['name'])}</td><td>{o['spec'].get('type')}</td><td>{o['spec'].get('clusterIP')}</td>"
            f"<td>{esc(','.join(i.get('ip', '') for i in o.get('status', {}).get('loadBalancer', {}).get('ingress', [])))}</td>"
            f"<td>{esc(','.join(str(x['port']) for x in o['spec'].get('ports', [])))}</td></tr>"
            for o in self.store.list("services", lambda o: self._in(p['id'], o)))
        body = (f"<html><head><title>Kubernetes Dashboard - {esc(p['name'])}</title></head><body>"
                f"<h1>kubernetes dashboard</h1><p>environment {esc(p['name'])} ({p['id']})</p>"
                f"<h2>Nodes</h2><table><tr><th>node</th><th>status</th><th>{GPU}</th><th>validated</th></tr>{rows}</table>"
                f"<h2>Deployments</h2><table><tr><th>namespace</th><th>name</th><th>ready</th><th>image</th></tr>{deps}</table>"
                f"<h2>Services</h2><table><tr><th>name</th><th>type</th><th>cluster IP</th><th>external IP</th>"
                f"<th>ports</th></tr>{svcs}</table>"
                "<h2>Deploy a containerized app</h2><form id='deploy'>"
                "<input name='name' placeholder='App name'> <input name='containerImage' placeholder='Container image'> "
                "<input name='replicas' value='1' size='3'> <input name='port' placeholder='Port'> "
                "<label><input type='checkbox' name='isExternal'> external</label> "
                f"<input name='gpus' value='0' size='3'> {GPU} <button>Deploy</button></form>"
                "<script>document.getElementById('deploy').addEventListener('submit', async (e) => {"
                "e.preventDefault(); const f = new FormData(e.target); const port = f.get('port');"
                "const body = {name: f.get('name'), containerImage: f.get('containerImage'),"
                " replicas: parseInt(f.get('replicas') || '1'), isExternal: f.get('isExternal') === 'on',"
                " gpuRequirement: parseInt(f.get('gpus') || '0'), namespace: 'default',"
                " portMappings: port ? [{port: parseInt(port), targetPort: parseInt(port), protocol: 'TCP'}] : []};"
                "await fetch('api/v1/appdeployment', {method: 'POST', headers: {'Content-Type': 'application/json'},"
                " body: JSON.stringify(body)}); location.reload(); });</script>"
                f"<pre>{esc(json.dumps(s, indent=1))}</pre></body></html>")
        return Response(200, body, content_type="text/html; charset=utf-8")

    async def h_app_deploy(self, req: Request, pid: str):
        """The dashboard's "Deploy a containerized app" form (kubernetes-dashboard
        ``POST api/v1/appdeployment``): a Deployment plus, with port mappings, a Service --
        how the reference's walkthrough launched Ghost (docs/detailed.md:261-283). Like the
        Rancher 1.x UI the reference used, the dashboard needs no API token."""
        import shlex

        p = self.project(pid)
        b = req.json()
        name = str(b.get("name") or "").strip()
        image = str(b.get("containerImage") or "").strip()
        if not name or not image:
            raise HttpError(422, "name and containerImage are required")
        ns = b.get("namespace") or "default"
        labels = {"app": name, **{str(lb["key"]): str(lb["value"]) for lb in b.get("labels") or []}}
        c = {"name": name, "image": image}
        if b.get("containerCommand"):
            c["command"] = shlex.split(str(b["containerCommand"]))
        if b.get("containerCommandArgs"):
            c["args"] = shlex.split(str(b["containerCommandArgs"]))
        if b.get("variables"):
            c["env"] = [{"name": str(v["name"]), "value": str(v.get("value", ""))} for v in b["variables"]]
        if int(b.get("gpuRequirement") or 0):
            c["resources"] = {"limits": {GPU: int(b["gpuRequirement"])}}
        ports = b.get("portMappings") or []
        if ports:
            c["ports"] = [{"containerPort": int(m["targetPort"]), "protocol": m.get("protocol", "TCP")} for m in ports]
        dep = {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": name, "labels": dict(labels)},
               "spec": {"replicas": int(b.get("replicas", 1)), "selector": {"matchLabels": {"app": name}},
                        "template": {"metadata": {"labels": labels}, "spec": {"containers": [c]}}}}
        out = {"deployment": self._strip(self.create(p["id"], "deployments", ns, dep))}
        if ports:
            svc = {"apiVersion": "v1", "kind": "Service", "metadata": {"name": name, "labels": {"app": name}},
                   "spec": {"type": "LoadBalancer" if b.get("isExternal") else "ClusterIP", "selector": {"app": name},
                            "ports": [{"name": f"{m.get('protocol', 'TCP').lower()}-{m['port']}-{m['targetPort']}",
                                       "port": int(m["port"]), "targetPort": int(m["targetPort"]),
                                       "protocol": m.get("protocol", "TCP")} for m in ports]}}
            out["service"] = self._strip(self.create(p["id"], "services", ns, svc))
        return Response(201, out)

    async def h_kubeconfig(self, req: Request, pid: str):
        p = self.project(pid)
        server = f"{self.base}/r/projects/{p['id']}/kubernetes"
        cfg = {"apiVersion": "v1", "kind": "Config", "current-context": p["name"].replace(" ", "-"),
               "clusters": [{"name": p["name"].replace(" ", "-"), "cluster": {"server": server}}],
               "users": [{"name": p["name"].replace(" ", "-"), "user": {"token": p["apiToken"]}}],
               "contexts": [{"name": p["name"].replace(" ", "-"),
                             "context": {"cluster": p["name"].replace(" ", "-"), "user": p["name"].replace(" ", "-")}}]}
        if req.q("format") == "json":
            return cfg
        import yaml  # local import: only this endpoint needs it

        return Response(200, yaml.safe_dump(cfg, sort_keys=False), content_type="text/yaml")

    async def h_containers(self, req: Request, pid: str):
        p = self.project(pid)
        pods = self.store.list("pods", lambda o: self._in(p["id"], o))
        return {"project": p["id"], "containers": [
            {"name": o["metadata"]["name"], "namespace": o["metadata"].get("namespace"),
             "node": o["spec"].get("nodeName"), "phase": o.get("status", {}).get("phase"),
             "gpus": o["metadata"].get("annotations", {}).get(GPU + "-ids")} for o in pods]}

    # ---- KV -------------------------------------------------------------------------
    async def h_kv_get(self, req: Request, key: str):
        wait = float(req.q("wait", "0") or 0)
        v = await self.store.wait_until(lambda: self.store.get("kv", key), min(wait, 120.0))
        if not v:
            raise HttpError(404, f"key {key} not found")
        return Response(200, v["value"], content_type="text/plain")

    async def h_kv_put(self, req: Request, key: str):
        self.store.put("kv", key, {"metadata": {"name": key}, "value": req.body.decode()})
        return Response(201, {"key": key})

    async def h_kv_delete(self, req: Request, key: str):
        self.store.delete("kv", key)
        return Response(200, {"key": key, "deleted": True})

    # ---- readiness -----------------------------------------------------------------------
    @staticmethod
    def _in(pid: str, obj: dict) -> bool:
        return obj.get("_project") == pid

    def summary(self, pid: str) -> dict:
        nodes = self.store.list("nodes", lambda n: self._in(pid, n))
        pods = self.store.list("pods", lambda o: self._in(pid, o))
        by_phase: dict[str, int] = {}
        for o in pods:
            ph = o.get("status", {}).get("phase", "Pending")
            by_phase[ph] = by_phase.get(ph, 0) + 1
        in_use = sum(pod_gpus(o) for o in pods if o.get("spec", {}).get("nodeName")
                     and o.get("status", {}).get("phase") not in TERMINAL)
        ready = [n for n in nodes if node_ready(n)]
        return {
            "project": pid, "nodes": len(nodes), "nodes_ready": len(ready),
            "nodes_validated": sum(1 for n in ready if node_validated(n)),
            "nodes_validation_failed": sum(1 for n in nodes if (_cond(n, "AMDGPUValidated") or {}).get("status") == "False"),
            "validation_failures": [{"node": n["metadata"]["name"], "reason": c.get("reason"),
                                     "message": (c.get("message") or "")[:300]}
                                    for n in nodes for c in [_cond(n, "AMDGPUValidated") or {}] if c.get("status") == "False"],
            "gpus_capacity": sum(int(n["status"]["capacity"].get(GPU, 0)) for n in nodes),
            "gpus_allocatable": sum(int(n["status"]["allocatable"].get(GPU, 0)) for n in ready),
            "gpus_in_use": in_use, "pods_by_phase": by_phase, "resourceVersion": self.store.rv,
            "node_names": sorted(n["metadata"]["name"] for n in nodes),
        }

    def _job_state(self, pid: str, ref: str | None) -> str | None:
        if not ref:
            return None
        ns, _, name = ref.rpartition("/")
        j = self.store.get("jobs", _key(pid, ns or "default", name))
        if j is None:
            return "Missing"
        for c in j.get("status", {}).get("conditions", []):
            if c["type"] in ("Complete", "Failed") and c["status"] == "True":
                return c["type"]
        return "Running"

    async def h_cluster_status(self, req: Request):
        p = self.project(req.q("project"))
        s = self.summary(p["id"])
        s["job"] = self._job_state(p["id"], req.q("job"))
        return s

    async def h_cluster_wait(self, req: Request):
        """Long-poll until `nodes` Ready (+validated) with >= `gpus` allocatable (+ job done)."""
        pid = req.q("project")
        want_nodes = int(req.q("nodes", "1"))
        want_gpus = int(req.q("gpus", "0"))
        validated = req.q("validated", "1") not in ("0", "false")
        job = req.q("job")
        timeout = min(float(req.q("timeout", "30")), 300.0)

        def check():
            try:
                p = self.project(pid)
            except HttpError:
                return None
            s = self.summary(p["id"])
            js = self._job_state(p["id"], job)
            failed = s["nodes_validation_failed"] > 0 or js in ("Failed", "Missing")
            ok = (s["nodes_ready"] >= want_nodes and (not validated or s["nodes_validated"] >= want_nodes)
                  and s["gpus_allocatable"] >= want_gpus and (js in (None, "Complete")))
            if ok or failed:
                s.update(ready=ok, failed=failed and not ok, job=js)
                return s
            return None

        res = await self.store.wait_until(check, timeout)
        if res:
            trace("cp", f"cluster wait -> ready={res.get('ready')}")
            return res
        p = self.project(pid)
        s = self.summary(p["id"])
        s.update(ready=False, failed=False, timed_out=True, job=self._job_state(p["id"], job))
        return Response(200, s)

    async def h_cp_events(self, req: Request):
        since = int(req.q("resourceVersion", "0") or 0)
        wait = min(float(req.q("timeoutSeconds", "0") or 0), 60.0)
        ev = await self.store.wait_events(since, None, wait)
        return {"resourceVersion": self.store.rv,
                "events": [{"type": e["type"], "kind": e["kind"], "name": e["object"].get("metadata", {}).get("name"),
                            "resourceVersion": e["resourceVersion"]} for e in ev]}

    # ---- k8s: nodes ----------------------------------------------------------------------
    def _pid(self, pid: str | None, req: Request) -> str:
        return self.project(pid or req.q("project")).get("id")

    def _strip(self, obj: dict) -> dict:
        return {k: v for k, v in obj.items() if not k.startswith("_")}

    async def _list_or_watch(self, req: Request, kind: str, pred) -> dict:
        if req.q("watch") in ("1", "true"):
            since = int(req.q("resourceVersion", "0") or 0)
            timeout = min(float(req.q("timeoutSeconds", "30") or 30), 300.0)
            ev = await self.store.wait_events(since, kind, timeout, pred)
            return {"kind": "WatchEventList", "resourceVersion": str(self.store.rv),
                    "events": [{"type": e["type"], "object": self._strip(e["object"])} for e in ev]}
        items = [self._strip(o) for o in self.store.list(kind, pred)]
        items.sort(key=lambda o: (o["metadata"].get("namespace", ""), o["metadata"]["name"]))
        return {"kind": "List", "apiVersion": "v1", "metadata": {"resourceVersion": str(self.store.rv)}, "items": items}

    async def h_nodes(self, req: Request, pid: str | None = None):
        p = self._pid(pid, req)
        sel = _parse_selector(req.q("labelSelector"))
        return await self._list_or_watch(req, "nodes", lambda n: self._in(p, n) and labels_match(sel, n["metadata"].get("labels")))

    async def h_node_get(self, req: Request, name: str, pid: str | None = None):
        p = self._pid(pid, req)
        n = self.store.get("nodes", _key(p, name))
        if n is None:
            raise HttpError(404, f"node {name} not found")
        return self._strip(n)

    def _node_secret_ok(self, req: Request, key: str) -> None:
        sec = self.store.get("nodesecrets", key)
        if sec is None or req.bearer != sec["nodeToken"]:
            raise HttpError(401, "invalid node token")

    async def h_node_status(self, req: Request, name: str, pid: str | None = None):
        """Heartbeat / status update from the node agent (the node lease)."""
        p = self._pid(pid, req)
        key = _key(p, name)
        self._node_secret_ok(req, key)
        body = req.json()
        self.leases[key] = time.monotonic()
        cur = self.store.get("nodes", key)
        if cur is None:
            raise HttpError(404, f"node {name} not found")
        changed = False
        new = copy.deepcopy(cur)
        st = new["status"]
        if "devices" in body:
            st["devices"] = body["devices"]
            healthy = sum(1 for d in body["devices"] if d.get("health", "Healthy") == "Healthy")
            if st["allocatable"].get(GPU) != str(healthy):
                st["allocatable"][GPU] = str(healthy)
            changed = True
        if "nodeInfo" in body:
            st["nodeInfo"] = body["nodeInfo"]
            changed = True
        if "annotations" in body:
            new["metadata"].setdefault("annotations", {}).update(body["annotations"])
            changed = True
        changed |= _set_ready(new)
        if changed:
            self.store.put("nodes", key, new)
            self.reconcile()
        return {"ok": True, "resourceVersion": self.store.rv}

    async def h_node_patch(self, req: Request, name: str, pid: str | None = None):
        p = self._pid(pid, req)
        self._auth(req, self.project(p))
        body = req.json()

        def fn(n):
            md = body.get("metadata", {})
            for f in ("labels", "annotations"):
                if f in md:
                    n["metadata"][f] = merge_patch(n["metadata"].get(f, {}), md[f] or {})
            if "spec" in body:
                n["spec"] = merge_patch(n["spec"], body["spec"])

        n = self.store.patch("nodes", _key(p, name), fn)
        if n is None:
            raise HttpError(404, f"node {name} not found")
        self.reconcile()
        return self._strip(n)

    async def h_node_delete(self, req: Request, name: str, pid: str | None = None):
        p = self._pid(pid, req)
        key = _key(p, name)
        sec = self.store.get("nodesecrets", key)
        if not (sec and req.bearer == sec["nodeToken"]):
            self._auth(req, self.project(p))
        n = self.store.delete("nodes", key)
        self.store.delete("nodesecrets", key)
        self.leases.pop(key, None)
        if n is None:
            raise HttpError(404, f"node {name} not found")
        self.reconcile()
        return {"kind": "Status", "status": "Success", "details": {"name": name, "kind": "nodes"}}

    async def h_namespaces(self, req: Request, pid: str | None = None):
        self._pid(pid, req)
        names = {"default", "kube-system", "amd-gpu"}
        for kind in ("pods", "daemonsets", "jobs", "deployments", "services", "configmaps", "secrets", "ingresses"):
            names |= {o["metadata"].get("namespace", "default") for o in self.store.list(kind)}
        return {"kind": "NamespaceList", "items": [{"metadata": {"name": n}} for n in sorted(names)]}

    # ---- k8s: generic namespaced kinds ------------------------------------------------
    async def h_pods(self, req: Request, pid: str | None = None):
        p = self._pid(pid, req)
        node = None
        fs = req.q("fieldSelector") or ""
        if fs.startswith("spec.nodeName="):
            node = fs.split("=", 1)[1]
        sel = _parse_selector(req.q("labelSelector"))
        return await self._list_or_watch(req, "pods", lambda o: self._in(p, o) and (node is None or o["spec"].get("nodeName") == node)
                                         and labels_match(sel, o["metadata"].get("labels")))

    def _lister(self, kind: str, all_ns: bool = False):
        async def h(req: Request, pid: str | None = None, ns: str | None = None):
            p = self._pid(pid, req)
            sel = _parse_selector(req.q("labelSelector"))
            return await self._list_or_watch(req, kind, lambda o: self._in(p, o) and (all_ns or o["metadata"].get("namespace") == ns)
                                             and labels_match(sel, o["metadata"].get("labels")))
        return h

    def _getter(self, kind: str):
        async def h(req: Request, ns: str, name: str, pid: str | None = None):
            p = self._pid(pid, req)
            o = self.store.get(kind, _key(p, ns, name))
            if o is None:
                raise HttpError(404, f'{kind} "{name}" not found')
            return self._strip(o)
        return h

    def _creator(self, kind: str):
        async def h(req: Request, ns: str, pid: str | None = None):
            p = self._pid(pid, req)
            self._auth(req, self.project(p))
            body = req.json()
            return Response(201, self._strip(self.create(p, kind, ns, body)))
        return h

    def _replacer(self, kind: str, merge: bool):
        async def h(req: Request, ns: str, name: str, pid: str | None = None):
            p = self._pid(pid, req)
            self._auth(req, self.project(p))
            body = req.json()
            if not isinstance(body, dict):
                raise HttpError(422, "the body must be a JSON object")
            return self._strip(self.replace(p, kind, ns, name, body, merge=merge))
        return h

    async def h_scale(self, req: Request, ns: str, name: str, pid: str | None = None):
        """The Deployment ``scale`` subresource (autoscaling/v1 Scale): kubectl scale."""
        p = self._pid(pid, req)
        d = self.store.get("deployments", _key(p, ns, name))
        if d is None:
            raise HttpError(404, f'deployments.apps "{name}" not found')
        if req.method in ("PUT", "PATCH"):
            self._auth(req, self.project(p))
            n = (req.json().get("spec") or {}).get("replicas")
            if not isinstance(n, int) or isinstance(n, bool) or n < 0:
                raise HttpError(422, "spec.replicas must be a non-negative integer")
            d = self.replace(p, "deployments", ns, name, {"spec": {"replicas": n}}, merge=True)
        sel = (d["spec"].get("selector") or {}).get("matchLabels") or {}
        return {"kind": "Scale", "apiVersion": "autoscaling/v1",
                "metadata": {"name": name, "namespace": ns, "resourceVersion": d["metadata"]["resourceVersion"]},
                "spec": {"replicas": int(d["spec"].get("replicas", 1))},
                "status": {"replicas": int(d.get("status", {}).get("replicas", 0)),
                           "selector": ",".join(f"{k}={v}" for k, v in sel.items())}}

    def _deleter(self, kind: str):
        async def h(req: Request, ns: str, name: str, pid: str | None = None):
            p = self._pid(pid, req)
            self._auth(req, self.project(p))
            o = self.store.delete(kind, _key(p, ns, name))
            if o is None:
                raise HttpError(404, f'{kind} "{name}" not found')
            if kind in ("services", "ingresses"):
                self._sync_proxy()
            if kind != "pods":
                for pod in self.store.list("pods", lambda x: self._in(p, x) and any(
                        r.get("uid") == o["metadata"]["uid"] for r in x["metadata"].get("ownerReferences", []))):
                    self.store.delete("pods", _key(p, ns, pod["metadata"]["name"]))
            self.reconcile()
            return {"kind": "Status", "status": "Success", "details": {"name": name, "kind": kind}}
        return h

    # ---- networking: pod CIDRs, Service IPs / ports, endpoints --------------------------
    def _next_pod_cidr(self) -> str:
        """One /24 of 127.128.0.0/9 per registered node: pods bind their own loopback IP."""
        used = {n.get("spec", {}).get("podCIDR") for n in self.store.list("nodes")}
        for k in range(1 << 15):
            c = f"127.{128 + (k >> 8)}.{k & 255}.0/24"
            if c not in used:
                return c
        raise HttpError(507, "pod CIDR space exhausted")

    def _alloc_service(self, body: dict, exclude: str | None = None) -> None:
        spec = body.setdefault("spec", {})
        stype = spec.setdefault("type", "ClusterIP")
        if stype not in ("ClusterIP", "NodePort", "LoadBalancer"):
            raise HttpError(422, f"service type {stype!r} is not supported")
        ports = spec.get("ports") or []
        if not ports:
            raise HttpError(422, "spec.ports is required")
        svcs = [o for o in self.store.list("services")
                if _key(o["_project"], o["metadata"]["namespace"], o["metadata"]["name"]) != exclude]
        used_ips = {o["spec"].get("clusterIP") for o in svcs}
        used_np = {p.get("nodePort") for o in svcs for p in o["spec"].get("ports", [])}
        used_lb = {(p.get("port")) for o in svcs if o["spec"].get("type") == "LoadBalancer" for p in o["spec"].get("ports", [])}
        if not spec.get("clusterIP"):
            spec["clusterIP"] = next(f"127.96.{k >> 8}.{k & 255}" for k in range(1, 1 << 16)
                                     if f"127.96.{k >> 8}.{k & 255}" not in used_ips)
        for i, port in enumerate(ports):
            if "port" not in port:
                raise HttpError(422, f"spec.ports[{i}].port is required")
            port.setdefault("name", str(port["port"]))
            port.setdefault("protocol", "TCP")
            port.setdefault("targetPort", port["port"])
            if stype in ("NodePort", "LoadBalancer") and not port.get("nodePort"):
                port["nodePort"] = next(n for n in range(30000, 32768) if n not in used_np)
                used_np.add(port["nodePort"])
            if stype == "LoadBalancer" and port["port"] in used_lb:
                raise HttpError(409, f"load balancer port {port['port']} is taken")
        if stype == "LoadBalancer":
            body["status"] = {"loadBalancer": {"ingress": [{"ip": self.advertise or self.host}]}}

    def _endpoints(self, svc_key: str, port_key: str) -> list[tuple[str, int]]:
        svc = self.store.get("services", svc_key)
        if svc is None:
            return []
        pid, ns = svc["_project"], svc["metadata"]["namespace"]
        sel = svc["spec"].get("selector") or {}
        port = next((p for p in svc["spec"]["ports"] if p["name"] == port_key), None)
        if port is None or not sel:
            return []
        out = []
        for o in self.store.list("pods", lambda o: self._in(pid, o) and o["metadata"].get("namespace") == ns):
            if o.get("status", {}).get("phase") != "Running" or not labels_match(sel, o["metadata"].get("labels")):
                continue
            ip = o.get("status", {}).get("podIP")
            tp = port["targetPort"]
            if isinstance(tp, str):  # named container port
                tp = next((cp.get("containerPort") for c in o["spec"].get("containers", [])
                           for cp in c.get("ports", []) if cp.get("name") == tp), None)
            if ip and tp:
                out.append((ip, host_port(int(tp))))
        return sorted(out)

    def _proxy_wanted(self) -> dict:
        wanted = {}
        lb_host = self.advertise or self.host
        for svc in self.store.list("services"):
            key = _key(svc["_project"], svc["metadata"]["namespace"], svc["metadata"]["name"])
            spec = svc["spec"]
            for p in spec.get("ports", []):
                wanted[(key, spec["clusterIP"], host_port(p["port"]))] = p["name"]
                if spec.get("type") in ("NodePort", "LoadBalancer") and p.get("nodePort"):
                    for h in {lb_host, "127.0.0.1"}:
                        wanted[(key, h, int(p["nodePort"]))] = p["name"]
                if spec.get("type") == "LoadBalancer":
                    wanted[(key, lb_host, host_port(p["port"]))] = p["name"]
        return wanted

    def _sync_proxy(self) -> None:
        try:
            loop = asyncio.get_running_loop()
        except RuntimeError:
            return
        loop.create_task(self.proxy.sync(self._proxy_wanted()))
        if self.ingress_port:
            loop.create_task(self.ingress.ensure(self.advertise or self.host, self.ingress_port,
                                                 bool(self.store.keys("ingresses"))))

    def _ingress_routes(self) -> list[tuple[str, str, str, str, str]]:
        """(host, path, pathType, service key, service port key) of every Ingress rule."""
        routes = []
        for ing in self.store.list("ingresses"):
            pid, ns = ing["_project"], ing["metadata"]["namespace"]

            def backend(b):
                svc = (b or {}).get("service") or {}
                key = _key(pid, ns, svc.get("name", ""))
                o = self.store.get("services", key)
                port = svc.get("port") or {}
                for sp in (o or {}).get("spec", {}).get("ports", []):
                    if sp.get("name") == port.get("name") or sp.get("port") == port.get("number"):
                        return key, sp["name"]
                return None

            spec = ing.get("spec", {})
            for rule in spec.get("rules") or []:
                for path in (rule.get("http") or {}).get("paths") or []:
                    b = backend(path.get("backend"))
                    if b:
                        routes.append((rule.get("host", ""), path.get("path", "/"), path.get("pathType", "Prefix"), *b))
            b = backend(spec.get("defaultBackend"))
            if b:
                routes.append(("", "/", "Prefix", *b))
        return routes

    def dns_resolve(self, name: str):
        """Cluster DNS answer for ``name``: [ips], None (NXDOMAIN) or False (REFUSED)."""
        from .dns import DOMAIN

        name = name.rstrip(".").lower()
        if name.endswith("." + DOMAIN):
            parts = name[: -len(DOMAIN) - 1].split(".")
        elif name.endswith(".svc"):
            parts = name.split(".")
        elif name.count(".") == 1 and any(o["metadata"].get("namespace") == name.split(".")[1]
                                          for kind in ("services", "pods") for o in self.store.list(kind)):
            parts = name.split(".")  # <svc>.<ns> short form, for namespaces the cluster has
        else:
            return False
        if len(parts) == 3 and parts[2] == "pod":
            ip = parts[0].replace("-", ".")
            try:
                import ipaddress

                ipaddress.IPv4Address(ip)
                return [ip]
            except ValueError:
                return None
        if parts and parts[-1] == "svc":
            parts = parts[:-1]
        if len(parts) != 2:
            return None
        svc, ns = parts
        projects = sorted(self.store.list("projects"), key=lambda p: p["created_seq"])
        for p in projects:
            o = self.store.get("services", _key(p["id"], ns, svc))
            if o and o["spec"].get("clusterIP"):
                return [o["spec"]["clusterIP"]]
        return None

    def create(self, pid: str, kind: str, ns: str, body: dict) -> dict:
        md = body.setdefault("metadata", {})
        name = md.get("name")
        if not name and md.get("generateName"):
            name = md["generateName"] + secrets.token_hex(3)
        if not name:
            raise HttpError(422, "metadata.name is required")
        md["name"] = name
        md["namespace"] = ns
        md.setdefault("labels", {})
        md.setdefault("annotations", {})
        body["_project"] = pid
        key = _key(pid, ns, name)
        if self.store.get(kind, key) is not None:
            raise HttpError(409, f'{kind} "{name}" already exists')
        _admit_gpu_visibility(kind, ns, body)
        if kind == "pods":
            spec = body.setdefault("spec", {})
            if not spec.get("containers"):
                raise HttpError(422, "spec.containers is required")
            spec.setdefault("restartPolicy", "Always")
            body["status"] = {"phase": "Pending", "conditions": []}
        elif kind in ("daemonsets", "deployments", "jobs"):
            tmpl = body.get("spec", {}).get("template", {})
            if not tmpl.get("spec", {}).get("containers"):
                raise HttpError(422, "spec.template.spec.containers is required")
            body.setdefault("status", {})
            md["generation"] = 1
        elif kind == "services":
            self._alloc_service(body)
        elif kind in ("configmaps", "secrets"):
            _normalize_data(kind, body)
        elif kind == "ingresses":
            body["status"] = {"loadBalancer": {"ingress": [{"ip": self.advertise or self.host}]}}
        o = self.store.put(kind, key, body)
        if kind in ("services", "ingresses"):
            self._sync_proxy()
        self.reconcile()
        return o

    def replace(self, pid: str, kind: str, ns: str, name: str, body: dict, merge: bool = False) -> dict:
        """PUT (``merge=False``: the whole object, optimistic concurrency on resourceVersion) or
        PATCH (``merge=True``: RFC 7386 merge patch). Status stays server-owned; identity fields,
        a Service's clusterIP and a Job's / Pod's spec are immutable, as in Kubernetes."""
        key = _key(pid, ns, name)
        cur = self.store.get(kind, key)
        if cur is None:
            raise HttpError(404, f'{kind} "{name}" not found')
        if merge:
            new = merge_patch(self._strip(cur), body)
        else:
            rv = (body.get("metadata") or {}).get("resourceVersion")
            if rv and rv != cur["metadata"].get("resourceVersion"):
                raise HttpError(409, f'Operation cannot be fulfilled on {kind} "{name}": the object has been '
                                     "modified; please apply your changes to the latest version and try again")
            new = copy.deepcopy(body)
        if "status" in cur:
            new["status"] = copy.deepcopy(cur["status"])
        md = new.setdefault("metadata", {})
        md.update(name=name, namespace=ns, uid=cur["metadata"]["uid"],
                  creationTimestamp=cur["metadata"].get("creationTimestamp"))
        md.pop("resourceVersion", None)
        md.setdefault("labels", {})
        md.setdefault("annotations", {})
        spec_changed = new.get("spec") != cur.get("spec")
        if kind == "pods" and spec_changed:
            raise HttpError(422, f'Pod "{name}" is invalid: spec: Forbidden: pod updates may not change '
                                 "fields other than metadata")
        if kind == "jobs" and new.get("spec", {}).get("template") != cur.get("spec", {}).get("template"):
            raise HttpError(422, f'Job.batch "{name}" is invalid: spec.template: field is immutable')
        if kind in ("daemonsets", "deployments", "jobs"):
            if not new.get("spec", {}).get("template", {}).get("spec", {}).get("containers"):
                raise HttpError(422, "spec.template.spec.containers is required")
            gen = int(cur["metadata"].get("generation", 1))
            md["generation"] = gen + 1 if spec_changed else gen
        if kind == "services":
            spec = new.setdefault("spec", {})
            cip = cur["spec"].get("clusterIP")
            if spec.get("clusterIP") and spec["clusterIP"] != cip:
                raise HttpError(422, f'Service "{name}" is invalid: spec.clusterIP: field is immutable')
            spec["clusterIP"] = cip
            old_np = {(p.get("port"), p.get("protocol", "TCP")): p.get("nodePort") for p in cur["spec"].get("ports", [])}
            for port in spec.get("ports") or []:
                if not port.get("nodePort") and old_np.get((port.get("port"), port.get("protocol", "TCP"))):
                    port["nodePort"] = old_np[(port.get("port"), port.get("protocol", "TCP"))]
            self._alloc_service(new, exclude=key)
        if kind in ("configmaps", "secrets"):
            _normalize_data(kind, new)
        new["_project"] = pid
        o = self.store.put(kind, key, new)
        if kind in ("services", "ingresses"):
            self._sync_proxy()
        self.reconcile()
        return o

    async def h_pod_status(self, req: Request, ns: str, name: str, pid: str | None = None):
        p = self._pid(pid, req)
        key = _key(p, ns, name)
        cur = self.store.get("pods", key)
        if cur is None:
            raise HttpError(404, f'pod "{name}" not found')
        node = cur["spec"].get("nodeName")
        if node:
            self._node_secret_ok(req, _key(p, node))
        body = req.json()
        st = body.get("status", body)
        ann = body.get("annotations")

        def fn(o):
            o.setdefault("status", {}).update(st)
            if ann:
                o["metadata"].setdefault("annotations", {}).update(ann)

        trace("cp", f"pod status {ns}/{name} {st.get('phase')}")
        o = self.store.patch("pods", key, fn)
        phase = st.get("phase")
        if phase in ("Running", "Succeeded", "Failed"):
            self._event(p, ns, {"kind": "Pod", "name": name}, {"Running": "Started", "Succeeded": "Completed",
                                                               "Failed": "Failed"}[phase],
                        f"pod {name} {phase.lower()} on {node}", "Warning" if phase == "Failed" else "Normal")
        self.reconcile()
        trace("cp", f"pod status {ns}/{name} reconciled")
        return self._strip(o)

    async def h_pod_log(self, req: Request, ns: str, name: str, pid: str | None = None):
        p = self._pid(pid, req)
        o = self.store.get("pods", _key(p, ns, name))
        if o is None:
            raise HttpError(404, f'pod "{name}" not found')
        path = o["metadata"].get("annotations", {}).get("tk8s.amd.com/log-path")
        if not path or not os.path.exists(path):
            return Response(200, "", content_type="text/plain")
        tail = int(req.q("tailLines", "0") or 0)
        text = Path(path).read_text(errors="replace")
        if tail:
            text = "\n".join(text.splitlines()[-tail:]) + "\n"
        return Response(200, text, content_type="text/plain")

    # ---- exec: a command in a running pod's environment (the kubelet's exec, request/response) --
    async def h_pod_exec(self, req: Request, ns: str, name: str, pid: str | None = None):
        """``kubectl exec POD -- CMD``: queued for the pod's node agent, which runs CMD with the
        pod's env in its directory and posts stdout/stderr/exit code back; this request waits for
        that (non-interactive; the API server's SPDY/websocket streams have no equivalent here)."""
        p = self._pid(pid, req)
        self._auth(req, self.project(p))
        pod = self.store.get("pods", _key(p, ns, name))
        if pod is None:
            raise HttpError(404, f'pod "{name}" not found')
        if pod.get("status", {}).get("phase") != "Running" or not pod["spec"].get("nodeName"):
            raise HttpError(400, f'pod "{name}" is not running')
        body = req.json()
        cmd = body.get("command")
        if not isinstance(cmd, list) or not cmd:
            raise HttpError(422, "command must be a non-empty list")
        timeout = min(float(body.get("timeoutSeconds", 60)), 600.0)
        self._seq += 1
        xid = f"x{self._seq:x}"
        node = pod["spec"]["nodeName"]
        key = _key(p, node, xid)
        self.store.put("execs", key, {"metadata": {"name": xid}, "_project": p, "node": node, "pod": name,
                                      "namespace": ns, "command": [str(c) for c in cmd],
                                      "stdin": str(body.get("stdin", "")), "timeoutSeconds": timeout,
                                      "status": {"phase": "Pending"}})
        done = await self.store.wait_until(
            lambda: (self.store.get("execs", key) or {}).get("status", {}).get("phase") == "Done", timeout + 10)
        x = self.store.delete("execs", key) or {}
        if not done:
            raise HttpError(504, f"exec in {name}: no result from node {node} within {timeout:.0f}s")
        st = x.get("status", {})
        return {"stdout": st.get("stdout", ""), "stderr": st.get("stderr", ""), "exitCode": st.get("exitCode", 1)}

    async def h_node_execs(self, req: Request, node: str, pid: str | None = None):
        """The node agent's long-poll for exec requests of its pods."""
        p = self._pid(pid, req)
        self._node_secret_ok(req, _key(p, node))

        def pending():
            return [self._strip(x) for x in self.store.list("execs", lambda x: x.get("_project") == p and
                    x.get("node") == node and x.get("status", {}).get("phase") == "Pending")]

        wait = min(float(req.q("timeoutSeconds", "20") or 20), 60.0)
        items = await self.store.wait_until(pending, wait) or []
        for x in items:  # handed out: not returned again
            self.store.patch("execs", _key(p, node, x["metadata"]["name"]),
                             lambda o: o["status"].update(phase="Running"))
        return {"items": items}

    async def h_exec_result(self, req: Request, node: str, xid: str, pid: str | None = None):
        p = self._pid(pid, req)
        self._node_secret_ok(req, _key(p, node))
        body = req.json()
        x = self.store.patch("execs", _key(p, node, xid), lambda o: o["status"].update(
            phase="Done", stdout=str(body.get("stdout", ""))[-1 << 20:], stderr=str(body.get("stderr", ""))[-1 << 20:],
            exitCode=int(body.get("exitCode", 1))))
        if x is None:
            raise HttpError(404, f"exec {xid} not found (timed out?)")
        return {"ok": True}

    # ---- controllers ------------------------------------------------------------------
    def reconcile(self) -> None:
        """Run every controller once (cheap at this scale; called after each mutation)."""
        if getattr(self, "_reconciling", False):
            self._again = True
            return
        self._reconciling = True
        try:
            for _ in range(8):
                self._again = False
                for p in self.store.list("projects"):
                    pid = p["id"]
                    self._ctl_daemonsets(pid)
                    self._ctl_jobs(pid)
                    self._ctl_deployments(pid)
                    self._ctl_validation(pid)
                    self._scheduler(pid)
                if not self._again:
                    break
        finally:
            self._reconciling = False

    def _new_pod(self, pid: str, ns: str, name: str, owner: dict, owner_kind: str, template: dict,
                 node: str | None = None, extra_env: dict | None = None, labels: dict | None = None,
                 annotations: dict | None = None) -> dict:
        spec = copy.deepcopy(template.get("spec", {}))
        if extra_env:
            for c in spec.get("containers", []):
                c.setdefault("env", []).extend({"name": k, "value": str(v)} for k, v in extra_env.items())
        if node:
            spec["nodeName"] = node
        md = copy.deepcopy(template.get("metadata", {}))
        md.update(name=name, namespace=ns)
        md.setdefault("labels", {}).update(labels or {})
        md.setdefault("annotations", {}).update(annotations or {})
        md["ownerReferences"] = [{"kind": owner_kind, "name": owner["metadata"]["name"], "uid": owner["metadata"]["uid"]}]
        pod = {"kind": "Pod", "apiVersion": "v1", "metadata": md, "spec": spec, "_project": pid,
               "status": {"phase": "Pending", "conditions": []}}
        spec.setdefault("restartPolicy", "Always")
        return self.store.put("pods", _key(pid, ns, name), pod)

    def _owned(self, pid: str, owner: dict) -> list[dict]:
        uid = owner["metadata"]["uid"]
        return self.store.list("pods", lambda o: self._in(pid, o) and any(
            r.get("uid") == uid for r in o["metadata"].get("ownerReferences", [])))

    def _ctl_daemonsets(self, pid: str) -> None:
        nodes = self.store.list("nodes", lambda n: self._in(pid, n))
        for ds in self.store.list("daemonsets", lambda o: self._in(pid, o)):
            ns = ds["metadata"]["namespace"]
            tmpl = ds["spec"]["template"]
            sel = tmpl.get("spec", {}).get("nodeSelector")
            pods = {o["spec"].get("nodeName"): o for o in self._owned(pid, ds)}
            eligible = [n for n in nodes if labels_match(sel, n["metadata"].get("labels"))
                        and not n["spec"].get("unschedulable")]
            for n in eligible:
                nn = n["metadata"]["name"]
                if nn not in pods:
                    pods[nn] = self._new_pod(pid, ns, f"{ds['metadata']['name']}-{nn}", ds, "DaemonSet", tmpl, node=nn,
                                             labels=ds["spec"].get("selector", {}).get("matchLabels"))
            phases = [o.get("status", {}).get("phase") for o in pods.values()]
            status = {"desiredNumberScheduled": len(eligible), "currentNumberScheduled": len(pods),
                      "numberReady": phases.count("Running") + phases.count("Succeeded"),
                      "numberSucceeded": phases.count("Succeeded"), "numberFailed": phases.count("Failed")}
            if ds.get("status") != status:
                self.store.patch("daemonsets", _key(pid, ns, ds["metadata"]["name"]), lambda o, s=status: o.__setitem__("status", s))

    def _ctl_validation(self, pid: str) -> None:
        """Node condition AMDGPUValidated from the validation DaemonSet's pod on that node."""
        for ds in self.store.list("daemonsets", lambda o: self._in(pid, o) and o["metadata"].get("labels", {}).get(VALIDATION_LABEL) == "true"):
            for pod in self._owned(pid, ds):
                nn = pod["spec"].get("nodeName")
                phase = pod.get("status", {}).get("phase")
                if not nn or phase not in TERMINAL:
                    continue
                key = _key(pid, nn)
                n = self.store.get("nodes", key)
                if n is None:
                    continue
                result = pod.get("status", {}).get("result") or {}
                view = _xgmi_view(result)
                want = ("True", "ProbesPassed") if phase == "Succeeded" else ("False", "ProbesFailed")
                if want[0] == "True" and view is not None and not view["healthy"]:
                    want = ("False", "XGMILinkDegraded")
                c = _cond(n, "AMDGPUValidated")
                if c and (c["status"], c["reason"]) == want:
                    continue

                def fn(node, want=want, result=result, pod=pod, view=view):
                    from .. import xgmi

                    msg = xgmi.message(view) if want[1] == "XGMILinkDegraded" else pod.get("status", {}).get("message", "")
                    _set_cond(node, "AMDGPUValidated", want[0], want[1], msg[:500])
                    ann = node["metadata"].setdefault("annotations", {})
                    if view is not None:
                        ann.update(xgmi.annotations(view))
                        if view["healthy"]:
                            _set_cond(node, "XGMILinksHealthy", "True", "LinksHealthy",
                                      f"{view['pulls']} pulls >= {view.get('min_fraction')} x median {view.get('median_gbps')} GB/s")
                        else:
                            _set_cond(node, "XGMILinksHealthy", "False", "XGMILinkDegraded", xgmi.message(view))
                        _set_ready(node)
                    for k, path in (("hbm-write-gbps", ("hbm", "gbps")), ("hbm-read-gbps", ("hbm", "read_gbps")),
                                    ("md5-mbps", ("md5", "mbps")),
                                    ("copy-gbps", ("copy", "kernel_gbps")), ("probe-ms", ("timings_ms", "total")),
                                    ("hip-init-ms", ("timings_ms", "hip_init"))):
                        v = result.get(path[0], {}).get(path[1]) if isinstance(result.get(path[0]), dict) else None
                        if v is not None:
                            ann[f"tk8s.amd.com/{k}"] = f"{v:.1f}"

                self.store.patch("nodes", key, fn)
                if want[1] == "XGMILinkDegraded":
                    from .. import xgmi

                    self._event(pid, "default", {"kind": "Node", "name": nn}, "XGMILinkDegraded", xgmi.message(view),
                                "Warning")

    def _ctl_jobs(self, pid: str) -> None:
        for job in self.store.list("jobs", lambda o: self._in(pid, o)):
            ns, jname = job["metadata"]["namespace"], job["metadata"]["name"]
            spec = job["spec"]
            completions = int(spec.get("completions", 1))
            parallelism = int(spec.get("parallelism", completions))
            backoff = int(spec.get("backoffLimit", 6))
            indexed = spec.get("completionMode") == "Indexed"
            pods = self._owned(pid, job)
            succeeded_idx, active, failed = set(), 0, 0
            for o in pods:
                ph = o.get("status", {}).get("phase")
                idx = int(o["metadata"].get("annotations", {}).get("batch.kubernetes.io/job-completion-index", -1))
                if ph == "Succeeded":
                    succeeded_idx.add(idx if indexed else o["metadata"]["name"])
                elif ph == "Failed":
                    failed += 1
                else:
                    active += 1
            done = any(c["type"] in ("Complete", "Failed") and c["status"] == "True" for c in job.get("status", {}).get("conditions", []))
            if not done and failed > backoff:
                for o in pods:  # stop the rest (a gang job cannot finish without all ranks)
                    if o.get("status", {}).get("phase") not in TERMINAL:
                        self.store.delete("pods", _key(pid, ns, o["metadata"]["name"]))
            elif not done:
                running_idx = {int(o["metadata"].get("annotations", {}).get("batch.kubernetes.io/job-completion-index", -1))
                               for o in pods if o.get("status", {}).get("phase") not in TERMINAL}
                need = [i for i in range(completions) if i not in succeeded_idx and i not in running_idx] if indexed \
                    else list(range(max(0, completions - len(succeeded_idx) - active)))
                for i in need[: max(0, parallelism - active)]:
                    self._seq += 1
                    name = f"{jname}-{i}-{self._seq:x}" if indexed else f"{jname}-{self._seq:x}"
                    env = {"JOB_COMPLETION_INDEX": i, "JOB_COMPLETIONS": completions, "JOB_NAME": jname} if indexed else {"JOB_NAME": jname}
                    self._new_pod(pid, ns, name, job, "Job", spec["template"], extra_env=env,
                                  labels={"job-name": jname},
                                  annotations={"batch.kubernetes.io/job-completion-index": str(i)} if indexed else None)
                    active += 1
            status = dict(job.get("status", {}))
            status.update(active=active, succeeded=len(succeeded_idx), failed=failed)
            conds = [c for c in status.get("conditions", [])]
            if not done:
                if len(succeeded_idx) >= completions:
                    conds.append({"type": "Complete", "status": "True", "lastTransitionTime": now_iso()})
                    status["completionTime"] = now_iso()
                elif failed > backoff:
                    conds.append({"type": "Failed", "status": "True", "reason": "BackoffLimitExceeded",
                                  "lastTransitionTime": now_iso()})
            status["conditions"] = conds
            if status != job.get("status"):
                self.store.patch("jobs", _key(pid, ns, jname), lambda o, s=status: o.__setitem__("status", s))

    def _ctl_deployments(self, pid: str) -> None:
        """Deployment controller with ReplicaSet-style generations: pods carry the
        ``pod-template-hash`` of the template they came from. A changed template rolls out with
        the RollingUpdate defaults (maxSurge 25 % rounded up, maxUnavailable 25 % rounded down;
        an old pod goes only when a new one runs), ``strategy: Recreate`` drops the old pods first."""
        for d in self.store.list("deployments", lambda o: self._in(pid, o)):
            ns, dname = d["metadata"]["namespace"], d["metadata"]["name"]
            spec = d["spec"]
            want = int(spec.get("replicas", 1))
            h = template_hash(spec["template"])
            match = (spec.get("selector") or {}).get("matchLabels") or {}

            def live():
                return [o for o in self._owned(pid, d) if o.get("status", {}).get("phase") not in TERMINAL]

            unavailable = want // 4
            for _ in range(2):  # scale down old -> room to surge again, in the same pass
                pods = live()
                new = [o for o in pods if o["metadata"].get("labels", {}).get("pod-template-hash") == h]
                old = [o for o in pods if o not in new]
                if (spec.get("strategy") or {}).get("type") == "Recreate" and old:
                    for o in old:
                        self.store.delete("pods", _key(pid, ns, o["metadata"]["name"]))
                    pods, old = new, []
                surge = max(1, -(-want // 4)) if old else 0
                for _ in range(max(0, min(want - len(new), want + surge - len(pods)))):
                    self._seq += 1
                    new.append(self._new_pod(pid, ns, f"{dname}-{h[:8]}-{self._seq:x}", d, "Deployment",
                                             spec["template"], labels={**match, "pod-template-hash": h}))
                ready_new = sum(1 for o in new if o.get("status", {}).get("phase") == "Running")
                keep_old = max(0, want - unavailable - ready_new)
                for o in sorted(old, key=lambda o: o["metadata"]["name"])[keep_old:]:
                    self.store.delete("pods", _key(pid, ns, o["metadata"]["name"]))
                for o in sorted(new, key=lambda o: o["metadata"]["name"])[want:]:
                    self.store.delete("pods", _key(pid, ns, o["metadata"]["name"]))
            pods = live()
            running = sum(1 for o in pods if o.get("status", {}).get("phase") == "Running")
            status = {"observedGeneration": int(d["metadata"].get("generation", 1)), "replicas": len(pods),
                      "updatedReplicas": sum(1 for o in pods if o["metadata"].get("labels", {}).get("pod-template-hash") == h),
                      "readyReplicas": running, "availableReplicas": running,
                      "unavailableReplicas": max(0, want - running)}
            if d.get("status") != status:
                self.store.patch("deployments", _key(pid, ns, dname), lambda o, s=status: o.__setitem__("status", s))

    def _scheduler(self, pid: str) -> None:
        pending = [o for o in self.store.list("pods", lambda o: self._in(pid, o))
                   if not o["spec"].get("nodeName") and o.get("status", {}).get("phase") == "Pending"]
        if not pending:
            return
        nodes = [n for n in self.store.list("nodes", lambda n: self._in(pid, n))
                 if node_ready(n) and not n["spec"].get("unschedulable")]
        used: dict[str, int] = {}
        count: dict[str, int] = {}
        for o in self.store.list("pods", lambda o: self._in(pid, o)):
            nn = o["spec"].get("nodeName")
            if nn and o.get("status", {}).get("phase") not in TERMINAL:
                used[nn] = used.get(nn, 0) + pod_gpus(o)
                count[nn] = count.get(nn, 0) + 1
        for pod in sorted(pending, key=lambda o: o["metadata"]["name"]):
            need = pod_gpus(pod)
            sel = pod["spec"].get("nodeSelector")
            best = None
            for n in nodes:
                nn = n["metadata"]["name"]
                free = int(n["status"]["allocatable"].get(GPU, 0)) - used.get(nn, 0)
                if need > free or not labels_match(sel, n["metadata"].get("labels")):
                    continue
                if need and not node_validated(n):
                    continue  # GPU pods only land on validated nodes
                score = (count.get(nn, 0), -free, nn)
                if best is None or score < best[0]:
                    best = (score, nn, free)
            key = _key(pid, pod["metadata"]["namespace"], pod["metadata"]["name"])
            if best is None:
                c = _cond(pod, "PodScheduled")
                if not c or c["status"] != "False":
                    self.store.patch("pods", key, lambda o, need=need: _set_cond(
                        o, "PodScheduled", "False", "Unschedulable", f"0/{len(nodes)} nodes available: need {need} {GPU}"))
                continue
            nn = best[1]
            used[nn] = used.get(nn, 0) + need
            count[nn] = count.get(nn, 0) + 1

            def bind(o, nn=nn):
                o["spec"]["nodeName"] = nn
                _set_cond(o, "PodScheduled", "True", "Scheduled", f"assigned to {nn}")

            self.store.patch("pods", key, bind)
            self._event(pid, pod["metadata"]["namespace"], {"kind": "Pod", "name": pod["metadata"]["name"]},
                        "Scheduled", f"Successfully assigned {pod['metadata']['name']} to {nn}")

    # ---- node lifecycle ---------------------------------------------------------------
    async def lease_loop(self) -> None:
        while True:
            await asyncio.sleep(min(0.25, self.node_grace / 4))
            now = time.monotonic()
            changed = False
            for key, t in list(self.leases.items()):
                if now - t > self.node_grace:
                    n = self.store.get("nodes", key)
                    if n is None:
                        self.leases.pop(key, None)
                        continue
                    c = _cond(n, "Ready")
                    if c and c["status"] == "True":
                        self.store.patch("nodes", key, lambda o: _set_cond(
                            o, "Ready", "Unknown", "NodeStatusUnknown", "tk8s agent stopped posting node status"))
                        pid = key.split("/", 1)[0]
                        self._event(pid, "default", {"kind": "Node", "name": n["metadata"]["name"]}, "NodeNotReady",
                                    f"lease expired after {self.node_grace:.1f}s", "Warning")
                        changed = True
            if changed:
                self.reconcile()

    async def snapshot_loop(self) -> None:
        if not self.state_dir:
            return
        last = -1
        while True:
            await asyncio.sleep(1.0)
            if self.store.rv != last:
                last = self.store.rv
                self.store.snapshot(self.state_dir / "controlplane.json")

    # ---- run --------------------------------------------------------------------------
    async def run(self, ready_file: str | None = None) -> None:
        if self.state_dir:
            self.state_dir.mkdir(parents=True, exist_ok=True)
            if self.store.restore(self.state_dir / "controlplane.json"):
                now = time.monotonic()
                for key in self.store.keys("nodes"):
                    self.leases[key] = now  # grace period for agents to resume heartbeats
                self._seq = self.store.rv + 1000
        self._ensure_templates()
        host, port = await self.http.start(self.host, self.port)
        self.port = port
        if self.store.keys("services"):
            await self.proxy.sync(self._proxy_wanted())  # services restored from a snapshot
        if self.store.keys("ingresses") and self.ingress_port:
            await self.ingress.ensure(self.advertise or self.host, self.ingress_port, True)

        tasks = [asyncio.create_task(self.lease_loop()), asyncio.create_task(self.snapshot_loop())]
        # Mirrors the rancher/server log line the reference waits for (ranchermaster:14-20).
        print(f"Listening on {host}:{port}", flush=True)
        if ready_file:
            from ..utils.fsutil import atomic_write_json

            atomic_write_json(ready_file, {"host": host, "port": port, "pid": os.getpid(), "base": self.base})
        dns_transport = None  # after "Listening on": not on the bring-up's critical path
        if self.dns_port:
            from .dns import DnsProtocol

            try:
                dns_transport, _ = await asyncio.get_running_loop().create_datagram_endpoint(
                    lambda: DnsProtocol(self.dns_resolve), local_addr=(self.advertise or self.host, self.dns_port))
            except OSError as e:
                self._log_error(f"cluster DNS: cannot listen on udp {self.advertise or self.host}:{self.dns_port}: {e}\n")
        self._stop = asyncio.Event()
        loop = asyncio.get_running_loop()
        for sig in (signal.SIGTERM, signal.SIGINT):
            loop.add_signal_handler(sig, self._stop.set)
        await self._stop.wait()
        for t in tasks:
            t.cancel()
        await self.proxy.close()
        await self.ingress.close()
        if dns_transport is not None:
            dns_transport.close()
        if self.state_dir:
            self.store.snapshot(self.state_dir / "controlplane.json")
        await self.http.close()


def _parse_selector(s: str | None) -> dict | None:
    if not s:
        return None
    out = {}
    for part in s.split(","):
        if "=" in part:
            k, v = part.split("=", 1)
            out[k.strip().rstrip("=")] = v.strip()
    return out


def await_args(path: str, timeout: float | None = None) -> list[str]:
    """Zygote mode: wait for the JSON argument list (orchestrator._boot_controlplane writes it
    atomically). A zygote nobody hands arguments to -- the bring-up failed before its master
    existed -- stops its supervisor and exits, so it never lingers or restarts."""
    if timeout is None:
        timeout = float(os.environ.get("TK8S_ZYGOTE_TIMEOUT", "120"))
    deadline = time.monotonic() + timeout
    t_fast = time.monotonic() + 2.0
    while True:
        try:
            with open(path) as f:
                argv = json.load(f)
            if isinstance(argv, list):
                return [str(a) for a in argv]
        except (OSError, ValueError):
            pass
        if time.monotonic() > deadline:
            parent = os.getppid()
            try:
                with open(f"/proc/{parent}/comm") as f:
                    if f.read().strip() == "tk8s-supervise":
                        os.kill(parent, signal.SIGTERM)
            except OSError:
                pass
            raise SystemExit(0)
        # 1 ms while a bring-up is on its way (the arguments normally arrive within ~0.1 s, on the
        # critical path), 50 ms once it is clearly not coming (a failed bring-up's leftover)
        time.sleep(0.001 if time.monotonic() < t_fast else 0.05)


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(prog="tk8s-controlplane", description=__doc__.splitlines()[0])
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=8080)
    ap.add_argument("--advertise", default=None, help="address put into URLs handed to agents")
    ap.add_argument("--state-dir", default=None)
    ap.add_argument("--node-grace", type=float, default=float(os.environ.get("TK8S_NODE_GRACE", "5")))
    ap.add_argument("--ready-file", default=None)
    ap.add_argument("--dns-port", type=int, default=None, help="cluster DNS (UDP) port; 0 disables (default 53, "
                    "shifted when not root)")
    ap.add_argument("--ingress-port", type=int, default=None, help="ingress controller port; 0 disables (default 80, "
                    "shifted when not root)")
    a = ap.parse_args(argv)
    cp = ControlPlane(a.host, a.port, a.state_dir, a.node_grace, a.advertise, a.dns_port, a.ingress_port)
    asyncio.run(cp.run(a.ready_file))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
