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
  events; watch = a Kubernetes watch stream (chunked JSON lines, ?watch=true), or long-poll
  batches for tk8s's own clients (?watch=1&batch=1&resourceVersion=N&timeoutSeconds=T).
  Discovery, typed lists, Status errors, field selectors, merge/JSON/strategic patches and
  server-side Tables follow the Kubernetes wire conventions (k8s_wire.py), so a stock kubectl
  works against the kubeconfig.
  Extended resource ``amd.com/gpu`` is scheduled like the AMD k8s-device-plugin exposes it.

Extras: /v1/kv/KEY (rendezvous store, e.g. RCCL unique ids), /v1/cluster/wait (event-driven
readiness, replaces the unbounded 15 s polling loop of setup.sh:59-85), /metrics.

Everything runs on one asyncio loop; the store is the single source of truth. The class is
assembled from mixins: rancher_api.py (environments, registration, KV, readiness), k8s_api.py
(nodes, namespaced kinds, networking, exec), controllers.py (DaemonSets, validation gate, Jobs,
Deployments), scheduler.py (amd.com/gpu-aware binding); objects.py holds the shared helpers.
This module keeps the process: routes, leases, snapshots, the asyncio run loop and main().
"""
from __future__ import annotations

import asyncio
import json
import os
import signal
import sys
import time
from pathlib import Path

from ..utils.net import host_port
from ..utils.trace import trace
from . import k8s_wire
from .controllers import Controllers
from .httpserver import HttpError, HttpServer, Request, Response, Router
from .k8s_api import KubernetesAPI
from .objects import UNREACHABLE, _cond, _key, _set_cond
from .rancher_api import RancherAPI
from .scheduler import Scheduler
from .workloads import Workloads
from .crds import CustomResources
from .metrics_api import MetricsAPI
from .disruption import Disruption
from .priority import Priority
from .webhooks import AdmissionWebhooks
from .podsecurity import PodSecurity
from .store import Store, now_iso
from .authn import Authentication, load_admin_token


_KIND_PLURAL = {r[2]: plural for plural, r in k8s_wire.RESOURCES.items()}


def _tolerates_taint(tol: dict, taint: dict) -> bool:
    from .placement import _tolerates

    return _tolerates(tol, taint)


def _group_doc(group: str, versions: list[str]) -> dict:
    return {"name": group, "versions": [{"groupVersion": f"{group}/{v}", "version": v} for v in versions],
            "preferredVersion": {"groupVersion": f"{group}/{versions[0]}", "version": versions[0]}}


class ControlPlane(Authentication, RancherAPI, KubernetesAPI, Controllers, Workloads, MetricsAPI, CustomResources, Disruption,
                   Priority, AdmissionWebhooks, PodSecurity, Scheduler):
    def __init__(self, host: str, port: int, state_dir: str | None = None, node_grace: float = 5.0,
                 advertise: str | None = None, dns_port: int | None = None, ingress_port: int | None = None):
        self.host, self.port = host, port
        self.advertise = advertise
        self.state_dir = Path(state_dir) if state_dir else None
        self.admin_token = load_admin_token(self.state_dir)  # authn.py: before anything can listen
        self.node_grace = node_grace
        self.store = Store()
        self.store.type_meta = k8s_wire.type_meta()
        self.router = Router()
        from .reqmetrics import RequestMetrics

        self.reqmetrics = RequestMetrics()
        self.http = HttpServer(self.router, on_error=self._log_error, error_body=self._error_body,
                               observe=self.reqmetrics.observe)
        self.leases: dict[str, float] = {}   # node key -> monotonic time of last heartbeat
        self.started = time.time()
        self._stop = None
        self._seq = 0
        self._reconciling = False
        self._again = False
        from .proxy import ServiceProxy

        from .ingress import IngressController

        self.proxy = ServiceProxy(self._endpoints, log=lambda m: self._log_error(m + "\n"), affinity=self._svc_affinity)
        self.ingress = IngressController(self._ingress_routes, self._endpoints, log=lambda m: self._log_error(m + "\n"))
        self.dns_port = host_port(53) if dns_port is None else dns_port          # 0 disables
        self.ingress_port = host_port(80) if ingress_port is None else ingress_port
        self.hpa_period = float(os.environ.get("TK8S_HPA_PERIOD", "15"))  # the HPA controller's sync period
        # how long pods stay on a node whose agent went silent (Kubernetes' default tolerations: 300 s)
        self.pod_eviction_timeout = float(os.environ.get("TK8S_POD_EVICTION_TIMEOUT", "300"))
        self._routes()

    @property
    def _seq(self) -> int:
        """The server's name sequence (generated names, ids): kept with the store, so it survives
        a restart (snapshot + journal) and no name is ever handed out twice."""
        return self.store.meta.get("seq", 0)

    @_seq.setter
    def _seq(self, v: int) -> None:
        self.store.meta["seq"] = v

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
        involved = dict(involved)
        plural = _KIND_PLURAL.get(involved.get("kind", ""))
        if plural:  # what kubectl describe selects an object's events by: kind, name, namespace, uid
            namespaced = k8s_wire.RESOURCES[plural][4]
            obj = self.store.get(plural, _key(project, ns, involved["name"]) if namespaced else _key(project, involved["name"]))
            involved.setdefault("apiVersion", k8s_wire.group_version(plural))
            if namespaced:
                involved.setdefault("namespace", ns)
            if obj is not None:
                involved.setdefault("uid", obj["metadata"].get("uid", ""))
        now = now_iso()
        # the event correlator: the same event again (object, reason, message, type) bumps the
        # count of the first one instead of adding another -- at most one write a second per event
        # (a controller that fails the same way on every reconcile pass cannot flood the store)
        agg = (project, ns, involved.get("kind"), involved.get("name"), involved.get("uid"), reason, message, etype)
        index = self.__dict__.setdefault("_event_index", {})
        hit = index.get(agg)
        if hit is not None:
            ekey, last = hit
            if self.store.get("events", ekey) is not None:
                if time.monotonic() - last >= 1.0:
                    index[agg] = (ekey, time.monotonic())
                    self.store.patch("events", ekey, lambda o: o.update(count=int(o.get("count", 1)) + 1,
                                                                          lastTimestamp=now))
                return
        if len(index) > 10000:
            index.clear()
        index[agg] = (_key(project, ns, name), time.monotonic())
        self.store.put("events", _key(project, ns, name), {
            "kind": "Event", "metadata": {"name": name, "namespace": ns}, "_project": project,
            "involvedObject": involved, "reason": reason, "message": message, "type": etype,
            "firstTimestamp": now, "lastTimestamp": now, "count": 1,
            "source": {"component": "tk8s-controlplane"}, "reportingComponent": "tk8s-controlplane",
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
        """A write to ``project``: its administrator, or a node / ServiceAccount the request's
        authorization (k8s_api._authorize: the Node authorizer, RBAC) already let through."""
        ident = getattr(req, "identity", None)
        if ident is None:
            ident = self._identity(project.get("id"), req.bearer)
        if ident is None:
            raise HttpError(401, "missing or invalid bearer token")

    def _gate(self, h):
        """Every route: authn.PUBLIC paths, or a bearer token the server knows (else 401)."""
        async def g(req: Request, **kw):
            self._authenticate(req)
            return await h(req, **kw)
        g.__name__ = getattr(h, "__name__", "handler")
        return g

    # ---- routes -----------------------------------------------------------------------
    def _routes(self) -> None:
        gate = self._gate

        class _Gated:  # every route behind the authentication gate
            @staticmethod
            def add(method, path, h):
                self.router.add(method, path, gate(h))

        r = _Gated
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
                r.add(method, pre + path, self._guarded(h))
            add("GET", r"/openapi/v3/?", self.h_openapi_root)
            add("GET", r"/openapi/v3/(?P<gv>api/[^/]+|apis/[^/]+/[^/]+)", self.h_openapi_gv)
            add("GET", r"/apis/metrics.k8s.io/v1beta1/?", self.h_metrics_resources)
            add("GET", r"/apis/metrics.k8s.io/v1beta1/nodes", self.h_node_metrics)
            add("GET", r"/apis/metrics.k8s.io/v1beta1/nodes/(?P<name>[^/]+)", self.h_node_metrics)
            add("GET", r"/apis/metrics.k8s.io/v1beta1/pods", self.h_pod_metrics)
            add("GET", r"/apis/metrics.k8s.io/v1beta1/namespaces/(?P<ns>[^/]+)/pods", self.h_pod_metrics)
            add("GET", r"/apis/metrics.k8s.io/v1beta1/namespaces/(?P<ns>[^/]+)/pods/(?P<name>[^/]+)", self.h_pod_metrics)
            add("POST", r"/apis/authorization.k8s.io/v1/selfsubjectaccessreviews", self.h_access_review)
            add("GET", r"/api/?", self.h_api_versions)
            add("GET", r"/apis/?", self.h_api_groups)
            add("GET", r"/api/v1/?", self.h_api_resources)
            add("GET", r"/apis/(?P<group>[^/]+)/?", self.h_api_group)
            add("GET", r"/apis/(?P<group>[^/]+)/(?P<version>[^/]+)/?", self.h_api_resources)
            add("GET", r"/api/v1/nodes", self.h_nodes)
            add("GET", r"/api/v1/nodes/(?P<name>[^/]+)", self.h_node_get)
            add("PUT", r"/api/v1/nodes/(?P<name>[^/]+)/status", self.h_node_status)
            add("PATCH", r"/api/v1/nodes/(?P<name>[^/]+)", self.h_node_patch)
            add("DELETE", r"/api/v1/nodes/(?P<name>[^/]+)", self.h_node_delete)
            add("GET", r"/api/v1/namespaces", self.h_namespaces)
            add("POST", r"/api/v1/namespaces", self.h_namespace_create)
            add("GET", r"/api/v1/namespaces/(?P<name>[^/]+)", self.h_namespace_get)
            add("PATCH", r"/api/v1/namespaces/(?P<name>[^/]+)", self.h_namespace_patch)
            add("DELETE", r"/api/v1/namespaces/(?P<name>[^/]+)", self.h_namespace_delete)
            add("GET", r"/api/v1/pods", self.h_pods)
            for method in ("GET", "PUT", "PATCH"):
                add(method, r"/apis/apps/v1/namespaces/(?P<ns>[^/]+)/(?P<kind>deployments|statefulsets|replicasets)"
                            r"/(?P<name>[^/]+)/scale", self.h_scale)
            add("PUT", r"/api/v1/namespaces/(?P<ns>[^/]+)/pods/(?P<name>[^/]+)/status", self.h_pod_status)
            add("GET", r"/api/v1/namespaces/(?P<ns>[^/]+)/pods/(?P<name>[^/]+)/log", self.h_pod_log)
            add("POST", r"/api/v1/namespaces/(?P<ns>[^/]+)/pods/(?P<name>[^/]+)/exec", self.h_pod_exec)
            add("GET", r"/api/v1/namespaces/(?P<ns>[^/]+)/pods/(?P<name>[^/]+)/exec", self.h_pod_exec_ws)
            add("GET", r"/api/v1/namespaces/(?P<ns>[^/]+)/pods/(?P<name>[^/]+)/portforward", self.h_pod_portforward_ws)
            add("GET", r"/api/v1/namespaces/(?P<ns>[^/]+)/pods/(?P<name>[^/]+)/attach", self.h_pod_attach_ws)
            add("POST", r"/api/v1/namespaces/(?P<ns>[^/]+)/pods/(?P<name>[^/]+)/eviction", self.h_pod_eviction)
            add("POST", r"/api/v1/namespaces/(?P<ns>[^/]+)/serviceaccounts/(?P<name>[^/]+)/token", self.h_token_request)
            add("GET", r"/api/v1/nodes/(?P<node>[^/]+)/execs", self.h_node_execs)
            add("PUT", r"/api/v1/nodes/(?P<node>[^/]+)/execs/(?P<xid>[^/]+)", self.h_exec_result)
            add("GET", r"/api/v1/nodes/(?P<node>[^/]+)/execs/(?P<xid>[^/]+)/stream", self.h_exec_stream)
            # every other object path, built-in kinds (KIND_GROUPS, CLUSTER_KIND_GROUPS) and custom
            # resources alike: two patterns resolved by plural (crds.h_resource), not a regex per
            # kind -- fewer routes to compile at start-up and to scan per request
            for method in ("GET", "POST", "PUT", "PATCH", "DELETE"):
                add(method, r"/api/(?P<version>v1)/(?P<rest>.+)", self.h_resource)
                add(method, r"/apis/(?P<group>[^/]+)/(?P<version>[^/]+)/(?P<rest>.+)", self.h_resource)

    # ---- Kubernetes discovery (k8s_wire.py) ----------------------------------------------
    @staticmethod
    def _error_body(path: str, e: HttpError):
        if k8s_wire.is_k8s_path(path):
            if e.custom_body and isinstance(e.body, dict) and e.body.get("kind") == "Status":
                return e.body  # e.g. a server-side apply conflict with its causes
            return k8s_wire.status_body(e.status, e.message)
        return e.body

    async def h_api_versions(self, req: Request, pid: str | None = None):
        return k8s_wire.api_versions(req.headers.get("host") or f"{self.host}:{self.port}")

    async def h_openapi_root(self, req: Request, pid: str | None = None):
        from . import k8s_openapi

        return k8s_openapi.root(f"/r/projects/{pid}/kubernetes" if pid else "")

    async def h_openapi_gv(self, req: Request, gv: str, pid: str | None = None):
        from . import k8s_openapi

        d = k8s_openapi.document(gv)
        if d is None:
            raise HttpError(404, f"no OpenAPI document for {gv}")
        doc, h = d
        # a hash-addressed document never changes: clients may cache it for good
        return Response(200, doc, headers={"Cache-Control": "public, immutable" if req.q("hash") == h else "no-cache",
                                           "Etag": f'"{h}"'})

    async def h_api_groups(self, req: Request, pid: str | None = None):
        out = k8s_wire.api_group_list()
        for g, versions in sorted(self._crd_groups().items()):  # custom resources' groups (crds.py)
            out["groups"].append(_group_doc(g, versions))
        return out

    async def h_api_group(self, req: Request, group: str, pid: str | None = None):
        g = k8s_wire.api_group(group)
        if g is None and group in self._crd_groups():
            return {"kind": "APIGroup", "apiVersion": "v1", **_group_doc(group, self._crd_groups()[group])}
        if g is None:
            raise HttpError(404, f"the server could not find the requested resource (group {group})")
        return g

    async def h_api_resources(self, req: Request, group: str = "", version: str = "v1", pid: str | None = None):
        if (group, version) == ("metrics.k8s.io", "v1beta1"):
            return await self.h_metrics_resources(req)
        if (group, version) == ("authorization.k8s.io", "v1"):
            return {"kind": "APIResourceList", "apiVersion": "v1", "groupVersion": "authorization.k8s.io/v1", "resources": [
                {"name": "selfsubjectaccessreviews", "singularName": "", "namespaced": False,
                 "kind": "SelfSubjectAccessReview", "verbs": ["create"]}]}
        r = k8s_wire.api_resource_list(group, version) or self._crd_resource_list(group, version)
        if r is None:
            raise HttpError(404, f"the server could not find the requested resource ({group}/{version})")
        return r

    # ---- misc handlers ---------------------------------------------------------------
    async def h_ping(self, req: Request, **_):
        return Response(200, "pong")

    async def h_version(self, req: Request):
        from .. import __version__

        return {"major": "1", "minor": "30", "gitVersion": f"v1.30.0-tk8s{__version__}", "platform": "linux/amd64",
                "tk8sVersion": __version__}

    async def h_metrics(self, req: Request):
        """Prometheus text: the server admin sees every environment and the host-wide series, an
        environment's API token its own environment's; node and ServiceAccount tokens get 403."""
        hit = self._require_project_admin(req)
        if hit[1] is not None:
            return Response(200, "\n".join(self._project_metric_lines(hit[1])) + "\n",
                            content_type="text/plain; version=0.0.4")
        lines = []
        for p in self.store.list("projects"):
            lines += self._project_metric_lines(p["id"])
        lines.append(f"tk8s_store_resource_version {self.store.rv}")
        lines += self.reqmetrics.lines()
        return Response(200, "\n".join(lines) + "\n", content_type="text/plain; version=0.0.4")

    def _project_metric_lines(self, pid: str) -> list[str]:
        s = self.summary(pid)
        lab = f'project="{pid}"'
        lines = [f"tk8s_nodes{{{lab}}} {s['nodes']}", f"tk8s_nodes_ready{{{lab}}} {s['nodes_ready']}",
                 f"tk8s_nodes_validated{{{lab}}} {s['nodes_validated']}",
                 f"tk8s_gpus_capacity{{{lab}}} {s['gpus_capacity']}",
                 f"tk8s_gpus_allocatable{{{lab}}} {s['gpus_allocatable']}",
                 f"tk8s_gpus_in_use{{{lab}}} {s['gpus_in_use']}"]
        for phase, n in s["pods_by_phase"].items():
            lines.append(f'tk8s_pods{{{lab},phase="{phase}"}} {n}')
        now = time.monotonic()
        for k, t in self.leases.items():
            if k.startswith(pid + "/"):
                lines.append(f'tk8s_node_heartbeat_age_seconds{{node="{k}"}} {now - t:.3f}')
        return lines + self._gpu_metric_lines(pid)

    def _gpu_metric_lines(self, pid: str) -> list[str]:
        """Per-GPU telemetry (AMD SMI, as the nodes report it), validation results and pod usage
        of environment ``pid``, in the Prometheus text format -- what a device-metrics exporter
        would scrape."""
        out = []
        for n in self.store.list("nodes", lambda o: o.get("_project") == pid):
            node = n["metadata"]["name"]
            ann = n["metadata"].get("annotations") or {}
            for d in n.get("status", {}).get("devices") or []:
                lab = f'node="{node}",gpu="{d.get("id")}",pci="{d.get("pciBusId", "")}"'
                out.append(f"tk8s_gpu_healthy{{{lab}}} {1 if d.get('health') == 'Healthy' else 0}")
                t = d.get("telemetry") or {}
                for name, v in (("temperature_hotspot_celsius", (t.get("temp_c") or {}).get("hotspot")),
                                ("power_watts", (t.get("power") or {}).get("current_w")),
                                ("vram_used_bytes", t.get("vram_used_bytes")),
                                ("gfx_activity_percent", (t.get("activity") or {}).get("gfx_pct")),
                                ("umc_activity_percent", (t.get("activity") or {}).get("umc_pct")),
                                ("ecc_uncorrectable_total", (t.get("ecc") or {}).get("uncorrectable")),
                                ("ecc_correctable_total", (t.get("ecc") or {}).get("correctable"))):
                    if isinstance(v, (int, float)):
                        out.append(f"tk8s_gpu_{name}{{{lab}}} {v}")
            for key, metric in (("tk8s.amd.com/hbm-write-gbps", "tk8s_validation_hbm_write_gbps"),
                                ("tk8s.amd.com/md5-mbps", "tk8s_validation_md5_mbps"),
                                ("tk8s.amd.com/copy-gbps", "tk8s_validation_copy_gbps")):
                try:
                    out.append(f'{metric}{{node="{node}"}} {float(ann[key])}')
                except (KeyError, ValueError):
                    pass
        for (mpid, node), m in sorted(getattr(self, "metrics", {}).items()):
            if mpid != pid:
                continue
            for key, cs in (m.get("pods") or {}).items():
                ns, pod = key.split("/", 1)
                for c in cs:
                    lab = f'namespace="{ns}",pod="{pod}",container="{c.get("name")}",node="{node}"'
                    out.append(f"tk8s_container_cpu_cores{{{lab}}} {c.get('cpu_cores', 0):.4f}")
                    out.append(f"tk8s_container_memory_bytes{{{lab}}} {int(c.get('memory_bytes', 0))}")
                    if c.get("gpu_pct") is not None:
                        out.append(f"tk8s_container_gpu_busy_percent{{{lab}}} {c['gpu_pct']:.1f}")
        return out

    # ---- node lifecycle ---------------------------------------------------------------
    async def lease_loop(self) -> None:
        period = min(0.25, self.node_grace / 4)
        last = time.monotonic()
        while True:
            await asyncio.sleep(period)
            now = time.monotonic()
            stall = now - last - period
            last = now
            if stall > 0.5:
                # this event loop did not run for a while (a slow admission webhook, a GC pause): the
                # heartbeats that came meanwhile are still queued, so the stall counts for no node
                for key in list(self.leases):
                    self.leases[key] += stall
            changed = False
            for key, t in list(self.leases.items()):
                if now - t > self.node_grace:
                    n = self.store.get("nodes", key)
                    if n is None:
                        self.leases.pop(key, None)
                        continue
                    c = _cond(n, "Ready")
                    if c and c["status"] == "True":
                        self._node_lost(key, f"lease expired after {self.node_grace:.1f}s")
                        changed = True
            changed |= self._taint_manager()
            changed |= self._pod_gc()
            if changed:
                self.reconcile()

    def _node_lost(self, key: str, why: str) -> None:
        """The node lifecycle controller's verdict on a silent agent: Ready=Unknown plus the
        ``node.kubernetes.io/unreachable`` NoSchedule/NoExecute taints (the next heartbeat lifts
        them, objects._set_ready); the taint manager evicts its pods after their toleration."""
        def lost(o):
            _set_cond(o, "Ready", "Unknown", "NodeStatusUnknown", "tk8s agent stopped posting node status")
            kept = [x for x in o.setdefault("spec", {}).get("taints") or [] if x.get("key") != UNREACHABLE]
            o["spec"]["taints"] = kept + [{"key": UNREACHABLE, "effect": e, "timeAdded": now_iso()}
                                          for e in ("NoSchedule", "NoExecute")]

        n = self.store.patch("nodes", key, lost)
        self._event(key.split("/", 1)[0], "default", {"kind": "Node", "name": n["metadata"]["name"]}, "NodeNotReady",
                    why, "Warning")

    def _pod_gc(self) -> bool:
        """Terminating pods whose agent never confirmed (it died, or lost its node): force-deleted
        15 s after their deadline (``metadata.deletionTimestamp``)."""
        import calendar

        now, gone = time.time(), False
        for pod in self.store.list("pods", lambda o: bool(o["metadata"].get("deletionTimestamp"))):
            try:
                deadline = calendar.timegm(time.strptime(pod["metadata"]["deletionTimestamp"], "%Y-%m-%dT%H:%M:%SZ"))
            except ValueError:
                deadline = 0
            nn = pod["spec"].get("nodeName")
            if now > deadline + 15 or (nn and self.store.get("nodes", _key(pod["_project"], nn)) is None):
                self.store.delete("pods", _key(pod["_project"], pod["metadata"]["namespace"], pod["metadata"]["name"]))
                gone = True
        return gone

    def _taint_manager(self) -> bool:
        """Evict pods from nodes with NoExecute taints they do not tolerate: at once for a taint
        the pod has no toleration for, after ``tolerationSeconds`` for one it tolerates for a while.
        The unreachable taint a lost lease adds is tolerated for ``pod_eviction_timeout`` seconds
        (300, as Kubernetes' default tolerations) unless the pod says otherwise. Their controllers
        (Deployment, StatefulSet, Job ...) then re-create them on the nodes that are left."""
        import calendar

        tainted = [n for n in self.store.list("nodes") if any(
            t.get("effect") == "NoExecute" for t in (n.get("spec") or {}).get("taints") or [])]
        if not tainted:
            return False
        now = time.time()
        evicted = False
        for n in tainted:
            pid, nn = n["_project"], n["metadata"]["name"]
            taints = [t for t in n["spec"]["taints"] if t.get("effect") == "NoExecute"]
            for pod in self.store.list("pods", lambda o: o.get("_project") == pid and o["spec"].get("nodeName") == nn
                                       and o.get("status", {}).get("phase") not in ("Succeeded", "Failed")):
                for t in taints:
                    tols = [x for x in pod["spec"].get("tolerations") or [] if _tolerates_taint(x, t)]
                    if not tols and t.get("key") == UNREACHABLE:
                        tols = [{"tolerationSeconds": self.pod_eviction_timeout}]
                    secs = [x.get("tolerationSeconds") for x in tols]
                    if tols and any(s is None for s in secs):
                        continue  # tolerated for good
                    try:
                        added = calendar.timegm(time.strptime(t.get("timeAdded") or "", "%Y-%m-%dT%H:%M:%SZ"))
                    except ValueError:
                        added = now
                    if not tols or now - added >= min(float(s) for s in secs):
                        ns, name = pod["metadata"].get("namespace", "default"), pod["metadata"]["name"]
                        self._delete_pod(pid, ns, name, disruption="DeletionByTaintManager")
                        self._event(pid, ns, {"kind": "Pod", "name": name}, "TaintManagerEviction",
                                    f"Marking for deletion Pod {ns}/{name}: node {nn} has taint {t.get('key')}:NoExecute",
                                    "Warning")
                        evicted = True
                        break
        return evicted

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
        trace("cp", "event loop up")
        if self.state_dir:
            self.state_dir.mkdir(parents=True, exist_ok=True)
            restored = self.store.restore(self.state_dir / "controlplane.json")
            replayed = self.store.open_journal(self.state_dir / "controlplane.journal")
            if restored or replayed:
                now = time.monotonic()
                for key in self.store.keys("nodes"):
                    self.leases[key] = now  # grace period for agents to resume heartbeats
                # names the server derives from its sequence never repeat one it handed out before
                self._seq = max(self._seq, self.store.rv) + 1000
        self._ensure_templates()
        trace("cp", "state ready")
        host, port = await self.http.start(self.host, self.port)
        self.port = port
        if self.store.keys("services"):
            await self.proxy.sync(self._proxy_wanted())  # services restored from a snapshot
        if self.store.keys("ingresses") and self.ingress_port:
            await self.ingress.ensure(self.advertise or self.host, self.ingress_port, True)

        tasks = [asyncio.create_task(self.lease_loop()), asyncio.create_task(self.snapshot_loop()),
                 asyncio.create_task(self.cron_loop()), asyncio.create_task(self.hpa_loop())]
        # Mirrors the rancher/server log line the reference waits for (ranchermaster:14-20).
        print(f"Listening on {host}:{port}", flush=True)
        trace("cp", "listening")
        if ready_file:
            from ..utils.fsutil import atomic_write_json

            atomic_write_json(ready_file, {"host": host, "port": port, "pid": os.getpid(), "base": self.base,
                                           "adminToken": self.admin_token})  # 0600, like every atomic_write
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
        loop.call_soon(_warm_up)
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


def _warm_up() -> None:
    """What the first authorised write of a bring-up imports (RBAC's request attributes, managed
    fields), loaded in the idle moment after "Listening on" rather than inside that request."""
    from . import rbac, ssa  # noqa: F401


def await_args(path: str, timeout: float | None = None) -> list[str]:
    """Zygote mode: wait for the JSON argument list (orchestrator._boot_controlplane writes it
    atomically). A zygote nobody hands arguments to -- the bring-up failed before its master
    existed -- stops its supervisor and exits, so it never lingers or restarts."""
    from ..utils.zygote import await_json

    return [str(a) for a in await_json(path, timeout, want=list)]


_OPTS = {"--host": ("host", str, "127.0.0.1"), "--port": ("port", int, 8080), "--advertise": ("advertise", str, None),
         "--state-dir": ("state_dir", str, None), "--ready-file": ("ready_file", str, None),
         "--node-grace": ("node_grace", float, None), "--dns-port": ("dns_port", int, None),
         "--ingress-port": ("ingress_port", int, None)}


def _parse_fast(argv: list[str]) -> dict | None:
    """The daemon's ``--opt value`` arguments without argparse (~2 ms of its start); None for
    anything else (``--help``, ``--opt=value``, an unknown option), which argparse then handles."""
    out = {dest: default for dest, _, default in _OPTS.values()}
    out["node_grace"] = float(os.environ.get("TK8S_NODE_GRACE", "5"))
    if len(argv) % 2:
        return None
    for flag, val in zip(argv[::2], argv[1::2]):
        if flag not in _OPTS:
            return None
        dest, typ, _ = _OPTS[flag]
        try:
            out[dest] = typ(val)
        except ValueError:
            return None
    return out


def main(argv: list[str] | None = None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    from .. import shortcut_on

    a = _parse_fast(argv) if shortcut_on("TK8S_FAST_ARGS") else None
    if a is None:
        import argparse

        ap = argparse.ArgumentParser(prog="tk8s-controlplane", description=__doc__.splitlines()[0])
        ap.add_argument("--host", default="127.0.0.1")
        ap.add_argument("--port", type=int, default=8080)
        ap.add_argument("--advertise", default=None, help="address put into URLs handed to agents")
        ap.add_argument("--state-dir", default=None)
        ap.add_argument("--node-grace", type=float, default=float(os.environ.get("TK8S_NODE_GRACE", "5")))
        ap.add_argument("--ready-file", default=None)
        ap.add_argument("--dns-port", type=int, default=None, help="cluster DNS (UDP) port; 0 disables (default 53, "
                        "shifted when not root)")
        ap.add_argument("--ingress-port", type=int, default=None, help="ingress controller port; 0 disables (default "
                        "80, shifted when not root)")
        a = vars(ap.parse_args(argv))
    cp = ControlPlane(a["host"], a["port"], a["state_dir"], a["node_grace"], a["advertise"], a["dns_port"],
                      a["ingress_port"])
    trace("cp", "constructed")
    asyncio.run(cp.run(a["ready_file"]))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
