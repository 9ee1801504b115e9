"""Rancher 1.x environment API of the control plane (what the reference's roles call:
ansible/roles/ranchermaster/tasks/main.yml:29-52, rancherhost/tasks/main.yml:11-34), the KV
rendezvous store and the readiness summary / long-poll (setup.sh:56-85). A mixin of
server.ControlPlane: it uses the store, the routes and the helpers the server sets up.
"""
from __future__ import annotations

import copy
import json
import os
import time

from ..utils.ids import token_hex
from ..utils.trace import trace
from .httpserver import HttpError, Request, Response
from .store import now_iso
from .objects import GPU, TERMINAL, _key, _cond, _set_cond, node_ready, _set_ready, node_validated, pod_gpus


class RancherAPI:
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
        hit = self._require_project_admin(req)  # the server admin sees every environment, an API token its own
        return {"type": "collection", "resourceType": "project",
                "data": [self._public_project(p) for p in self.store.list("projects") if hit[1] in (None, p["id"])]}

    def _public_project(self, p: dict) -> dict:
        return {k: v for k, v in p.items() if k not in ("apiToken",)}

    async def h_project_create(self, req: Request):
        if not self._server_admin(req):  # authn.py: environments are the server administrator's
            raise HttpError(403, "creating an environment needs the server admin token")
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
             "created": now_iso(), "created_seq": self._seq, "apiToken": token_hex(16),
             "links": {"self": f"{self.base}/v2-beta/projects/{pid}"},
             "metadata": {"name": pid}}
        self.store.put("projects", pid, p)
        return Response(201, self._public_project(p))

    async def h_project_get(self, req: Request, pid: str):
        p = self.project(pid)
        self._require_project_admin(req, p["id"])
        return self._public_project(p)

    async def h_project_delete(self, req: Request, pid: str):
        p = self.project(pid)
        self._require_admin(req, p["id"])
        for kind in list(self.store.objs):
            for k in self.store.keys(kind):
                if k.startswith(pid + "/"):
                    self.store.delete(kind, k)
        self.store.delete("projects", p["id"])
        return {"id": pid, "state": "removed"}

    async def h_token_create(self, req: Request):
        pid = req.q("projectId") or req.json().get("projectId")
        p = self.project(pid)
        self._require_admin(req, p["id"])
        tid = self._next_id("1c")
        token = token_hex(20)
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
        self._require_admin(req, t["projectId"])
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
        ntok = token_hex(16)
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
        # the pods already bound to it (the validation DaemonSet's, made by the reconcile above) and
        # the version they are at: the agent starts them and watches from there, no list first
        pods = sorted((self._strip(o) for o in self.store.list(
            "pods", lambda o: o["spec"].get("nodeName") == name and self._in(pid, o))),
            key=lambda o: (o["metadata"].get("namespace", ""), o["metadata"]["name"]))
        return Response(201, {"node": name, "nodeToken": ntok, "projectId": pid, "podCIDR": cidr,
                              "apiPrefix": f"/r/projects/{pid}/kubernetes",
                              "heartbeatSeconds": max(0.2, self.node_grace / 5),
                              "pods": {"resourceVersion": str(self.store.rv), "items": pods}})

    async def h_dashboard(self, req: Request, pid: str):
        p = self.project(pid)
        s = self.summary(p["id"])
        if s["nodes_ready"] == 0:
            return Response(503, "Service Unavailable", content_type="text/plain")
        import html

        esc = html.escape
        rows = "".join(
            f"<tr><td>{esc(n['metadata']['name'])}</td><td>{'Ready' if node_ready(n) else 'NotReady'}</td>"
            f"<td>{n['status']['allocatable'].get(GPU, '0')}</td><td>{'yes' if node_validated(n) else 'no'}</td></tr>"
            for n in self.store.list("nodes", lambda n: self._in(p['id'], n)))
        # the node table is the readiness oracle anyone may poll (setup.sh:66-68); workloads and the
        # deploy form need the environment's token (authn.py), as a header or ?token= for a browser
        hit = self._tokens().get(req.bearer or req.q("token") or "")
        if not (hit is not None and hit[0] == "admin" and hit[1] in (None, p["id"])):
            body = (f"<html><head><title>Kubernetes Dashboard - {esc(p['name'])}</title></head><body>"
                    f"<h1>kubernetes dashboard</h1><p>environment {esc(p['name'])} ({p['id']})</p>"
                    f"<h2>Nodes</h2><table><tr><th>node</th><th>status</th><th>{GPU}</th><th>validated</th></tr>{rows}"
                    "</table><p>Workloads: open this page with <code>?token=</code> the kubeconfig's token.</p>"
                    "</body></html>")
            return Response(200, body, content_type="text/html; charset=utf-8")
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
                "const tok = new URLSearchParams(location.search).get('token');"
                "await fetch('api/v1/appdeployment', {method: 'POST', headers: {'Content-Type': 'application/json',"
                " 'Authorization': 'Bearer ' + tok},"
                " body: JSON.stringify(body)}); location.reload(); });</script>"
                f"<pre>{esc(json.dumps(s, indent=1))}</pre></body></html>")
        return Response(200, body, content_type="text/html; charset=utf-8")

    async def h_app_deploy(self, req: Request, pid: str):
        """The dashboard's "Deploy a containerized app" form (kubernetes-dashboard
        ``POST api/v1/appdeployment``): a Deployment plus, with port mappings, a Service --
        how the reference's walkthrough launched Ghost (docs/detailed.md:261-283). Unlike the
        Rancher 1.x UI the reference used (access control off), it needs the environment's token."""
        import shlex

        p = self.project(pid)
        self._require_admin(req, p["id"])
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
        self._require_admin(req, p["id"])  # it holds the environment's API token
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
        self._require_admin(req, p["id"])
        pods = self.store.list("pods", lambda o: self._in(p["id"], o))
        return {"project": p["id"], "containers": [
            {"name": o["metadata"]["name"], "namespace": o["metadata"].get("namespace"),
             "node": o["spec"].get("nodeName"), "phase": o.get("status", {}).get("phase"),
             "gpus": o["metadata"].get("annotations", {}).get(GPU + "-ids")} for o in pods]}

    # ---- KV -------------------------------------------------------------------------
    # The rendezvous store of multi-process jobs (RCCL unique ids, torch addresses). Keys live in
    # the caller's keyspace, <project>/<namespace>/<key> (authn.kv_key): a pod's ServiceAccount
    # token reaches its own namespace only, so no other tenant can read or overwrite a Job's
    # rendezvous, and the URL a pod uses ($TK8S_KV_URL/<job>/uid) is unchanged.
    async def h_kv_get(self, req: Request, key: str):
        sk = self.kv_key(req, key)
        wait = float(req.q("wait", "0") or 0)
        v = await self.store.wait_until(lambda: self.store.get("kv", sk), min(wait, 120.0))
        if not v:
            raise HttpError(404, f"key {key} not found")
        return Response(200, v["value"], content_type="text/plain")

    async def h_kv_put(self, req: Request, key: str):
        sk = self.kv_key(req, key)
        pid, ns, _ = sk.split("/", 2)
        self.store.put("kv", sk, {"metadata": {"name": key, "namespace": ns}, "_project": pid,
                                  "value": req.body.decode()})
        return Response(201, {"key": key})

    async def h_kv_delete(self, req: Request, key: str):
        self.store.delete("kv", self.kv_key(req, key))
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
        p = self._caller_project(req, req.q("project"))
        s = self.summary(p["id"])
        s["job"] = self._job_state(p["id"], req.q("job"))
        return s

    async def h_cluster_wait(self, req: Request):
        """Long-poll until `nodes` Ready (+validated) with >= `gpus` allocatable (+ job done)."""
        pid = self._caller_project(req, req.q("project"))["id"]
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
        """The store's change feed, filtered to what the caller's token may see (authn.event_filter)."""
        allowed = self.event_filter(req)
        since = int(req.q("resourceVersion", "0") or 0)
        deadline = time.monotonic() + min(float(req.q("timeoutSeconds", "0") or 0), 60.0)
        while True:
            ev = [e for e in self.store.events_since(since, None) if allowed(e["kind"], e["object"])]
            left = deadline - time.monotonic()
            if ev or left <= 0:
                break
            await self.store.wait_change(left)
        return {"resourceVersion": self.store.rv,
                "events": [{"type": e["type"], "kind": e["kind"], "name": e["object"].get("metadata", {}).get("name"),
                            "resourceVersion": e["resourceVersion"]} for e in ev]}

