"""CustomResourceDefinitions (apiextensions.k8s.io/v1) and their custom resources: the API
server's extension point that operators and Helm charts rely on. A mixin of server.ControlPlane.

A CRD (cluster-scoped, named ``<plural>.<group>``) registers a resource: its group, served
versions, plural/singular/kind/listKind/shortNames, scope (Namespaced or Cluster) and whether it
has a ``status`` subresource. From then on its objects are served under
``/apis/<group>/<version>/[namespaces/<ns>/]<plural>[/<name>[/status]]`` by the same generic
handlers as the built-in kinds (list/watch/get/create/update/patch incl. server-side apply/
delete, field selectors, managed fields, RBAC), kept in the store under the kind
``<plural>.<group>``, and listed by discovery (``/apis``, ``/apis/<group>[/<version>]``).
Deleting the CRD deletes its objects. The schema (``openAPIV3Schema``) is stored but not
enforced; ``x-kubernetes-preserve-unknown-fields`` is therefore the effective behaviour.
"""
from __future__ import annotations

from . import k8s_wire
from .httpserver import HttpError, Request
from .objects import _key

CRD_KIND = "customresourcedefinitions"
# built-in kinds with routes of their own (server._routes), never the generic ones
_SPECIAL = {"nodes", "namespaces"}


class CustomResources:
    def _crds(self) -> dict[str, dict]:
        """store kind ``<plural>.<group>`` -> the resource's meta, from the stored CRDs."""
        if getattr(self, "_crd_rv", None) == self.store.rv:
            return self._crd_cache
        out = {}
        for crd in self.store.list(CRD_KIND):
            spec = crd.get("spec") or {}
            names = spec.get("names") or {}
            versions = [v["name"] for v in spec.get("versions") or [] if v.get("served", True)]
            storage = next((v["name"] for v in spec.get("versions") or [] if v.get("storage")), versions[0] if versions else "v1")
            out[f"{names.get('plural')}.{spec.get('group')}"] = {
                "group": spec.get("group"), "versions": versions, "storage": storage, "plural": names.get("plural"),
                "kind": names.get("kind"), "listKind": names.get("listKind") or f"{names.get('kind')}List",
                "singular": names.get("singular") or (names.get("kind") or "").lower(),
                "shortNames": names.get("shortNames") or [], "namespaced": spec.get("scope", "Namespaced") == "Namespaced",
                "status": any((v.get("subresources") or {}).get("status") is not None for v in spec.get("versions") or []),
                "project": crd.get("_project")}
        self._crd_cache, self._crd_rv = out, self.store.rv
        return out

    def _kind_meta(self, kind: str) -> tuple[str, str, bool]:
        """(apiVersion, Kind, namespaced) of a built-in plural or a custom resource's store kind."""
        if kind in k8s_wire.RESOURCES:
            r = k8s_wire.RESOURCES[kind]
            return k8s_wire.group_version(kind), r[2], r[4]
        m = self._crds().get(kind)
        if m is None:
            return "v1", "Status", True
        return f"{m['group']}/{m['storage']}", m["kind"], m["namespaced"]

    def _crd_groups(self) -> dict[str, list[str]]:
        groups: dict[str, list[str]] = {}
        for m in self._crds().values():
            for v in m["versions"]:
                groups.setdefault(m["group"], [])
                if v not in groups[m["group"]]:
                    groups[m["group"]].append(v)
        return groups

    def _crd_resource_list(self, group: str, version: str) -> dict | None:
        res = []
        for m in self._crds().values():
            if m["group"] != group or version not in m["versions"]:
                continue
            res.append({"name": m["plural"], "singularName": m["singular"], "namespaced": m["namespaced"],
                        "kind": m["kind"], "verbs": ["create", "delete", "deletecollection", "get", "list", "patch",
                                                     "update", "watch"], "shortNames": m["shortNames"]})
            if m["status"]:
                res.append({"name": f"{m['plural']}/status", "singularName": "", "namespaced": m["namespaced"],
                            "kind": m["kind"], "verbs": ["get", "patch", "update"]})
        if not res:
            return None
        return {"kind": "APIResourceList", "apiVersion": "v1", "groupVersion": f"{group}/{version}", "resources": res}

    def _admit_crd(self, name: str, body: dict) -> None:
        spec = body.get("spec") or {}
        names = spec.get("names") or {}
        if not spec.get("group") or not names.get("plural") or not names.get("kind") or not spec.get("versions"):
            raise HttpError(422, f'CustomResourceDefinition.apiextensions.k8s.io "{name}" is invalid: spec.group, '
                                 "spec.names.plural, spec.names.kind and spec.versions are required")
        if name != f"{names['plural']}.{spec['group']}":
            raise HttpError(422, f'CustomResourceDefinition.apiextensions.k8s.io "{name}" is invalid: metadata.name: '
                                 f"must be spec.names.plural+\".\"+spec.group ({names['plural']}.{spec['group']})")
        if spec["group"] in {g for g, *_ in k8s_wire.RESOURCES.values()} | {""}:
            raise HttpError(422, f"spec.group: {spec['group']!r} is a built-in API group")
        if sum(1 for v in spec["versions"] if v.get("storage")) != 1:
            raise HttpError(422, "spec.versions: exactly one version must be the storage version")
        body["status"] = {"acceptedNames": dict(names), "storedVersions": [v["name"] for v in spec["versions"] if v.get("storage")],
                          "conditions": [{"type": "NamesAccepted", "status": "True", "reason": "NoConflicts"},
                                         {"type": "Established", "status": "True", "reason": "InitialNamesAccepted"}]}

    def _handler(self, op: str, kind: str, flag: bool = False):
        """The generic handler ``op`` of ``kind`` (k8s_api.py), made once."""
        cache = self.__dict__.setdefault("_handlers", {})
        h = cache.get((op, kind, flag))
        if h is None:
            h = {"list": lambda: self._lister(kind, all_ns=flag), "create": lambda: self._creator(kind),
                 "get": lambda: self._getter(kind), "update": lambda: self._replacer(kind, flag),
                 "delete": lambda: self._deleter(kind)}[op]()
            cache[(op, kind, flag)] = h
        return h

    def _resolve(self, group: str, version: str, plural: str) -> tuple[str, bool, bool] | None:
        """(store kind, namespaced, has a status subresource) of group/version/plural, or None."""
        r = k8s_wire.RESOURCES.get(plural)
        if r is not None and (r[0], r[1]) == (group, version) and plural not in _SPECIAL:
            return plural, r[4], False
        m = self._crds().get(f"{plural}.{group}") if group else None
        if m is not None and version in m["versions"]:
            return f"{plural}.{group}", m["namespaced"], m["status"]
        return None

    async def h_resource(self, req: Request, version: str, rest: str, group: str = "", pid: str | None = None):
        """Every object path that no specific route took: ``[namespaces/<ns>/]<plural>[/<name>
        [/status]]`` of a built-in kind or a custom resource."""
        parts = [x for x in rest.split("/") if x]
        ns = ""
        if len(parts) >= 3 and parts[0] == "namespaces":
            ns, parts = parts[1], parts[2:]
        where = f"{group}/{version}" if group else version
        if not parts or len(parts) > 3:
            raise HttpError(404, f"the server could not find the requested resource ({where} {rest})")
        hit = self._resolve(group, version, parts[0])
        if hit is None:
            raise HttpError(404, f"the server could not find the requested resource ({parts[0]} in {where})")
        kind, namespaced, has_status = hit
        if (namespaced and not ns and not (len(parts) == 1 and req.method == "GET")) or (not namespaced and ns):
            raise HttpError(404, f"{parts[0]} is {'namespaced' if namespaced else 'cluster-scoped'}")
        name = parts[1] if len(parts) > 1 else None
        sub = parts[2] if len(parts) > 2 else None
        if sub is not None and not (sub == "status" and has_status):
            raise HttpError(404, f"the server could not find the requested resource ({parts[0]}/{sub})")
        if name is None:
            if req.method == "GET":
                return await self._handler("list", kind, not ns)(req, pid=pid, ns=ns or None)
            if req.method == "POST":
                return await self._handler("create", kind)(req, ns=ns, pid=pid)
            raise HttpError(405, f"method {req.method} not allowed")
        if sub == "status":
            return await self._status_subresource(req, kind, ns, name, pid)
        op = {"GET": ("get", False), "PUT": ("update", False), "PATCH": ("update", True), "DELETE": ("delete", False)}.get(
            req.method)
        if op is None:
            raise HttpError(405, f"method {req.method} not allowed")
        return await self._handler(op[0], kind, op[1])(req, ns=ns, name=name, pid=pid)

    async def _status_subresource(self, req: Request, kind: str, ns: str, name: str, pid: str | None):
        """``/status`` of a custom resource: only ``status`` changes (a controller's update)."""
        p = self._pid(pid, req)
        cur = self.store.get(kind, _key(p, ns, name))
        if cur is None:
            raise HttpError(404, f'{kind} "{name}" not found')
        if req.method == "GET":
            return self._strip(cur)
        self._auth(req, self.project(p))
        body = req.json()
        from .objects import merge_patch

        st = (body or {}).get("status", {}) if req.method == "PUT" else merge_patch(cur.get("status") or {},
                                                                                 (body or {}).get("status") or {})
        return self._strip(self.store.patch(kind, _key(p, ns, name), lambda o: o.__setitem__("status", st)))
