"""Dynamic admission control: MutatingWebhookConfigurations and ValidatingWebhookConfigurations
(admissionregistration.k8s.io/v1, cluster-scoped). A mixin of server.ControlPlane.

On a create or update (and, for validating webhooks, a delete) of an object that a webhook's
``rules`` match -- operations, apiGroups, apiVersions, resources (``*``, ``<plural>``,
``<plural>/<sub>``), scope -- and whose namespace and labels its ``namespaceSelector`` and
``objectSelector`` select, the API server POSTs an ``admission.k8s.io/v1`` AdmissionReview to the
webhook and acts on the answer: ``allowed: false`` refuses the request with the webhook's status
(403 by default), a mutating webhook's ``patchType: JSONPatch`` patch is applied to the object.
Mutating webhooks run first, in order, then the built-in admission, then the validating ones --
Kubernetes' order. ``failurePolicy`` (``Fail`` by default) decides what an unreachable or broken
webhook means, ``timeoutSeconds`` (default 10, at most 30) bounds the call, and ``dryRun``
requests go only to ``sideEffects: None|NoneOnDryRun`` webhooks.

``clientConfig.url`` is called as given; ``clientConfig.service`` is resolved to a Ready pod
behind the Service (its Endpoints) and called directly -- not through the Service proxy, which
runs on this server's own event loop. HTTPS verifies the server against ``caBundle`` (the host
name is not checked when a pod is called by its IP).

The call is made on the control plane's event loop, so a webhook holds every other request for
as long as it takes (``timeoutSeconds``): keep webhooks fast. The node lease loop forgives such a
stall (server.lease_loop), so a slow webhook cannot mark heartbeating nodes lost.
"""
from __future__ import annotations

import contextvars
import json

from .httpserver import HttpError
from .objects import _key

MUTATING = "mutatingwebhookconfigurations"
VALIDATING = "validatingwebhookconfigurations"
CALLER: contextvars.ContextVar = contextvars.ContextVar("tk8s_caller", default=None)  # (pid, bearer)
# admission warnings of the current request (webhook warnings, PodSecurity warn level): Warning headers
WARNINGS: contextvars.ContextVar = contextvars.ContextVar("tk8s_warnings", default=None)


def warn(text: str) -> None:
    w = WARNINGS.get()
    if w is not None:
        w.append(text)


def _match_rule(rule: dict, op: str, group: str, version: str, resource: str, namespaced: bool) -> bool:
    ops = rule.get("operations") or []
    if "*" not in ops and op not in ops:
        return False
    if not any(g in ("*", group) for g in rule.get("apiGroups") or []):
        return False
    if not any(v in ("*", version) for v in rule.get("apiVersions") or []):
        return False
    if not any(r in ("*", resource, "*/*") for r in rule.get("resources") or []):
        return False
    scope = rule.get("scope", "*")
    return scope == "*" or (scope == "Namespaced") == namespaced


class AdmissionWebhooks:
    def _user_info(self) -> dict:
        caller = CALLER.get()
        who = self._identity(*caller) if caller else None
        if who is None:
            return {"username": "system:anonymous", "groups": ["system:unauthenticated"]}
        if who == "admin":
            return {"username": "tk8s:admin", "groups": ["system:masters", "system:authenticated"]}
        if who.startswith("node:"):
            return {"username": f"system:node:{who[5:]}", "groups": ["system:nodes", "system:authenticated"]}
        _sa, ns, name = who.split(":", 2)
        return {"username": f"system:serviceaccount:{ns}:{name}",
                "groups": ["system:serviceaccounts", f"system:serviceaccounts:{ns}", "system:authenticated"]}

    def _webhook_target(self, pid: str, cc: dict) -> str:
        if cc.get("url"):
            return cc["url"]
        svc = cc.get("service") or {}
        ns, name = svc.get("namespace", "default"), svc.get("name", "")
        o = self.store.get("services", _key(pid, ns, name))
        if o is None:
            raise OSError(f'service "{ns}/{name}" not found')
        want = int(svc.get("port", 443))
        sp = next((p for p in o["spec"].get("ports") or [] if int(p.get("port", 0)) == want), None)
        if sp is None:
            raise OSError(f'service "{ns}/{name}" has no port {want}')
        for pod in self.store.list("pods", lambda x: x.get("_project") == pid and x["metadata"].get("namespace") == ns):
            if (pod.get("status") or {}).get("phase") != "Running" or not pod["status"].get("podIP"):
                continue
            if not _sel({"matchLabels": o["spec"].get("selector") or {}}, pod["metadata"].get("labels")):
                continue
            tp = sp.get("targetPort", sp["port"])
            if isinstance(tp, str) and not tp.isdigit():
                tp = next((cp.get("containerPort") for c in pod["spec"].get("containers", [])
                           for cp in c.get("ports") or [] if cp.get("name") == tp), None)
            if tp:
                return f"https://{pod['status']['podIP']}:{tp}{svc.get('path') or '/'}"
        raise OSError(f'service "{ns}/{name}" has no ready endpoints')

    @staticmethod
    def _post_review(url: str, review: dict, cc: dict, timeout: float) -> dict:
        import http.client
        from urllib.parse import urlsplit

        import base64

        u = urlsplit(url)
        body = json.dumps(review).encode()
        if u.scheme == "https":
            import sys

            if "ssl" in sys.modules and sys.modules["ssl"] is None:
                del sys.modules["ssl"]  # __main__ kept ssl off the start-up path; an HTTPS webhook needs it
            import ssl

            ctx = ssl.create_default_context(cadata=base64.b64decode(cc["caBundle"]).decode()) if cc.get("caBundle") \
                else ssl.create_default_context()
            if not cc.get("url"):
                ctx.check_hostname = False  # a pod by IP: the certificate is checked, the name is not
            import socket

            # (http.client may have been imported without ssl: wrap the socket ourselves)
            conn = http.client.HTTPConnection(u.hostname, u.port or 443, timeout=timeout)
            conn.sock = ctx.wrap_socket(socket.create_connection((u.hostname, u.port or 443), timeout=timeout),
                                        server_hostname=u.hostname)
        else:
            conn = http.client.HTTPConnection(u.hostname, u.port or 80, timeout=timeout)
        try:
            conn.request("POST", (u.path or "/") + (f"?{u.query}" if u.query else ""), body=body,
                         headers={"Content-Type": "application/json", "Accept": "application/json"})
            r = conn.getresponse()
            data = r.read()
            if r.status != 200:
                raise OSError(f"HTTP {r.status}")
            return json.loads(data)
        finally:
            conn.close()

    def _admit_webhooks(self, pid: str, op: str, kind: str, ns: str, name: str, obj: dict | None, old: dict | None,
                        mutating: bool, dry_run: bool = False, sub: str = "") -> dict | None:
        """Run the matching webhooks of one phase; the (possibly mutated) object."""
        store_kind = MUTATING if mutating else VALIDATING
        if kind in (MUTATING, VALIDATING) or not self.store.keys(store_kind):
            return obj
        api_version, kind_name, namespaced = self._kind_meta(kind)
        group, _, version = api_version.rpartition("/")
        resource = kind.split(".")[0] + (f"/{sub}" if sub else "")
        target = obj if obj is not None else old
        labels = ((target or {}).get("metadata") or {}).get("labels") or {}
        ns_labels = {}
        if ns:
            nso = self.store.get("namespaces", _key(pid, ns))
            ns_labels = {**(((nso or {}).get("metadata") or {}).get("labels") or {}), "kubernetes.io/metadata.name": ns}
        for cfg in sorted(self.store.list(store_kind, lambda o: self._in(pid, o)), key=lambda o: o["metadata"]["name"]):
            for wh in cfg.get("webhooks") or []:
                if not any(_match_rule(r, op, group, version, resource, namespaced) for r in wh.get("rules") or []):
                    continue
                if ns and not _sel(wh.get("namespaceSelector"), ns_labels):
                    continue
                if not _sel(wh.get("objectSelector"), labels):
                    continue
                if dry_run and wh.get("sideEffects", "None") not in ("None", "NoneOnDryRun"):
                    raise HttpError(400, f'admission webhook "{wh.get("name")}" does not support dry run')
                import uuid  # (off the control plane's start-up path)

                uid = str(uuid.uuid4())
                review = {"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview", "request": {
                    "uid": uid, "kind": {"group": group, "version": version, "kind": kind_name},
                    "resource": {"group": group, "version": version, "resource": kind.split(".")[0]},
                    "requestKind": {"group": group, "version": version, "kind": kind_name},
                    "requestResource": {"group": group, "version": version, "resource": kind.split(".")[0]},
                    **({"subResource": sub} if sub else {}), "name": name, "namespace": ns, "operation": op,
                    "userInfo": self._user_info(), "object": obj, "oldObject": old, "dryRun": dry_run,
                    "options": {"apiVersion": "meta.k8s.io/v1", "kind": f"{op.capitalize()}Options"}}}
                cc = wh.get("clientConfig") or {}
                try:
                    url = self._webhook_target(pid, cc)
                    out = self._post_review(url, review, cc, min(float(wh.get("timeoutSeconds", 10)), 30.0))
                    resp = out.get("response") or {}
                    if resp.get("uid") != uid:
                        raise OSError("the response's uid does not match the request's")
                except (OSError, ValueError) as e:
                    if wh.get("failurePolicy", "Fail") == "Ignore":
                        continue
                    raise HttpError(500, f'Internal error occurred: failed calling webhook "{wh.get("name")}": {e}') from e
                for w in resp.get("warnings") or []:
                    warn(str(w))
                if not resp.get("allowed"):
                    st = resp.get("status") or {}
                    code = int(st.get("code") or 403)
                    msg = st.get("message") or "denied the request"
                    raise HttpError(code, f'admission webhook "{wh.get("name")}" denied the request: {msg}')
                if mutating and resp.get("patch"):
                    import base64

                    if resp.get("patchType", "JSONPatch") != "JSONPatch":
                        raise HttpError(500, f'admission webhook "{wh.get("name")}": unsupported patchType')
                    from . import k8s_wire

                    try:
                        obj = k8s_wire.json_patch(obj, json.loads(base64.b64decode(resp["patch"])))
                    except (k8s_wire.PatchError, ValueError) as e:
                        raise HttpError(500, f'admission webhook "{wh.get("name")}" returned a bad patch: {e}') from e
        return obj


def _sel(sel, labels) -> bool:
    from .placement import selector_matches  # (lazy: off the control plane's start-up imports)

    return selector_matches(sel, labels)
