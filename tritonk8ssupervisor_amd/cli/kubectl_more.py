"""The rest of the everyday kubectl verbs (cli/kubectl.py dispatches here): ``run``, ``set
image|env|resources``, ``autoscale``, ``patch``, ``replace``, ``edit``, ``diff``, ``events``,
``explain``, ``api-resources``, ``api-versions``, ``auth can-i``, ``config
view|current-context|get-contexts`` and ``rollout pause|resume``.

All of them are plain API calls a stock kubectl makes too -- discovery, OpenAPI v3,
SelfSubjectAccessReview, dry-run server-side apply for ``diff`` -- so they work the same against
the tk8s control plane and against any other Kubernetes API server.
"""
from __future__ import annotations

import difflib
import json
import os
import shlex
import subprocess
import sys
import tempfile
import time

import yaml

from ..controlplane.client import ApiError
from ..kube import KINDS, collection_path, kind_key, object_path

VERBS = ("run", "set", "autoscale", "patch", "replace", "edit", "diff", "events", "explain", "api-resources",
         "api-versions", "auth", "config", "kustomize")
_WORKLOADS = ("deployment", "statefulset", "daemonset", "replicaset", "job", "pod")


def _split_target(args: list[str]) -> tuple[str, str, list[str]]:
    """TYPE/NAME rest... or TYPE NAME rest...  ->  (kind key, name, rest)."""
    if not args:
        raise SystemExit("error: a resource is required (TYPE/NAME or TYPE NAME)")
    if "/" in args[0]:
        what, name = args[0].split("/", 1)
        return kind_key(what), name, args[1:]
    if len(args) < 2:
        raise SystemExit("error: a resource name is required")
    return kind_key(args[0]), args[1], args[2:]


def _path(k, kind: str, name: str, ns: str) -> str:
    return k.k8s(f"/api/v1/nodes/{name}" if kind == "node" else f"/api/v1/namespaces/{name}" if kind == "namespace"
                 else object_path(kind, name, ns))


def _pod_spec(obj: dict) -> dict:
    return obj["spec"] if obj.get("kind") == "Pod" else obj["spec"].setdefault("template", {}).setdefault("spec", {})


def _kv_list(pairs: list[str]) -> dict[str, str]:
    out = {}
    for p in pairs:
        for item in p.split(","):
            if item:
                key, _, val = item.partition("=")
                out[key] = val
    return out


def _dump(obj: dict, output: str | None) -> str:
    obj = {**obj, "metadata": {k: v for k, v in obj.get("metadata", {}).items() if k != "managedFields"}}
    return json.dumps(obj, indent=2) if output == "json" else yaml.safe_dump(obj, sort_keys=False).rstrip()


# ---- run / set / autoscale -------------------------------------------------------------------
def _run(k, a, ns: str) -> int:
    """kubectl run NAME --image=IMG [--env K=V] [--port P] [--labels k=v] [--restart Never|OnFailure|Always]
    [--limits amd.com/gpu=1,cpu=2] [--command] [-i] [-t] [--rm] [-- ARGS...]: one Pod labelled run=NAME.
    ``-i`` starts the container with ``stdin: true, stdinOnce: true`` and ``-t`` with ``tty: true``;
    either attaches this terminal once the pod runs (``kubectl_streams.attach_interactive``) and
    returns the container's exit code; ``--rm`` deletes the pod after the session."""
    if not a.args or not a.image:
        raise SystemExit("usage: kubectl run NAME --image=IMAGE [--env K=V] [--port P] [--limits R=Q] [-- ARGS...]")
    name = a.args[0]
    c = {"name": name, "image": a.image}
    if a.command:
        c["command" if a.command_flag else "args"] = list(a.command)
    if a.env:
        c["env"] = [{"name": key, "value": val} for key, val in _kv_list(a.env).items()]
    if a.port:
        c["ports"] = [{"containerPort": a.port}]
    if a.stdin:
        c["stdin"] = c["stdinOnce"] = True
    if a.tty:
        c["tty"] = True
    if a.rm and not (a.stdin or a.tty):
        raise SystemExit("error: --rm should only be used for attached containers")
    if a.limits or a.requests:
        c["resources"] = {**({"limits": _kv_list([a.limits])} if a.limits else {}),
                          **({"requests": _kv_list([a.requests])} if a.requests else {})}
    labels = _kv_list([a.labels]) if a.labels else {"run": name}
    pod = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "labels": labels},
           "spec": {"containers": [c], "restartPolicy": a.restart or "Always"}}
    if a.dry_run == "client":
        print(_dump(pod, a.output or "yaml"))
        return 0
    query = {"dryRun": "All"} if a.dry_run == "server" else None
    k.request("POST", k.k8s(collection_path("pod", ns)), body=pod, query=query)
    if query or not (a.stdin or a.tty):
        print(f"pod/{name} created" + (" (server dry run)" if query else ""))
        return 0
    return _run_attached(k, a, ns, name)


def _run_attached(k, a, ns: str, name: str) -> int:
    """`kubectl run -i/-t`: wait (up to a minute) for the pod to run, attach, and return the
    container's exit code; a pod that ended before the attach prints its log instead, like kubectl."""
    from .kubectl_streams import attach_interactive

    path = k.k8s(object_path("pod", name, ns))
    code, phase, st, deadline = 1, None, {}, time.time() + 60.0
    try:
        while time.time() < deadline:
            st = k.get(path).get("status") or {}
            phase = st.get("phase")
            if phase in ("Running", "Succeeded", "Failed"):
                break
            time.sleep(0.1)
        if phase == "Running":
            code = attach_interactive(k, ns, name, a.stdin, a.tty, name)
            for _ in range(50):  # the agent reports the end a moment after the session's Status
                st = k.get(path).get("status") or {}
                if st.get("phase") != "Running":
                    break
                time.sleep(0.1)
            phase = st.get("phase")
        elif phase in ("Succeeded", "Failed"):
            sys.stdout.write(k.get(path + "/log", raw=True))
        if phase in ("Succeeded", "Failed"):
            term = next(((cs.get("state") or {}).get("terminated") for cs in st.get("containerStatuses") or []
                         if (cs.get("state") or {}).get("terminated")), None)
            code = int(term.get("exitCode", 1)) if term else (0 if phase == "Succeeded" else 1)
        elif phase != "Running":
            print(f"error: timed out waiting for pod {name} to run (phase {phase})", file=sys.stderr)
    finally:
        if a.rm:
            try:
                k.request("DELETE", path)
                print(f'pod "{name}" deleted', file=sys.stderr)
            except ApiError as e:
                print(f"error: deleting pod {name}: {e}", file=sys.stderr)
    return code


def _set(k, a, ns: str) -> int:
    """kubectl set image TYPE/NAME C=IMG...  |  set env TYPE/NAME K=V... K-  |  set resources TYPE/NAME
    [-c C] --limits=R=Q,... --requests=R=Q,...   (a changed pod template rolls the workload out)."""
    sub = a.args[0] if a.args else ""
    if sub not in ("image", "env", "resources"):
        raise SystemExit("usage: kubectl set image|env|resources TYPE/NAME ...")
    kind, name, rest = _split_target(a.args[1:])
    if kind not in _WORKLOADS:
        raise SystemExit(f"error: cannot set {sub} on {kind}")
    path = _path(k, kind, name, ns)
    obj = k.get(path)
    containers = _pod_spec(obj).get("containers") or []
    picked = [c for c in containers if not a.container or c["name"] == a.container]
    if sub == "image":
        want = _kv_list(rest)
        for key in want:
            if key != "*" and not any(c["name"] == key for c in containers):
                raise SystemExit(f'error: unable to find container named "{key}"')
        for c in containers:
            if c["name"] in want or "*" in want:
                c["image"] = want.get(c["name"], want.get("*"))
    elif sub == "env":
        for c in picked:
            env = {e["name"]: e for e in c.get("env") or []}
            for item in rest:
                if item.endswith("-") and "=" not in item:
                    env.pop(item[:-1], None)
                else:
                    key, _, val = item.partition("=")
                    env[key] = {"name": key, "value": val}
            c["env"] = list(env.values())
    else:
        for c in picked:
            res = c.setdefault("resources", {})
            if a.limits:
                res.setdefault("limits", {}).update(_kv_list([a.limits]))
            if a.requests:
                res.setdefault("requests", {}).update(_kv_list([a.requests]))
    k.request("PUT", path, body=obj)
    print(f"{kind}/{name} {'image updated' if sub == 'image' else sub + ' updated'}")
    return 0


def _autoscale(k, a, ns: str) -> int:
    """kubectl autoscale deployment NAME --max N [--min M] [--cpu-percent P]: an autoscaling/v2 HPA."""
    kind, name, _rest = _split_target(a.args)
    if kind not in ("deployment", "statefulset", "replicaset") or not a.max:
        raise SystemExit("usage: kubectl autoscale deployment NAME --max N [--min M] [--cpu-percent P]")
    hpa = {"apiVersion": "autoscaling/v2", "kind": "HorizontalPodAutoscaler", "metadata": {"name": a.name or name},
           "spec": {"scaleTargetRef": {"apiVersion": "apps/v1", "kind": KINDS[kind][0], "name": name},
                    "minReplicas": a.min or 1, "maxReplicas": a.max,
                    "metrics": [{"type": "Resource", "resource": {"name": "cpu", "target": {
                        "type": "Utilization", "averageUtilization": a.cpu_percent or 80}}}]}}
    k.post(k.k8s(collection_path("horizontalpodautoscaler", ns)), hpa)
    print(f"horizontalpodautoscaler.autoscaling/{a.name or name} autoscaled")
    return 0


# ---- patch / replace / edit / diff -----------------------------------------------------------
_PATCH_TYPES = {"strategic": "application/strategic-merge-patch+json", "merge": "application/merge-patch+json",
                "json": "application/json-patch+json"}


def _patch(k, a, ns: str) -> int:
    """kubectl patch TYPE NAME -p PATCH [--type strategic|merge|json]."""
    kind, name, _rest = _split_target(a.args)
    if not a.patch:
        raise SystemExit("usage: kubectl patch TYPE NAME -p PATCH [--type strategic|merge|json]")
    ptype = a.type if a.type in _PATCH_TYPES else "strategic"
    try:
        body = json.loads(a.patch)
    except json.JSONDecodeError:
        body = yaml.safe_load(a.patch)
    before = k.get(_path(k, kind, name, ns))
    after = k.request("PATCH", _path(k, kind, name, ns), body=body, content_type=_PATCH_TYPES[ptype])
    same = {**before, "metadata": {}} == {**after, "metadata": {}}
    print(f"{kind}/{name} {'patched (no change)' if same else 'patched'}")
    return 0


def _objects(a) -> list[dict]:
    from .kubectl import _manifests

    return _manifests(a)


def _kustomize(a) -> int:
    """kubectl kustomize DIR: the built objects as one YAML stream."""
    from .. import kustomize

    try:
        objs = kustomize.build(a.args[0] if a.args else ".")
    except kustomize.KustomizeError as e:
        raise SystemExit(f"error: {e}") from e
    print("\n---\n".join(yaml.safe_dump(o, sort_keys=False).rstrip() for o in objs))
    return 0


def _replace(k, a, ns: str) -> int:
    """kubectl replace -f FILE|-k DIR: PUT each object (it must exist)."""
    for obj in _objects(a):
        kind, name = kind_key(obj["kind"]), obj["metadata"]["name"]
        path = _path(k, kind, name, obj["metadata"].get("namespace", ns))
        cur = k.get(path)
        obj.setdefault("metadata", {})["resourceVersion"] = cur["metadata"].get("resourceVersion")
        k.request("PUT", path, body=obj)
        print(f"{kind}/{name} replaced")
    return 0


def _strip_volatile(obj: dict) -> dict:
    md = {k: v for k, v in (obj.get("metadata") or {}).items()
          if k not in ("managedFields", "resourceVersion", "generation", "uid", "creationTimestamp")}
    return {**{k: v for k, v in obj.items() if k != "status"}, "metadata": md}


def _diff(k, a, ns: str) -> int:
    """kubectl diff -f FILE: live objects against what a server-side dry-run apply would make of
    them, as a unified YAML diff. Exit 0 without differences, 1 with."""
    from ..controlplane.k8s_wire import APPLY_PATCH

    changed = False
    for obj in _objects(a):
        kind, name = kind_key(obj["kind"]), obj["metadata"]["name"]
        path = _path(k, kind, name, obj["metadata"].get("namespace", ns))
        try:
            live = k.get(path)
        except ApiError as e:
            if e.status != 404:
                raise
            live = None
        merged = k.request("PATCH", path, body=obj, content_type=APPLY_PATCH,
                           query={"fieldManager": "kubectl", "force": "true", "dryRun": "All"})
        old = yaml.safe_dump(_strip_volatile(live), sort_keys=True).splitlines(keepends=True) if live else []
        new = yaml.safe_dump(_strip_volatile(merged), sort_keys=True).splitlines(keepends=True)
        lines = list(difflib.unified_diff(old, new, f"live/{kind}/{name}", f"merged/{kind}/{name}"))
        if lines:
            changed = True
            sys.stdout.writelines(lines)
    return 1 if changed else 0


def _edit(k, a, ns: str) -> int:
    """kubectl edit TYPE/NAME: the object as YAML in $KUBE_EDITOR / $EDITOR (vi), PUT back if changed."""
    kind, name, _rest = _split_target(a.args)
    path = _path(k, kind, name, ns)
    obj = k.get(path)
    text = _dump(obj, a.output if a.output == "json" else "yaml") + "\n"
    editor = os.environ.get("KUBE_EDITOR") or os.environ.get("EDITOR") or "vi"
    with tempfile.NamedTemporaryFile("w", suffix=".yaml", prefix=f"kubectl-edit-{name}-", delete=False) as f:
        f.write(text)
    try:
        if subprocess.run([*shlex.split(editor), f.name]).returncode != 0:
            print("error: the editor exited with an error; nothing changed", file=sys.stderr)
            return 1
        with open(f.name) as g:
            edited = g.read()
    finally:
        os.unlink(f.name)
    if edited == text:
        print("Edit cancelled, no changes made.")
        return 0
    new = yaml.safe_load(edited)
    new.setdefault("metadata", {})["resourceVersion"] = obj["metadata"].get("resourceVersion")
    k.request("PUT", path, body=new)
    print(f"{kind}/{name} edited")
    return 0


# ---- events / explain / discovery / auth / config --------------------------------------------
def _events(k, a, ns: str) -> int:
    """kubectl events [--for TYPE/NAME] [-A]: oldest first, as kubectl events lists them."""
    path = "/api/v1/events" if a.all_namespaces else f"/api/v1/namespaces/{ns}/events"
    items = k.get(k.k8s(path))["items"]
    if a.for_:
        what, _, name = a.for_.partition("/")
        kind = KINDS.get(kind_key(what), (what.capitalize(),))[0] if kind_key(what) not in ("node",) else "Node"
        items = [e for e in items if (e.get("involvedObject") or {}).get("name") == name
                 and (e.get("involvedObject") or {}).get("kind") == kind]
    items.sort(key=lambda e: e.get("lastTimestamp") or e.get("eventTime") or e["metadata"].get("creationTimestamp") or "")
    rows = [["LAST SEEN", "TYPE", "REASON", "OBJECT", "MESSAGE"]]
    now = time.time()
    for e in items:
        ts = e.get("lastTimestamp") or e["metadata"].get("creationTimestamp")
        try:
            age = max(0, int(now - time.mktime(time.strptime(ts, "%Y-%m-%dT%H:%M:%SZ")) + time.timezone))
            seen = f"{age}s" if age < 120 else f"{age // 60}m"
        except (TypeError, ValueError):
            seen = "<unknown>"
        io = e.get("involvedObject") or {}
        rows.append([seen, e.get("type", "Normal"), e.get("reason", ""), f"{io.get('kind', '').lower()}/{io.get('name', '')}",
                     e.get("message", "")])
    if len(rows) == 1:
        print(f"No events found in {ns} namespace." if not a.all_namespaces else "No events found.")
        return 0
    widths = [max(len(str(r[i])) for r in rows) for i in range(4)]
    for r in rows:
        print("   ".join(str(c).ljust(w) for c, w in zip(r[:4], widths)) + "   " + str(r[4]))
    return 0


def _resources(k) -> list[tuple[str, dict]]:
    """(groupVersion, resource) of every served resource, core first."""
    out = [("v1", r) for r in k.get(k.k8s("/api/v1"))["resources"]]
    for g in k.get(k.k8s("/apis"))["groups"]:
        gv = g["preferredVersion"]["groupVersion"]
        try:
            out += [(gv, r) for r in k.get(k.k8s(f"/apis/{gv}"))["resources"]]
        except ApiError:
            continue
    return out


def _api_resources(k, a) -> int:
    rows = [["NAME", "SHORTNAMES", "APIVERSION", "NAMESPACED", "KIND"]]
    for gv, r in _resources(k):
        if "/" in r["name"]:
            continue
        if a.namespaced is not None and r.get("namespaced") != (a.namespaced == "true"):
            continue
        if a.output == "name":
            print(r["name"] + ("" if "/" not in gv else "." + gv.split("/")[0]))
            continue
        rows.append([r["name"], ",".join(r.get("shortNames") or []), gv, str(r.get("namespaced")).lower(), r["kind"]])
    if a.output != "name":
        widths = [max(len(x[i]) for x in rows) for i in range(5)]
        for r in rows:
            print("   ".join(c.ljust(w) for c, w in zip(r, widths)).rstrip())
    return 0


def _api_versions(k) -> int:
    print("\n".join(sorted({gv for gv, _ in _resources(k)} | {"v1"})))
    return 0


def _find_resource(k, word: str) -> tuple[str, dict]:
    w = word.lower()
    for gv, r in _resources(k):
        if "/" not in r["name"] and w in {r["name"], r.get("singularName", ""), r["kind"].lower(), *(r.get("shortNames") or [])}:
            return gv, r
    raise SystemExit(f'error: the server doesn\'t have a resource type "{word}"')


def _explain(k, a) -> int:
    """kubectl explain RESOURCE[.FIELD...]: the kind's schema from the server's OpenAPI v3."""
    if not a.args:
        raise SystemExit("usage: kubectl explain RESOURCE[.FIELD...]")
    word, *fields = a.args[0].split(".")
    gv, r = _find_resource(k, word)
    doc = k.get(k.k8s("/openapi/v3/" + ("api/v1" if gv == "v1" else f"apis/{gv}")))
    schemas = doc.get("components", {}).get("schemas", {})
    schema = next((s for s in schemas.values() if any(x.get("kind") == r["kind"] for x in s.get("x-kubernetes-group-version-kind") or [])), None)
    if schema is None:
        raise SystemExit(f"error: no schema for {r['kind']}")
    for f in fields:
        nxt = (schema.get("properties") or {}).get(f)
        if nxt is None:
            raise SystemExit(f'error: field "{f}" does not exist')
        if "$ref" in nxt:
            nxt = schemas.get(nxt["$ref"].rsplit("/", 1)[-1], nxt)
        schema = nxt
    print(f"GROUP:      {gv.split('/')[0] if '/' in gv else ''}\nKIND:       {r['kind']}\nVERSION:    {gv.split('/')[-1]}\n")
    if fields:
        print(f"FIELD: {fields[-1]} <{schema.get('type', 'Object')}>\n")
    print("DESCRIPTION:\n    " + (schema.get("description") or "<empty>"))
    props = schema.get("properties") or {}
    if props:
        print("\nFIELDS:")
        for name, p in props.items():
            typ = p.get("type") or ("Object" if "$ref" in p else "")
            print(f"  {name}\t<{typ}>")
            if p.get("description"):
                print(f"    {p['description']}")
    elif schema.get("x-kubernetes-preserve-unknown-fields"):
        print("\n(this server does not publish the field schema below this level)")
    return 0


def _auth(k, a, ns: str) -> int:
    """kubectl auth can-i VERB RESOURCE[/NAME] [--subresource S]: a SelfSubjectAccessReview; yes/no, exit 0/1."""
    if len(a.args) < 3 or a.args[0] != "can-i":
        raise SystemExit("usage: kubectl auth can-i VERB RESOURCE[/NAME]")
    verb, res = a.args[1], a.args[2]
    res, _, name = res.partition("/")
    group = ""
    if res != "*":
        try:
            gv, r = _find_resource(k, res.split(".")[0])
            res, group = r["name"], gv.split("/")[0] if "/" in gv else ""
        except SystemExit:
            pass
    attrs = {"verb": verb, "resource": res, "group": group, **({"name": name} if name else {}),
             **({} if a.all_namespaces else {"namespace": ns})}
    if a.subresource:
        attrs["subresource"] = a.subresource
    out = k.post(k.k8s("/apis/authorization.k8s.io/v1/selfsubjectaccessreviews"), {
        "apiVersion": "authorization.k8s.io/v1", "kind": "SelfSubjectAccessReview", "spec": {"resourceAttributes": attrs}})
    ok = bool((out.get("status") or {}).get("allowed"))
    print("yes" if ok else "no")
    return 0 if ok else 1


def _config(a, cfg: dict) -> int:
    sub = a.args[0] if a.args else "view"
    if sub == "view":
        red = json.loads(json.dumps(cfg))
        for u in red.get("users") or []:
            for key in ("token", "client-key-data", "password"):
                if key in (u.get("user") or {}):
                    u["user"][key] = "REDACTED"
        print(json.dumps(red, indent=2) if a.output == "json" else yaml.safe_dump(red, sort_keys=False).rstrip())
    elif sub == "current-context":
        print(cfg.get("current-context", ""))
    elif sub == "get-contexts":
        cur = cfg.get("current-context")
        print(f"{'CURRENT':<8} {'NAME':<24} {'CLUSTER':<24} {'AUTHINFO':<24} NAMESPACE")
        for c in cfg.get("contexts") or []:
            ctx = c.get("context") or {}
            print(f"{'*' if c['name'] == cur else '':<8} {c['name']:<24} {ctx.get('cluster', ''):<24} "
                  f"{ctx.get('user', ''):<24} {ctx.get('namespace', '')}")
    else:
        raise SystemExit("usage: kubectl config view|current-context|get-contexts")
    return 0


def rollout_pause(k, name: str, ns: str, pause: bool) -> int:
    k.request("PATCH", k.k8s(object_path("deployment", name, ns)), body={"spec": {"paused": pause}},
              content_type="application/merge-patch+json")
    print(f"deployment.apps/{name} {'paused' if pause else 'resumed'}")
    return 0


def dispatch(k, a, ns: str, cfg: dict) -> int:
    if a.verb == "run":
        return _run(k, a, ns)
    if a.verb == "set":
        return _set(k, a, ns)
    if a.verb == "autoscale":
        return _autoscale(k, a, ns)
    if a.verb == "patch":
        return _patch(k, a, ns)
    if a.verb == "replace":
        return _replace(k, a, ns)
    if a.verb == "edit":
        return _edit(k, a, ns)
    if a.verb == "diff":
        return _diff(k, a, ns)
    if a.verb == "events":
        return _events(k, a, ns)
    if a.verb == "explain":
        return _explain(k, a)
    if a.verb == "api-resources":
        return _api_resources(k, a)
    if a.verb == "api-versions":
        return _api_versions(k)
    if a.verb == "auth":
        return _auth(k, a, ns)
    if a.verb == "kustomize":
        return _kustomize(a)
    return _config(a, cfg)
