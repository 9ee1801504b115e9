"""Minimal kubectl for the tk8s control plane (the CLI half of docs/detailed.md:285-370).

  kubectl get nodes|pods|ds|jobs|deploy|svc|cm|secrets|ing|events [-n NS | -A] [-l k=v] [-o wide|json|yaml]
  kubectl describe node NAME | pod NAME
  kubectl create|apply -f FILE        kubectl delete -f FILE | KIND NAME
  kubectl create configmap|secret generic NAME --from-literal k=v --from-file [k=]PATH
  kubectl scale deploy/NAME --replicas N
  kubectl rollout status|restart deploy/NAME
  kubectl label|annotate KIND NAME k=v k-
  kubectl logs POD [--tail N] [-f]    kubectl cordon|uncordon|drain NODE
  kubectl exec [-it] POD -- CMD [ARGS...]   (-it: a terminal in the pod, streaming; else stdout/stderr/exit code)
  kubectl top nodes                   (amd.com/gpu in use, hotspot temperature, power, VRAM)
  kubectl wait job/NAME [--timeout S] kubectl cluster-info | version

The kubeconfig comes from --kubeconfig, $KUBECONFIG, or <workdir>/.tk8s/kubeconfig.json (written
by setup; the same document the control plane serves at /env/<env>/kubernetes/kubectl).
"""
from __future__ import annotations

import argparse
import base64
import json
import os
import sys
import time
from pathlib import Path

import yaml

from ..controlplane.client import ApiError, client_from_kubeconfig
from ..kube import (apply_objects, collection_path, delete_objects, job_state, kind_key, load_manifests,
                    object_path, server_apply_objects, wait_job, wait_rollout)
from ..utils.net import host_port
from .kubectl_more import VERBS as MORE_VERBS, dispatch as more_dispatch

GPU = "amd.com/gpu"


def _load_kubeconfig(path: str | None, workdir: str) -> dict:
    p = path or os.environ.get("KUBECONFIG") or str(Path(workdir) / ".tk8s" / "kubeconfig.json")
    text = Path(p).read_text()
    return json.loads(text) if text.lstrip().startswith("{") else yaml.safe_load(text)


def _age(obj: dict) -> str:
    ts = obj.get("metadata", {}).get("creationTimestamp")
    if not ts:
        return "-"
    try:
        t = time.mktime(time.strptime(ts, "%Y-%m-%dT%H:%M:%SZ")) - time.timezone
        s = max(0, int(time.time() - t))
    except ValueError:
        return "-"
    return f"{s}s" if s < 120 else f"{s // 60}m" if s < 7200 else f"{s // 3600}h"


def _cond(obj: dict, t: str) -> dict:
    return next((c for c in obj.get("status", {}).get("conditions", []) if c.get("type") == t), {})


def _table(rows: list[list[str]]) -> str:
    if not rows:
        return "No resources found."
    w = [max(len(str(r[i])) for r in rows) for i in range(len(rows[0]))]
    return "\n".join("   ".join(str(c).ljust(w[i]) for i, c in enumerate(r)).rstrip() for r in rows)


def fmt_nodes(items: list[dict], wide: bool) -> str:
    rows = [["NAME", "STATUS", "ROLES", "AGE", "VERSION", "GPU", "VALIDATED"] + (["INTERNAL-IP", "GPU-IDS"] if wide else [])]
    for n in items:
        ready = _cond(n, "Ready").get("status")
        st = "Ready" if ready == "True" else "NotReady"
        if n.get("spec", {}).get("unschedulable"):
            st += ",SchedulingDisabled"
        val = _cond(n, "AMDGPUValidated")
        row = [n["metadata"]["name"], st, "worker", _age(n), n["status"].get("nodeInfo", {}).get("kubeletVersion", "-"),
               f"{n['status']['allocatable'].get(GPU, '0')}/{n['status']['capacity'].get(GPU, '0')}",
               {"True": "yes", "False": "FAILED"}.get(val.get("status"), "pending")]
        if wide:
            ip = next((a["address"] for a in n["status"].get("addresses", []) if a["type"] == "InternalIP"), "")
            row += [ip, ",".join(d["id"] for d in n["status"].get("devices", []))]
        rows.append(row)
    return _table(rows)


def fmt_pods(items: list[dict], wide: bool, all_ns: bool) -> str:
    head = (["NAMESPACE"] if all_ns else []) + ["NAME", "READY", "STATUS", "RESTARTS", "AGE"] + (["IP", "NODE", "GPUS"] if wide else [])
    rows = [head]
    for p in items:
        st = p.get("status", {})
        cs = (st.get("containerStatuses") or [{}])[0]
        phase = st.get("phase", "Pending")
        if phase == "Pending" and _cond(p, "PodScheduled").get("status") == "False":
            phase = "Pending(Unschedulable)"
        if p["metadata"].get("deletionTimestamp"):
            phase = "Terminating"
        row = ([p["metadata"].get("namespace", "")] if all_ns else []) + [
            p["metadata"]["name"], "1/1" if phase == "Running" else "0/1", phase, str(cs.get("restartCount", 0)), _age(p)]
        if wide:
            row += [st.get("podIP") or "<none>", p["spec"].get("nodeName") or "<none>",
                    p["metadata"].get("annotations", {}).get("amd.com/gpu-ids", "")]
        rows.append(row)
    return _table(rows)


def fmt_generic(kind: str, items: list[dict], all_ns: bool) -> str:
    k = kind_key(kind)
    if k == "daemonset":
        head = ["NAME", "DESIRED", "CURRENT", "READY", "SUCCEEDED", "FAILED", "AGE"]
        rows = [head] + [[o["metadata"]["name"], *(str(o.get("status", {}).get(f, 0)) for f in (
            "desiredNumberScheduled", "currentNumberScheduled", "numberReady", "numberSucceeded", "numberFailed")), _age(o)]
            for o in items]
    elif k == "job":
        rows = [["NAME", "COMPLETIONS", "STATUS", "AGE"]] + [[o["metadata"]["name"],
                f"{o.get('status', {}).get('succeeded', 0)}/{o['spec'].get('completions', 1)}", job_state(o), _age(o)] for o in items]
    elif k in ("deployment", "statefulset"):
        rows = [["NAME", "READY", "AGE"]] + [[o["metadata"]["name"],
                f"{o.get('status', {}).get('readyReplicas', 0)}/{o['spec'].get('replicas', 1)}", _age(o)] for o in items]
    elif k == "replicaset":
        rows = [["NAME", "DESIRED", "CURRENT", "READY", "AGE"]] + [[o["metadata"]["name"], str(o["spec"].get("replicas", 1)),
                str(o.get("status", {}).get("replicas", 0)), str(o.get("status", {}).get("readyReplicas", 0)), _age(o)]
                for o in items]
    elif k == "poddisruptionbudget":
        rows = [["NAME", "MIN AVAILABLE", "MAX UNAVAILABLE", "ALLOWED DISRUPTIONS", "AGE"]] + [[
            o["metadata"]["name"], str(o["spec"].get("minAvailable", "N/A")), str(o["spec"].get("maxUnavailable", "N/A")),
            str(o.get("status", {}).get("disruptionsAllowed", 0)), _age(o)] for o in items]
    elif k == "cronjob":
        rows = [["NAME", "SCHEDULE", "SUSPEND", "ACTIVE", "LAST SCHEDULE", "AGE"]] + [[
            o["metadata"]["name"], o["spec"].get("schedule", ""), str(bool(o["spec"].get("suspend", False))),
            str(len(o.get("status", {}).get("active") or [])), o.get("status", {}).get("lastScheduleTime", "<none>"), _age(o)]
            for o in items]
    elif k == "service":
        def ports(o):
            return ",".join(f"{p['port']}" + (f"(host {host_port(p['port'])})" if host_port(p["port"]) != p["port"] else "")
                            + (f":{p['nodePort']}" if p.get("nodePort") else "") + f"/{p.get('protocol', 'TCP')}"
                            for p in o["spec"].get("ports", []))

        def ext(o):
            ing = o.get("status", {}).get("loadBalancer", {}).get("ingress") or []
            return ",".join(i.get("ip", "") for i in ing) or ("<pending>" if o["spec"].get("type") == "LoadBalancer" else "<none>")

        rows = [["NAME", "TYPE", "CLUSTER-IP", "EXTERNAL-IP", "PORT(S)", "AGE"]] + [[
            o["metadata"]["name"], o["spec"].get("type", "ClusterIP"), o["spec"].get("clusterIP", ""), ext(o), ports(o), _age(o)]
            for o in items]
    elif k == "horizontalpodautoscaler":
        def targets(o):
            out = []
            for m in o.get("status", {}).get("currentMetrics") or []:
                r = m.get("resource") or {}
                cur = (r.get("current") or {}).get("averageUtilization")
                want = next((((x.get("resource") or {}).get("target") or {}).get("averageUtilization")
                            for x in o["spec"].get("metrics") or [] if (x.get("resource") or {}).get("name") == r.get("name")), None)
                out.append(f"{r.get('name')}: {cur}%/{want}%")
            return ", ".join(out) or "<unknown>"

        rows = [["NAME", "REFERENCE", "TARGETS", "MINPODS", "MAXPODS", "REPLICAS", "AGE"]] + [[
            o["metadata"]["name"], f"{o['spec']['scaleTargetRef'].get('kind')}/{o['spec']['scaleTargetRef'].get('name')}",
            targets(o), str(o["spec"].get("minReplicas", 1)), str(o["spec"].get("maxReplicas")),
            str(o.get("status", {}).get("currentReplicas", 0)), _age(o)] for o in items]
    elif k == "namespace":
        rows = [["NAME", "STATUS", "AGE"]] + [[o["metadata"]["name"], o.get("status", {}).get("phase", "Active"), _age(o)]
                                             for o in items]
    elif k in ("configmap", "secret"):
        rows = [["NAME"] + (["TYPE"] if k == "secret" else []) + ["DATA", "AGE"]] + [
            [o["metadata"]["name"]] + ([o.get("type", "Opaque")] if k == "secret" else [])
            + [str(len(o.get("data") or {})), _age(o)] for o in items]
    elif k == "ingress":
        rows = [["NAME", "HOSTS", "ADDRESS", "AGE"]] + [[
            o["metadata"]["name"], ",".join(r.get("host", "*") or "*" for r in o.get("spec", {}).get("rules") or []) or "*",
            ",".join(i.get("ip", "") for i in o.get("status", {}).get("loadBalancer", {}).get("ingress", [])), _age(o)]
            for o in items]
    elif k == "event":
        rows = [["TYPE", "REASON", "OBJECT", "MESSAGE"]] + [[o.get("type", ""), o.get("reason", ""),
                f"{o.get('involvedObject', {}).get('kind', '').lower()}/{o.get('involvedObject', {}).get('name', '')}",
                o.get("message", "")] for o in items]
    else:
        rows = [["NAME", "AGE"]] + [[o["metadata"]["name"], _age(o)] for o in items]
    if all_ns and len(rows) > 1:
        rows = [["NAMESPACE"] + rows[0]] + [[o["metadata"].get("namespace", "")] + r for o, r in zip(items, rows[1:])]
    return _table(rows)


def _target(args: list[str]) -> tuple[str, str]:
    """KIND/NAME or KIND NAME."""
    if not args:
        raise SystemExit("error: a resource (KIND/NAME or KIND NAME) is required")
    if "/" in args[0]:
        what, name = args[0].split("/", 1)
        return what, name
    if len(args) < 2:
        raise SystemExit("error: a resource name is required")
    return args[0], args[1]


def _cp(k, ns: str, args: list[str], container: str | None = None) -> int:
    """``kubectl cp SRC DST`` with one side ``[namespace/]pod:path``: a tar archive through exec,
    as kubectl does (the pod needs ``tar``)."""
    import base64
    import io
    import posixpath
    import tarfile

    if len(args) != 2 or sum(":" in x for x in args) != 1:
        raise SystemExit("usage: kubectl cp LOCAL POD:PATH | kubectl cp POD:PATH LOCAL")
    src, dst = args

    def pod_side(spec: str) -> tuple[str, str, str]:
        who, path = spec.split(":", 1)
        pns, pod = who.split("/", 1) if "/" in who else (ns, who)
        return pns, pod, path

    def run(pns: str, pod: str, cmd: list[str], stdin: bytes = b"") -> dict:
        r = k.post(k.k8s(object_path("pod", pod, pns) + "/exec"), {
            "command": cmd, "stdin_b64": base64.b64encode(stdin).decode(), "binary": True, "timeoutSeconds": 600},
            timeout=660)
        if r.get("exitCode", 1) != 0:
            raise SystemExit(f"error: {' '.join(cmd)}: {r.get('stderr', '').strip()}")
        return r

    if ":" in dst:  # local -> pod
        pns, pod, path = pod_side(dst)
        buf = io.BytesIO()
        with tarfile.open(fileobj=buf, mode="w") as t:
            t.add(src, arcname=posixpath.basename(path.rstrip("/")) or Path(src).name)
        run(pns, pod, ["tar", "xf", "-", "-C", posixpath.dirname(path.rstrip("/")) or "."], buf.getvalue())
    else:  # pod -> local
        pns, pod, path = pod_side(src)
        r = run(pns, pod, ["tar", "cf", "-", "-C", posixpath.dirname(path.rstrip("/")) or ".",
                           posixpath.basename(path.rstrip("/"))])
        with tarfile.open(fileobj=io.BytesIO(base64.b64decode(r["stdout_b64"]))) as t:
            for m in t.getmembers():  # never outside the destination
                if m.name.startswith("/") or ".." in Path(m.name).parts or m.issym() or m.islnk():
                    raise SystemExit(f"error: refusing archive member {m.name!r}")
            base = posixpath.basename(path.rstrip("/"))
            out = Path(dst)
            for m in t.getmembers():
                rel = Path(m.name).relative_to(base) if m.name != base else Path()
                target = out / rel
                if m.isdir():
                    target.mkdir(parents=True, exist_ok=True)
                elif m.isfile():
                    target.parent.mkdir(parents=True, exist_ok=True)
                    target.write_bytes(t.extractfile(m).read())
    return 0


def _jsonpath(obj, expr: str):
    """The value at a simple JSONPath (``{.status.phase}``, ``{.status.conditions[0].type}``)."""
    import re

    cur = obj
    for name, idx in re.findall(r"\.([^.\[\]]+)|\[(\d+)\]", expr.strip().strip("{}")):
        if cur is None:
            return None
        cur = (cur.get(name) if isinstance(cur, dict) else None) if name else (
            cur[int(idx)] if isinstance(cur, list) and int(idx) < len(cur) else None)
    return cur


def _jsonpath_all(obj, expr: str) -> list:
    """Every value a JSONPath selects, ``[*]`` fanning out over list elements (or map values)."""
    import re

    cur = [obj]
    for name, idx in re.findall(r"\.([^.\[\]]+)|\[(\*|-?\d+)\]", expr.strip().strip("{}")):
        nxt = []
        for x in cur:
            if name:
                if isinstance(x, dict) and name in x:
                    nxt.append(x[name])
            elif idx == "*":
                nxt += list(x) if isinstance(x, list) else list(x.values()) if isinstance(x, dict) else []
            elif isinstance(x, list) and -len(x) <= int(idx) < len(x):
                nxt.append(x[int(idx)])
        cur = nxt
    return cur


def _fmt_value(v) -> str:
    return v if isinstance(v, str) else json.dumps(v, separators=(",", ":")) if isinstance(v, (dict, list)) else str(v)


def render_jsonpath(obj, template: str) -> str:
    """kubectl's ``-o jsonpath=TEMPLATE``: literal text with ``{...}`` expressions (values
    joined by spaces)."""
    import re

    out, pos = [], 0
    for m in re.finditer(r"\{([^{}]*)\}", template):
        out.append(template[pos:m.start()].replace("\\n", "\n").replace("\\t", "\t"))
        out.append(" ".join(_fmt_value(v) for v in _jsonpath_all(obj, m.group(1))))
        pos = m.end()
    out.append(template[pos:].replace("\\n", "\n").replace("\\t", "\t"))
    return "".join(out)


def render_custom_columns(items: list[dict], spec: str) -> str:
    cols = [c.split(":", 1) for c in spec.split(",") if c]
    rows = [[h for h, _ in cols]] + [[",".join(_fmt_value(v) for v in _jsonpath_all(o, e)) or "<none>" for _h, e in cols]
                                     for o in items]
    return _table(rows)


def _watch_rows(k, what: str, ns: str, name: str | None, q: dict | None, a) -> int:
    path = k.k8s("/api/v1/nodes" if what == "node" else "/api/v1/pods" if what == "pod" and a.all_namespaces
                 else collection_path(what, ns))
    query = dict(q or {})
    if name:
        query["fieldSelector"] = f"metadata.name={name}"
    rv = int(k.get(path, query=query)["metadata"]["resourceVersion"])
    deadline = time.monotonic() + float(a.timeout.rstrip("s"))
    try:
        while time.monotonic() < deadline:
            rv, events = k.watch(path, rv, timeout=min(5.0, max(0.1, deadline - time.monotonic())), query=query)
            for ev in events:
                o = ev["object"]
                if ev["type"] == "DELETED" and what == "pod":
                    o = {**o, "metadata": {**o["metadata"], "deletionTimestamp": o["metadata"].get("deletionTimestamp") or "-"}}
                table = (fmt_pods([o], a.output == "wide", a.all_namespaces) if what == "pod" else
                         fmt_nodes([o], a.output == "wide") if what == "node" else fmt_generic(what, [o], a.all_namespaces))
                print(table.splitlines()[-1], flush=True)
    except KeyboardInterrupt:
        pass
    return 0


def _wait_met(obj: dict | None, cond: str) -> bool:
    if cond == "delete":
        return obj is None
    if obj is None:
        return False
    if cond.startswith("condition="):
        ctype, _, want = cond[len("condition="):].partition("=")
        return any(c.get("type", "").lower() == ctype.lower() and str(c.get("status")).lower() == (want or "true").lower()
                   for c in (obj.get("status") or {}).get("conditions") or [])
    if cond.startswith("jsonpath="):
        expr, _, want = cond[len("jsonpath="):].rpartition("=") if "}=" in cond else (cond[len("jsonpath="):], "", "")
        v = _jsonpath(obj, expr)
        return v is not None if not want else str(v) == want.strip("'\"")
    raise SystemExit(f"error: unrecognized condition: {cond!r} (condition=TYPE[=STATUS], delete, jsonpath={{...}}=VALUE)")


def _wait(k, ns: str, args: list[str], cond: str, selector: str | None, timeout: float) -> int:
    """``kubectl wait TYPE/NAME... | TYPE -l SEL --for=condition=Ready|delete|jsonpath=...``."""
    if len(args) == 1 and "/" not in args[0] and not selector:
        raise SystemExit("error: resource name or selector required")
    targets = [tuple(x.split("/", 1)) for x in args] if "/" in args[0] else [(args[0], n) for n in args[1:]]
    kind = kind_key(targets[0][0] if targets else args[0])
    if selector:
        items = k.get(k.k8s(collection_path(kind, ns)), query={"labelSelector": selector})["items"]
        targets += [(kind, o["metadata"]["name"]) for o in items]
        if not targets:
            print(f"error: no matching resources found", file=sys.stderr)
            return 1
    deadline = time.monotonic() + timeout
    rc = 0
    for what, name in targets:
        path = k.k8s(f"/api/v1/nodes/{name}" if kind_key(what) == "node" else object_path(what, name, ns))
        while True:
            try:
                obj = k.get(path)
            except ApiError as e:
                if e.status != 404:
                    raise
                obj = None
            if _wait_met(obj, cond):
                print(f"{kind_key(what)}/{name} {'deleted' if cond == 'delete' else 'condition met'}")
                break
            if obj is None:
                print(f'Error from server (NotFound): {kind_key(what)}s "{name}" not found', file=sys.stderr)
                rc = 1
                break
            if time.monotonic() >= deadline:
                print(f"error: timed out waiting for the condition on {kind_key(what)}s/{name}", file=sys.stderr)
                rc = 1
                break
            time.sleep(0.2)
    return rc


def _rollout_other(k, kind: str, name: str, ns: str, sub: str, timeout: float) -> int:
    """rollout status|restart of a StatefulSet (and status of a DaemonSet)."""
    path = k.k8s(object_path(kind, name, ns))
    if sub == "restart":
        if kind != "statefulset":
            raise SystemExit("error: rollout restart is served for Deployments and StatefulSets")
        k.request("PATCH", path, body={"spec": {"template": {"metadata": {"annotations": {
            "kubectl.kubernetes.io/restartedAt": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())}}}}})
        print(f"statefulset.apps/{name} restarted")
        return 0
    deadline = time.monotonic() + timeout
    last = None
    while True:
        o = k.get(path)
        st = o.get("status") or {}
        if kind == "statefulset":
            want = int(o["spec"].get("replicas", 1))
            have, upd = int(st.get("readyReplicas", 0)), int(st.get("updatedReplicas", 0))
            done = have == want and upd == want and st.get("currentRevision") == st.get("updateRevision")
            msg = f"Waiting for {want - have} pods to be ready..." if have < want else \
                f"Waiting for partitioned roll out to finish: {upd} out of {want} new pods have been updated..."
        else:
            want, have = int(st.get("desiredNumberScheduled", 0)), int(st.get("numberReady", 0))
            done = have == want
            msg = f'Waiting for daemon set "{name}" rollout to finish: {have} of {want} updated pods are available...'
        if done:
            print(f"partitioned roll out complete: {want} new pods have been updated..." if kind == "statefulset"
                  else f'daemon set "{name}" successfully rolled out')
            return 0
        if msg != last:
            print(msg, flush=True)
            last = msg
        if time.monotonic() > deadline:
            print(f"error: timed out waiting for the condition", file=sys.stderr)
            return 1
        time.sleep(0.2)


def _create_job(k, a, ns: str) -> int:
    """kubectl create job NAME --image=IMG [-- CMD...] | --from=cronjob/CJ (run a CronJob now)."""
    if len(a.args) < 2:
        raise SystemExit("usage: kubectl create job NAME (--image=IMAGE [-- COMMAND...] | --from=cronjob/NAME)")
    name = a.args[1]
    if a.from_:
        what, _, src = a.from_.partition("/")
        if kind_key(what) != "cronjob":
            raise SystemExit("error: --from must be cronjob/NAME")
        cj = k.get(k.k8s(object_path("cronjob", src, ns)))
        jt = cj["spec"].get("jobTemplate") or {}
        body = {"apiVersion": "batch/v1", "kind": "Job", "metadata": {
            "name": name, "labels": dict((jt.get("metadata") or {}).get("labels") or {}),
            "annotations": {**((jt.get("metadata") or {}).get("annotations") or {}), "cronjob.kubernetes.io/instantiate": "manual"},
            "ownerReferences": [{"apiVersion": "batch/v1", "kind": "CronJob", "name": src, "uid": cj["metadata"]["uid"]}]},
            "spec": jt.get("spec") or {}}
    else:
        if not a.image:
            raise SystemExit("error: --image or --from is required")
        c = {"name": name, "image": a.image, **({"command": list(a.command)} if a.command else {})}
        body = {"apiVersion": "batch/v1", "kind": "Job", "metadata": {"name": name},
                "spec": {"template": {"spec": {"restartPolicy": "Never", "containers": [c]}}}}
    k.post(k.k8s(collection_path("job", ns)), body)
    print(f"job.batch/{name} created")
    return 0


def _manifests(a) -> list[dict]:
    """The objects of ``-f FILE`` or ``-k DIR`` (a kustomization, kustomize.py)."""
    if a.kustomize:
        from .. import kustomize

        try:
            return kustomize.build(a.kustomize)
        except kustomize.KustomizeError as e:
            raise SystemExit(f"error: {e}") from e
    if not a.filename:
        raise SystemExit("error: must specify one of -f and -k")
    return load_manifests(a.filename)


def _logs_many(k, ns: str, a) -> int:
    """kubectl logs -l SELECTOR | TYPE/NAME | --all-containers | --previous [--prefix]: every
    selected pod's (and container's) log, one after the other."""
    if a.selector:
        pods = k.get(k.k8s(collection_path("pod", ns)), query={"labelSelector": a.selector})["items"]
    elif a.args and "/" in a.args[0] and kind_key(a.args[0].split("/")[0]) != "pod":
        what, name = a.args[0].split("/", 1)  # deploy/web, job/x, ...: its pods, as kubectl picks them
        obj = k.get(k.k8s(object_path(what, name, ns)))
        sel = ((obj.get("spec") or {}).get("selector") or {}).get("matchLabels") or (
            {"job-name": name} if kind_key(what) == "job" else {})
        pods = k.get(k.k8s(collection_path("pod", ns)),
                     query={"labelSelector": ",".join(f"{x}={y}" for x, y in sel.items())})["items"][:1]
    else:
        name = a.args[0].split("/", 1)[-1]
        pods = [k.get(k.k8s(object_path("pod", name, ns)))]
    rc = 0
    for p in pods:
        names = [c["name"] for c in p["spec"].get("containers") or []]
        conts = names if (a.all_containers or a.selector) and not a.container else [a.container or names[0]]
        for c in conts:
            q = {"container": c, **({"previous": "true"} if a.previous else {}),
                 **({"tailLines": str(a.tail)} if a.tail else {})}
            try:
                text = k.get(k.k8s(object_path("pod", p["metadata"]["name"], ns) + "/log"), query=q, raw=True)
            except ApiError as e:
                print(f"Error from server: {e}", file=sys.stderr)
                rc = 1
                continue
            pre = f"[pod/{p['metadata']['name']}/{c}] " if a.prefix else ""
            for line in text.splitlines(keepends=True):
                sys.stdout.write(pre + line)
    sys.stdout.flush()
    return rc


def _drain(k, node: str, timeout: float, disable_eviction: bool) -> int:
    """Cordon, then evict every pod but DaemonSets' and finished ones through the Eviction API,
    retrying those a PodDisruptionBudget holds back (429) until ``timeout``."""
    k.request("PATCH", k.k8s(f"/api/v1/nodes/{node}"), body={"spec": {"unschedulable": True}})
    print(f"node/{node} cordoned")
    pods = []
    for p in k.get(k.k8s("/api/v1/pods"), query={"fieldSelector": f"spec.nodeName={node}"})["items"]:
        owners = {r.get("kind") for r in p["metadata"].get("ownerReferences", [])}
        if "DaemonSet" in owners or p.get("status", {}).get("phase") in ("Succeeded", "Failed"):
            continue
        pods.append((p["metadata"]["namespace"], p["metadata"]["name"]))
    deadline = time.monotonic() + timeout
    while pods:
        left = []
        for pns, name in pods:
            path = k.k8s(object_path("pod", name, pns))
            try:
                if disable_eviction:
                    k.delete(path)
                else:
                    k.post(path + "/eviction", {"apiVersion": "policy/v1", "kind": "Eviction",
                                                "metadata": {"name": name, "namespace": pns}})
                print(f"{'deleting' if disable_eviction else 'evicting'} pod {pns}/{name}")
            except ApiError as e:
                if e.status == 404:
                    continue
                if e.status != 429:
                    raise
                print(f'error when evicting pods/"{name}" -n "{pns}" (will retry after 1s): {e}', file=sys.stderr)
                left.append((pns, name))
        pods = left
        if pods:
            if time.monotonic() >= deadline:
                print(f"error: unable to drain node {node!r} due to error: global timeout reached: {timeout:g}s, "
                      f"{len(pods)} pod(s) left", file=sys.stderr)
                return 1
            time.sleep(1.0)
    print(f"node/{node} drained")
    return 0


def _rollout_history(k, name: str, ns: str, sub: str, to_revision: int = 0) -> int:
    """``rollout history`` lists the Deployment's revisions (its ReplicaSets); ``rollout undo``
    puts the template of the previous revision (or ``--to-revision``) back, as kubectl does."""
    d = k.get(k.k8s(object_path("deployment", name, ns)))
    uid = d["metadata"]["uid"]
    rss = [rs for rs in k.get(k.k8s(collection_path("replicaset", ns)))["items"]
           if any(r.get("uid") == uid for r in rs["metadata"].get("ownerReferences", []))]
    revs = sorted(((int(rs["metadata"].get("annotations", {}).get("deployment.kubernetes.io/revision", 0)), rs)
                   for rs in rss), key=lambda x: x[0])
    if sub == "history":
        print(f"deployment.apps/{name}\nREVISION  CHANGE-CAUSE")
        for rev, rs in revs:
            print(f"{rev:<9} {rs['metadata'].get('annotations', {}).get('kubernetes.io/change-cause', '<none>')}")
        return 0
    if len(revs) < 2 and not to_revision:
        raise SystemExit(f"error: no rollout history found for deployment {name!r}")
    target = next((rs for rev, rs in revs if rev == to_revision), None) if to_revision else revs[-2][1]
    if target is None:
        raise SystemExit(f"error: unable to find specified revision {to_revision} in history")
    tmpl = target["spec"]["template"]
    tmpl.get("metadata", {}).get("labels", {}).pop("pod-template-hash", None)
    k.put(k.k8s(object_path("deployment", name, ns)), {**{x: v for x, v in d.items() if x != "status"},
                                                     "spec": {**d["spec"], "template": tmpl}})
    print(f"deployment.apps/{name} rolled back")
    return 0


def _create_deployment(k, a, ns: str) -> int:
    """kubectl create deployment NAME --image IMAGE [--replicas N] [--port P]: labels app=NAME."""
    if len(a.args) < 2 or not a.image:
        raise SystemExit("usage: kubectl create deployment NAME --image IMAGE [--replicas N] [--port P]")
    name = a.args[1]
    container = {"name": a.image.rsplit("/", 1)[-1].split(":", 1)[0].split("@", 1)[0] or name, "image": a.image}
    if a.port:
        container["ports"] = [{"containerPort": a.port}]
    body = {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": name, "labels": {"app": name}},
            "spec": {"replicas": 1 if a.replicas is None else a.replicas, "selector": {"matchLabels": {"app": name}},
                     "template": {"metadata": {"labels": {"app": name}}, "spec": {"containers": [container]}}}}
    k.post(k.k8s(collection_path("deployment", ns)), body)
    print(f"deployment.apps/{name} created")
    return 0


def _expose(k, a, ns: str) -> int:
    """kubectl expose deployment NAME --port P [--target-port T] [--type T] [--name SVC]: a Service
    selecting the Deployment's pods."""
    if len(a.args) < 2 or kind_key(a.args[0]) != "deployment" or not a.port:
        raise SystemExit("usage: kubectl expose deployment NAME --port P [--target-port T] [--type TYPE] [--name SVC]")
    if a.type not in (None, "ClusterIP", "NodePort", "LoadBalancer"):
        raise SystemExit(f"error: --type must be ClusterIP, NodePort or LoadBalancer, not {a.type!r}")
    d = k.get(k.k8s(object_path("deployment", a.args[1], ns)))
    sel = d["spec"].get("selector", {}).get("matchLabels") or d["spec"]["template"]["metadata"].get("labels", {})
    name = a.name or a.args[1]
    body = {"apiVersion": "v1", "kind": "Service", "metadata": {"name": name, "labels": dict(sel)},
            "spec": {"type": a.type or "ClusterIP", "selector": sel,
                     "ports": [{"port": a.port, "targetPort": a.target_port or a.port, "protocol": "TCP"}]}}
    k.post(k.k8s(collection_path("service", ns)), body)
    print(f"service/{name} exposed")
    return 0


def _create_data(k, a, ns: str) -> int:
    """kubectl create configmap NAME / create secret generic NAME (--from-literal, --from-file)."""
    secret = a.args[0] == "secret"
    rest = a.args[1:]
    if secret and rest and rest[0] == "generic":
        rest = rest[1:]
    if not rest:
        raise SystemExit("usage: kubectl create configmap|secret generic NAME --from-literal k=v --from-file [k=]PATH")
    data: dict[str, str] = {}
    for kv in a.from_literal:
        key, _, val = kv.partition("=")
        data[key] = val
    for spec in a.from_file:
        key, _, path = spec.partition("=") if "=" in spec else (Path(spec).name, "", spec)
        data[key] = Path(path).read_text()
    body = {"apiVersion": "v1", "kind": "Secret" if secret else "ConfigMap", "metadata": {"name": rest[0]}}
    if secret:
        body.update(type="Opaque", data={key: base64.b64encode(v.encode()).decode() for key, v in data.items()})
    else:
        body["data"] = data
    k.post(k.k8s(collection_path("secret" if secret else "configmap", ns)), body)
    print(f"{'secret' if secret else 'configmap'}/{rest[0]} created")
    return 0


def fmt_top(nodes: list[dict], pods: list[dict], usage: dict | None = None) -> str:
    """Per node: CPU and memory in use (metrics.k8s.io, when the agents have sampled), amd.com/gpu
    in use / allocatable and the last AMD SMI sample of its GPUs."""
    used: dict[str, int] = {}
    for p in pods:
        nn = p["spec"].get("nodeName")
        if nn and p.get("status", {}).get("phase") not in ("Succeeded", "Failed"):
            used[nn] = used.get(nn, 0) + sum(int(c.get("resources", {}).get("limits", {}).get(GPU, 0) or 0)
                                             for c in p["spec"].get("containers", []))
    from ..utils import quantity

    usage = usage or {}
    rows = [["NAME", "CPU(cores)", "MEMORY(bytes)", "GPU(USED/ALLOC)", "HOTSPOT-MAX", "POWER", "VRAM-USED"]]
    for n in nodes:
        tel = [d.get("telemetry") or {} for d in n["status"].get("devices", [])]
        hot = [t["temp_c"]["hotspot"] for t in tel if "hotspot" in t.get("temp_c", {})]
        watts = [t["power"]["current_w"] for t in tel if "current_w" in t.get("power", {})]
        vram = [t["vram_used_bytes"] for t in tel if "vram_used_bytes" in t]
        name = n["metadata"]["name"]
        u = usage.get(name) or {}
        rows.append([name, f"{int(quantity.parse(u['cpu']) * 1000)}m" if u.get("cpu") else "<unknown>",
                     f"{int(quantity.parse(u['memory']) / 2**20)}Mi" if u.get("memory") else "<unknown>",
                     f"{used.get(name, 0)}/{n['status']['allocatable'].get(GPU, '0')}",
                     f"{max(hot)}C" if hot else "-", f"{sum(watts):.0f}W" if watts else "-",
                     f"{sum(vram) / 2**30:.1f}GiB" if vram else "-"])
    return _table(rows)


def _hide_managed_fields(obj):
    """What kubectl does unless --show-managed-fields: managedFields are noise in -o yaml/json."""
    if isinstance(obj, dict):
        if isinstance(obj.get("metadata"), dict) and "managedFields" in obj["metadata"]:
            obj = {**obj, "metadata": {k: v for k, v in obj["metadata"].items() if k != "managedFields"}}
        if isinstance(obj.get("items"), list):
            obj = {**obj, "items": [_hide_managed_fields(i) for i in obj["items"]]}
    return obj


def _print(obj, output: str | None, show_managed: bool = False) -> None:
    if not show_managed:
        obj = _hide_managed_fields(obj)
    if output == "json":
        print(json.dumps(obj, indent=2))
    else:
        print(yaml.safe_dump(obj, sort_keys=False).rstrip())


def _device_line(d: dict) -> str:
    line = f"  {d['id']}: {d['health']} {d.get('gfx', '')} {d.get('pciBusId', '')}".rstrip()
    if d.get("reason"):
        line += f" ({d['reason']})"
    t = d.get("telemetry") or {}
    if t:
        hot = t.get("temp_c", {}).get("hotspot")
        watts = t.get("power", {}).get("current_w")
        ecc = t.get("ecc", {})
        line += (f"  hotspot={hot}C" if hot is not None else "") + (f" power={watts}W" if watts is not None else "")
        if ecc:
            line += f" ecc(ue/ce)={ecc.get('uncorrectable', 0)}/{ecc.get('correctable', 0)}"
    return line


def _platform(workdir: str) -> str:
    try:
        for line in (Path(workdir) / "config").read_text().splitlines():
            if line.startswith("TK8S_PLATFORM="):
                return line.split("=", 1)[1].strip().strip('"')
    except OSError:
        pass
    return "tk8s"


def _real_kubectl(argv: list[str], kubeconfig: Path) -> int:
    """The kubeadm platform is a real Kubernetes: hand the command to the real kubectl with the
    kubeconfig the kubeadmmaster role fetched (ansible/tmp/kubeconfig)."""
    import shutil
    import subprocess

    here = Path(__file__).resolve().parents[2]
    exe = next((c for c in (shutil.which("kubectl", path=p) for p in os.environ.get("PATH", "").split(os.pathsep))
                if c and Path(c).resolve().parent != here), None)
    if exe is None:
        print(f"this cluster runs real Kubernetes (--platform kubeadm): install kubectl and run\n"
              f"    KUBECONFIG={kubeconfig} kubectl {' '.join(argv)}", file=sys.stderr)
        return 1
    return subprocess.run([exe, *argv], env={**os.environ, "KUBECONFIG": str(kubeconfig)}).returncode


def main(argv: list[str] | None = None, workdir: str | None = None) -> int:
    ap = argparse.ArgumentParser(prog="kubectl")
    ap.add_argument("--kubeconfig")
    ap.add_argument("-n", "--namespace", default="default")
    ap.add_argument("-A", "--all-namespaces", action="store_true")
    ap.add_argument("-o", "--output")
    ap.add_argument("-l", "--selector")
    ap.add_argument("-f", "--filename")
    ap.add_argument("-k", "--kustomize")
    ap.add_argument("--tail", type=int, default=0)
    ap.add_argument("--timeout", default="300s")
    ap.add_argument("--replicas", type=int)
    ap.add_argument("--from-literal", action="append", default=[])
    ap.add_argument("--from-file", action="append", default=[])
    ap.add_argument("--ignore-daemonsets", action="store_true")
    ap.add_argument("--follow", dest="follow", action="store_true")
    ap.add_argument("--previous", action="store_true")
    ap.add_argument("--all-containers", action="store_true")
    ap.add_argument("--prefix", action="store_true")
    ap.add_argument("--image")
    ap.add_argument("--port", type=int)
    ap.add_argument("--target-port", type=int)
    ap.add_argument("--type")  # a Service type (expose) or a patch type (patch)
    ap.add_argument("--name")
    ap.add_argument("--server-side", action="store_true")
    ap.add_argument("--force-conflicts", action="store_true")
    ap.add_argument("--field-manager", default="kubectl")
    ap.add_argument("--dry-run", choices=["none", "client", "server"], default="none")
    ap.add_argument("--show-managed-fields", action="store_true")
    ap.add_argument("--address", default="127.0.0.1")
    ap.add_argument("-c", "--container")
    ap.add_argument("-i", "--stdin", action="store_true")  # exec: pass stdin (with -t: interactive)
    ap.add_argument("-t", "--tty", action="store_true")    # exec: a terminal in the pod
    ap.add_argument("--rm", action="store_true")           # run -it: delete the pod after the session
    ap.add_argument("-q", "--quiet", action="store_true")
    ap.add_argument("--to-revision", type=int, default=0)
    ap.add_argument("--for", dest="for_")
    ap.add_argument("--disable-eviction", action="store_true")
    ap.add_argument("--delete-emptydir-data", action="store_true")  # (accepted: emptyDirs go with their pod)
    ap.add_argument("--force", action="store_true")
    # run / set / autoscale / patch / api-resources / auth (kubectl_more.py)
    ap.add_argument("--env", action="append", default=[])
    ap.add_argument("--labels")
    ap.add_argument("--restart", choices=["Always", "OnFailure", "Never"])
    ap.add_argument("--limits")
    ap.add_argument("--requests")
    ap.add_argument("--command", dest="command_flag", action="store_true")
    ap.add_argument("-p", "--patch")
    ap.add_argument("--min", type=int)
    ap.add_argument("--max", type=int)
    ap.add_argument("--cpu-percent", type=int)
    ap.add_argument("--namespaced", choices=["true", "false"])
    ap.add_argument("--subresource")
    ap.add_argument("--cascade", choices=["background", "foreground", "orphan"])
    ap.add_argument("--grace-period", type=int)
    ap.add_argument("--sort-by")
    ap.add_argument("--from", dest="from_")
    ap.add_argument("-w", "--watch", action="store_true")
    ap.add_argument("--wait", choices=["true", "false"], default="true")
    ap.add_argument("verb")
    ap.add_argument("args", nargs="*")
    argv = list(sys.argv[1:] if argv is None else argv)
    wd = workdir or os.environ.get("TK8S_WORKDIR", os.getcwd())
    if "--kubeconfig" not in argv and not os.environ.get("KUBECONFIG") and _platform(wd) == "kubeadm":
        return _real_kubectl(argv, Path(wd) / "ansible" / "tmp" / "kubeconfig")
    command: list[str] = []
    if "--" in argv:  # kubectl exec POD -- CMD ARGS...
        command = argv[argv.index("--") + 1:]
        argv = argv[:argv.index("--")]
    if argv[:1] in (["exec"], ["attach"], ["run"]):  # `kubectl exec -it POD`: flags may precede the name
        flags = [x for x in argv if x in ("-i", "-t", "-it", "-ti", "--stdin", "--tty", "--rm", "-q", "--quiet")]
        argv = [x for x in argv if x not in flags] + flags
    if argv[:1] == ["logs"]:  # `-f` means --filename and `-p` --patch everywhere but logs
        argv = [{"-f": "--follow", "-p": "--previous"}.get(x, x) for x in argv]
    a = ap.parse_intermixed_args(argv) if argv[:1] in (["run"], ["attach"]) else ap.parse_args(argv)
    a.command = command
    workdir = workdir or os.environ.get("TK8S_WORKDIR", os.getcwd())
    if a.verb == "kustomize":  # a local build: no cluster needed
        return more_dispatch(None, a, a.namespace, {})
    try:
        cfg = _load_kubeconfig(a.kubeconfig, workdir)
        if a.verb == "config":
            return more_dispatch(None, a, a.namespace, cfg)
        k = client_from_kubeconfig(cfg)
    except (OSError, ValueError, KeyError, StopIteration) as e:
        print(f"error: no usable kubeconfig ({e}); run ./setup.sh first", file=sys.stderr)
        return 1
    ns = a.namespace
    try:
        from ..kube import KINDS, learn_kind

        for word in ([a.args[0].split("/")[0]] if a.args and a.verb in ("get", "describe", "delete", "label", "annotate")
                     else []):
            if kind_key(word) not in KINDS and kind_key(word) not in ("node", "namespace"):
                learn_kind(k, word)  # a custom resource: ask discovery where it lives
        if a.verb in ("version",):
            print(json.dumps(k.get("/version"), indent=1))
        elif a.verb in MORE_VERBS:
            return more_dispatch(k, a, ns, cfg)
        elif a.verb == "cluster-info":
            print(f"Kubernetes control plane is running at {k.base}{k.prefix}")
        elif a.verb == "get" and a.args[:1] == ["all"]:
            # the "all" category: every workload kind and Services, one table each (empty ones left out)
            first = True
            for kind in ("pod", "service", "daemonset", "deployment", "replicaset", "statefulset", "job", "cronjob",
                         "horizontalpodautoscaler"):
                path = ("/api/v1/pods" if kind == "pod" else collection_path(kind).replace("/namespaces/default", "")) \
                    if a.all_namespaces else collection_path(kind, ns)
                items = k.get(k.k8s(path), query={"labelSelector": a.selector} if a.selector else None)["items"]
                if not items:
                    continue
                for o in items:
                    o["metadata"] = {**o["metadata"], "name": f"{kind}/{o['metadata']['name']}"}
                table = fmt_pods(items, a.output == "wide", a.all_namespaces) if kind == "pod" else \
                    fmt_generic(kind, items, a.all_namespaces)
                print(("" if first else "\n") + table)
                first = False
            if first:
                print(f"No resources found in {ns} namespace.")
        elif a.verb == "get":
            what = kind_key(a.args[0]) if a.args else "pod"
            name = a.args[1] if len(a.args) > 1 else None
            if "/" in (a.args[0] if a.args else ""):
                what, name = kind_key(a.args[0].split("/")[0]), a.args[0].split("/")[1]
            q = {"labelSelector": a.selector} if a.selector else None
            if name:
                obj = k.get(k.k8s(f"/api/v1/nodes/{name}" if what == "node" else object_path(what, name, ns)))
                if a.output in ("json", "yaml"):
                    _print(obj, a.output, a.show_managed_fields)
                    return 0
                items = [obj]  # a one-row table, as kubectl prints it
            elif what == "node":
                items = k.get(k.k8s("/api/v1/nodes"), query=q)["items"]
            elif a.all_namespaces:
                path = "/api/v1/pods" if what == "pod" else collection_path(what).replace("/namespaces/default", "")
                items = k.get(k.k8s(path), query=q)["items"]
            else:
                items = k.get(k.k8s(collection_path(what, ns)), query=q)["items"]
            if a.sort_by:
                def key(o):
                    v = (_jsonpath_all(o, a.sort_by) or [""])[0]
                    return (0, float(v), "") if isinstance(v, (int, float)) else (1, 0.0, _fmt_value(v))
                items.sort(key=key)
            out = (a.output or "")
            if out in ("json", "yaml"):
                _print({"apiVersion": "v1", "kind": "List", "items": items} if not name else items[0], a.output,
                       a.show_managed_fields)
            elif out == "name":
                print("\n".join(f"{what}/{o['metadata']['name']}" for o in items))
            elif out.startswith("jsonpath="):
                print(render_jsonpath({"apiVersion": "v1", "kind": "List", "items": items} if not name else items[0],
                                      out[len("jsonpath="):]))
            elif out.startswith("custom-columns="):
                print(render_custom_columns(items, out[len("custom-columns="):]))
            elif what == "node":
                print(fmt_nodes(items, a.output == "wide"))
            elif what == "pod":
                print(fmt_pods(items, a.output == "wide", a.all_namespaces))
            else:
                print(fmt_generic(what, items, a.all_namespaces))
            if a.watch:  # -w: a row per change until --timeout (kubectl runs until interrupted)
                return _watch_rows(k, what, ns, name, q, a)
        elif a.verb == "describe":
            what, name = _target(a.args)
            what = kind_key(what)
            o = k.get(k.k8s(f"/api/v1/nodes/{name}" if what == "node" else object_path(what, name, ns)))
            print(f"Name:         {o['metadata']['name']}")
            print(f"Labels:       {', '.join(f'{x}={y}' for x, y in o['metadata'].get('labels', {}).items())}")
            print(f"Annotations:  {', '.join(f'{x}={y}' for x, y in o['metadata'].get('annotations', {}).items())}")
            st = o.get("status", {})
            if what == "node":
                print("Capacity:\n" + "\n".join(f"  {x}: {y}" for x, y in st.get("capacity", {}).items()))
                print("Allocatable:\n" + "\n".join(f"  {x}: {y}" for x, y in st.get("allocatable", {}).items()))
                print("Devices:\n" + "\n".join(_device_line(d) for d in st.get("devices", [])))
                taints = (o.get("spec") or {}).get("taints") or []
                print("Taints:       " + (", ".join(f"{t['key']}{'=' + str(t['value']) if t.get('value') else ''}:{t['effect']}"
                                                   for t in taints) or "<none>"))
                print(f"Unschedulable: {str(bool((o.get('spec') or {}).get('unschedulable'))).lower()}")
                enf = o["metadata"].get("annotations", {}).get("tk8s.amd.com/resource-enforcement")
                if enf:
                    print(f"Resource enforcement: {enf}")
                pods = [p for p in k.get(k.k8s("/api/v1/pods"), query={"fieldSelector": f"spec.nodeName={name}"})["items"]
                        if p.get("status", {}).get("phase") not in ("Succeeded", "Failed")]
                used = sum(int(((c.get("resources") or {}).get("limits") or {}).get(GPU, 0) or 0)
                           for p in pods for c in p["spec"].get("containers", []))
                print(f"Non-terminated Pods: ({len(pods)} in total)\n"
                      + "".join(f"  {p['metadata'].get('namespace', 'default'):<14} {p['metadata']['name']}\n" for p in pods)
                      + f"Allocated resources:\n  {GPU}: {used} of {st.get('allocatable', {}).get(GPU, '0')}")
            print("Conditions:\n" + "\n".join(f"  {c['type']:<18} {c['status']:<8} {c.get('reason', '')}  {c.get('message', '')}"
                                              for c in st.get("conditions", [])))
            if what == "pod":
                status = st.get("phase")
                if o["metadata"].get("deletionTimestamp"):
                    status = (f"Terminating (lasts until {o['metadata']['deletionTimestamp']}, grace period "
                              f"{o['metadata'].get('deletionGracePeriodSeconds', '?')}s)")
                print(f"Node:         {o['spec'].get('nodeName')}\nStatus:       {status}")
                if o["spec"].get("priorityClassName") or o["spec"].get("priority"):
                    print(f"Priority:     {o['spec'].get('priority', 0)} ({o['spec'].get('priorityClassName', '')})")
                vols = o["spec"].get("volumes") or []
                if vols:
                    print("Volumes:\n" + "\n".join(f"  {v.get('name')}: {next((k for k in v if k != 'name'), '?')}"
                                                   for v in vols))
                ann = o["metadata"].get("annotations", {})
                if "tk8s.amd.com/gpu-isolation" in ann or "tk8s.amd.com/isolation" in ann:
                    print("Isolation:\n"
                          f"  GPU:        {ann.get('tk8s.amd.com/gpu-isolation', '-')}\n"
                          f"  Namespaces: {ann.get('tk8s.amd.com/isolation', '-')}\n"
                          f"  Resources:  {ann.get('tk8s.amd.com/resources', '-')}")
                for c in st.get("containerStatuses") or []:
                    term = (c.get("state") or {}).get("terminated") or ((c.get("lastState") or {}).get("terminated"))
                    if term:
                        which = "State" if "terminated" in (c.get("state") or {}) else "Last State"
                        print(f"  {c.get('name')}: {which}: Terminated, Reason: {term.get('reason')}, "
                              f"Exit Code: {term.get('exitCode')}, Restart Count: {c.get('restartCount', 0)}")
            # the object's events, selected as kubectl describe does (kind, name, namespace, uid)
            sel = f"involvedObject.kind={o.get('kind', '')},involvedObject.name={o['metadata']['name']}"
            if o["metadata"].get("uid"):
                sel += f",involvedObject.uid={o['metadata']['uid']}"
            try:
                evs = k.get(k.k8s(f"/api/v1/namespaces/{ns if what != 'node' else 'default'}/events"),
                            query={"fieldSelector": sel})["items"]
            except ApiError:
                evs = []
            print("Events:" + ("  <none>" if not evs else ""))
            for e in evs[-20:]:
                print(f"  {e.get('type', ''):<8} {e.get('reason', ''):<20} {e.get('message', '')}")
        elif a.verb == "create" and a.args and a.args[0] in ("configmap", "cm", "secret"):
            return _create_data(k, a, ns)
        elif a.verb == "create" and a.args and kind_key(a.args[0]) == "namespace":
            if len(a.args) < 2:
                raise SystemExit("usage: kubectl create namespace NAME")
            k.post(k.k8s("/api/v1/namespaces"), {"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": a.args[1]}})
            print(f"namespace/{a.args[1]} created")
        elif a.verb == "create" and a.args and kind_key(a.args[0]) == "deployment":
            return _create_deployment(k, a, ns)
        elif a.verb == "create" and a.args and kind_key(a.args[0]) == "job":
            return _create_job(k, a, ns)
        elif a.verb == "expose":
            return _expose(k, a, ns)
        elif a.verb == "apply" and a.server_side:
            for r in server_apply_objects(k, _manifests(a), a.field_manager, a.force_conflicts,
                                          dry_run=a.dry_run == "server"):
                print(f"{r['kind'].lower()}/{r['name']} {r['action']}" + (" (server dry run)" if a.dry_run == "server" else ""))
        elif a.verb in ("create", "apply"):
            res = apply_objects(k, _manifests(a))
            for r in res:
                print(f"{r['kind'].lower()}/{r['name']} {r['action'] if a.verb == 'apply' else ('created' if r['created'] else 'unchanged')}")
        elif a.verb == "scale":
            what, name = _target(a.args)
            if a.replicas is None or kind_key(what) not in ("deployment", "statefulset", "replicaset"):
                raise SystemExit("usage: kubectl scale deploy|sts|rs/NAME --replicas N")
            k.request("PATCH", k.k8s(object_path(kind_key(what), name, ns) + "/scale"), body={"spec": {"replicas": a.replicas}},
                      query={"fieldManager": "kubectl-scale"})
            print(f"{kind_key(what)}.apps/{name} scaled")
        elif a.verb == "rollout":
            sub = a.args[0] if a.args else ""
            what, name = _target(a.args[1:])
            if kind_key(what) in ("statefulset", "daemonset") and sub in ("status", "restart"):
                return _rollout_other(k, kind_key(what), name, ns, sub, float(a.timeout.rstrip("s")))
            if kind_key(what) != "deployment" or sub not in ("status", "restart", "history", "undo", "pause", "resume"):
                raise SystemExit("usage: kubectl rollout status|restart|history|undo|pause|resume deploy/NAME")
            if sub in ("pause", "resume"):
                from .kubectl_more import rollout_pause

                return rollout_pause(k, name, ns, sub == "pause")
            if sub in ("history", "undo"):
                return _rollout_history(k, name, ns, sub, a.to_revision)
            if sub == "restart":  # a new template annotation = a new pod-template-hash = a rolling update
                k.request("PATCH", k.k8s(object_path("deployment", name, ns)), body={"spec": {"template": {"metadata": {
                    "annotations": {"kubectl.kubernetes.io/restartedAt": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())}}}}})
                print(f"deployment.apps/{name} restarted")
                return 0

            def progress(d):
                st, want = d.get("status", {}), d["spec"].get("replicas", 1)
                print(f'Waiting for deployment "{name}" rollout to finish: {st.get("updatedReplicas", 0)} of {want} '
                      f'updated replicas are available...', flush=True)

            wait_rollout(k, name, ns, timeout=float(a.timeout.rstrip("s")), progress=progress)
            print(f'deployment "{name}" successfully rolled out')
        elif a.verb in ("label", "annotate"):
            what, name = _target(a.args)
            pairs = a.args[1:] if "/" in a.args[0] else a.args[2:]
            field = "labels" if a.verb == "label" else "annotations"
            patch = {}
            for kv in pairs:
                if kv.endswith("-") and "=" not in kv:
                    patch[kv[:-1]] = None
                else:
                    key, _, val = kv.partition("=")
                    patch[key] = val
            path = f"/api/v1/nodes/{name}" if kind_key(what) == "node" else object_path(what, name, ns)
            k.request("PATCH", k.k8s(path), body={"metadata": {field: patch}})
            print(f"{kind_key(what)}/{name} {'labeled' if a.verb == 'label' else 'annotated'}")
        elif a.verb == "drain":
            return _drain(k, a.args[0], float(a.timeout.rstrip("s")), a.disable_eviction)
        elif a.verb == "top":
            if not a.args or kind_key(a.args[0]) not in ("node", "pod"):
                raise SystemExit("usage: kubectl top nodes|pods")
            if kind_key(a.args[0]) == "node":
                try:
                    usage = {m["metadata"]["name"]: m["usage"] for m in
                             k.get(k.k8s("/apis/metrics.k8s.io/v1beta1/nodes"))["items"]}
                except ApiError:
                    usage = {}
                print(fmt_top(k.get(k.k8s("/api/v1/nodes"))["items"], k.get(k.k8s("/api/v1/pods"))["items"], usage))
            else:  # the resource metrics API (metrics.k8s.io), as a stock kubectl top pods reads it
                from ..utils import quantity

                path = "/apis/metrics.k8s.io/v1beta1/" + ("pods" if a.all_namespaces else f"namespaces/{ns}/pods")
                items = k.get(k.k8s(path), query={"labelSelector": a.selector} if a.selector else None)["items"]
                rows = [["NAME", "CPU(cores)", "MEMORY(bytes)"]] + [[
                    m["metadata"]["name"],
                    f"{int(sum(quantity.parse(c['usage']['cpu']) for c in m['containers']) * 1000)}m",
                    f"{int(sum(quantity.parse(c['usage']['memory']) for c in m['containers']) / 2**20)}Mi"] for m in items]
                print(_table(rows))
        elif a.verb == "delete":
            if a.filename or a.kustomize:
                n = delete_objects(k, _manifests(a))
            else:
                what, name = kind_key(a.args[0].split("/")[0]), (a.args[0].split("/", 1)[1] if "/" in a.args[0] else a.args[1])
                q = {**({"propagationPolicy": a.cascade.capitalize()} if a.cascade else {}),
                     **({"gracePeriodSeconds": "0"} if a.force else {"gracePeriodSeconds": str(a.grace_period)}
                        if a.grace_period is not None and a.grace_period >= 0 else {})}
                path = k.k8s(f"/api/v1/nodes/{name}" if what == "node" else object_path(what, name, ns))
                out = k.delete(path, query=q or None)
                if a.wait != "false" and isinstance(out, dict) and (out.get("metadata") or {}).get("deletionTimestamp"):
                    # a Terminating pod (or an object held by finalizers): wait until it is gone, as kubectl does
                    deadline = time.monotonic() + float(a.timeout.rstrip("s"))
                    while time.monotonic() < deadline:
                        try:
                            k.get(path)
                        except ApiError as e:
                            if e.status == 404:
                                break
                            raise
                        time.sleep(0.1)
                n = 1
            print(f"{n} object(s) deleted")
        elif a.verb == "logs" and (a.selector or a.all_containers or a.previous or (a.args and "/" in a.args[0])):
            return _logs_many(k, ns, a)
        elif a.verb == "logs":
            path = k.k8s(object_path("pod", a.args[0], ns) + "/log")
            full = k.get(path, query={"container": a.container}, raw=True)  # one read: nothing slips between
            text = "".join(full.splitlines(keepends=True)[-a.tail:]) if a.tail else full
            print(text, end="", flush=True)
            if a.follow:  # -f: print what the pod appends until it terminates
                seen = len(full)
                while True:
                    phase = k.get(k.k8s(object_path("pod", a.args[0], ns))).get("status", {}).get("phase")
                    full = k.get(path, query={"container": a.container}, raw=True)
                    print(full[seen:], end="", flush=True)
                    seen = len(full)
                    if phase in ("Succeeded", "Failed"):
                        break
                    time.sleep(0.2)
        elif a.verb == "exec":
            if not a.command:
                raise SystemExit("usage: kubectl exec [-it] POD -- COMMAND [ARGS...]")
            if a.tty:  # interactive: a terminal in the pod, bytes streaming both ways
                from .kubectl_streams import exec_tty

                return exec_tty(k, ns, a.args[0], a.command, a.stdin)
            r = k.post(k.k8s(object_path("pod", a.args[0], ns) + "/exec"),
                       {"command": a.command, "timeoutSeconds": float(a.timeout.rstrip("s"))},
                       timeout=float(a.timeout.rstrip("s")) + 30)
            sys.stdout.write(r.get("stdout", ""))
            sys.stderr.write(r.get("stderr", ""))
            return int(r.get("exitCode", 1))
        elif a.verb == "port-forward":
            from .kubectl_streams import port_forward

            if not a.args:
                raise SystemExit("usage: kubectl port-forward TYPE/NAME [LOCAL_PORT:]REMOTE_PORT ...")
            return port_forward(k, ns, a.args[0], a.args[1:], a.address)
        elif a.verb == "attach":
            from .kubectl_streams import attach

            what, name = _target(a.args) if "/" in (a.args[0] if a.args else "") else ("pod", (a.args or [""])[0])
            if a.stdin or a.tty:
                from .kubectl_streams import attach_interactive

                return attach_interactive(k, ns, name, a.stdin, a.tty, a.container, quiet=a.quiet)
            return attach(k, ns, name)
        elif a.verb == "taint":
            # kubectl taint nodes NAME key[=value]:Effect ... (a trailing "-" removes the taint)
            what, name = _target(a.args)
            if kind_key(what) != "node":
                raise SystemExit("usage: kubectl taint nodes NAME key[=value]:Effect[-] ...")
            node = k.get(k.k8s(f"/api/v1/nodes/{name}"))
            taints = list((node.get("spec") or {}).get("taints") or [])
            for spec in (a.args[1:] if "/" in a.args[0] else a.args[2:]):
                remove = spec.endswith("-")
                kv, _, effect = spec.rstrip("-").partition(":")
                key, _, value = kv.partition("=")
                taints = [t for t in taints if not (t.get("key") == key and (not effect or t.get("effect") == effect))]
                if not remove:
                    taints.append({"key": key, **({"value": value} if value else {}), "effect": effect or "NoSchedule"})
            k.request("PATCH", k.k8s(f"/api/v1/nodes/{name}"), body={"spec": {"taints": taints}})
            print(f"node/{name} {'untainted' if all(s.endswith('-') for s in a.args[1:]) else 'tainted'}")
        elif a.verb == "cp":
            return _cp(k, ns, a.args, a.container)
        elif a.verb in ("cordon", "uncordon"):
            k.request("PATCH", k.k8s(f"/api/v1/nodes/{a.args[0]}"), body={"spec": {"unschedulable": a.verb == "cordon"}})
            print(f"node/{a.args[0]} {a.verb}ed")
        elif a.verb == "wait" and getattr(a, "for_", None):
            return _wait(k, ns, a.args, a.for_, a.selector, float(a.timeout.rstrip("s")))
        elif a.verb == "wait":
            what, name = a.args[0].split("/", 1)
            if kind_key(what) != "job":
                raise SystemExit("wait without --for is job/NAME only (until Complete or Failed)")
            j = wait_job(k, name, ns, timeout=float(a.timeout.rstrip("s")))
            print(f"job.batch/{name} condition met ({job_state(j)})")
            return 0 if job_state(j) == "Complete" else 1
        else:
            print(f"error: unknown command {a.verb!r}", file=sys.stderr)
            return 1
    except ApiError as e:
        print(f"Error from server: {e}", file=sys.stderr)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
