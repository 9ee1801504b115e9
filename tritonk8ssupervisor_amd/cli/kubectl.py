"""Minimal kubectl for the tk8s control plane (the CLI half of docs/detailed.md:285-370).

  kubectl get nodes|pods|ds|jobs|deploy|svc|events [-n NS | -A] [-l k=v] [-o wide|json|yaml]
  kubectl describe node NAME | pod NAME
  kubectl create|apply -f FILE        kubectl delete -f FILE | KIND NAME
  kubectl logs POD [--tail N]         kubectl cordon|uncordon NODE
  kubectl wait job/NAME [--timeout S] kubectl cluster-info | version

The kubeconfig comes from --kubeconfig, $KUBECONFIG, or <workdir>/.tk8s/kubeconfig.json (written
by setup; the same document the control plane serves at /env/<env>/kubernetes/kubectl).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import yaml

from ..controlplane.client import ApiError, client_from_kubeconfig
from ..kube import (apply_objects, collection_path, delete_objects, job_state, kind_key, load_manifests,
                    object_path, wait_job)

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
    elif k == "deployment":
        rows = [["NAME", "READY", "AGE"]] + [[o["metadata"]["name"],
                f"{o.get('status', {}).get('readyReplicas', 0)}/{o['spec'].get('replicas', 1)}", _age(o)] for o in items]
    elif k == "service":
        def ports(o):
            return ",".join(f"{p['port']}" + (f":{p['nodePort']}" if p.get("nodePort") else "") + f"/{p.get('protocol', 'TCP')}"
                            for p in o["spec"].get("ports", []))

        def ext(o):
            ing = o.get("status", {}).get("loadBalancer", {}).get("ingress") or []
            return ",".join(i.get("ip", "") for i in ing) or ("<pending>" if o["spec"].get("type") == "LoadBalancer" else "<none>")

        rows = [["NAME", "TYPE", "CLUSTER-IP", "EXTERNAL-IP", "PORT(S)", "AGE"]] + [[
            o["metadata"]["name"], o["spec"].get("type", "ClusterIP"), o["spec"].get("clusterIP", ""), ext(o), ports(o), _age(o)]
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


def _print(obj, output: str | None) -> None:
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


def main(argv: list[str] | None = None, workdir: str | None = None) -> int:
    ap = argparse.ArgumentParser(prog="kubectl")
    ap.add_argument("--kubeconfig")
    ap.add_argument("-n", "--namespace", default="default")
    ap.add_argument("-A", "--all-namespaces", action="store_true")
    ap.add_argument("-o", "--output")
    ap.add_argument("-l", "--selector")
    ap.add_argument("-f", "--filename")
    ap.add_argument("--tail", type=int, default=0)
    ap.add_argument("--timeout", default="300s")
    ap.add_argument("verb")
    ap.add_argument("args", nargs="*")
    a = ap.parse_args(argv)
    workdir = workdir or os.environ.get("TK8S_WORKDIR", os.getcwd())
    try:
        k = client_from_kubeconfig(_load_kubeconfig(a.kubeconfig, workdir))
    except (OSError, ValueError, KeyError, StopIteration) as e:
        print(f"error: no usable kubeconfig ({e}); run ./setup.sh first", file=sys.stderr)
        return 1
    ns = a.namespace
    try:
        if a.verb in ("version",):
            print(json.dumps(k.get("/version"), indent=1))
        elif a.verb == "cluster-info":
            print(f"Kubernetes control plane is running at {k.base}{k.prefix}")
        elif a.verb == "get":
            what = kind_key(a.args[0]) if a.args else "pod"
            name = a.args[1] if len(a.args) > 1 else None
            if "/" in (a.args[0] if a.args else ""):
                what, name = kind_key(a.args[0].split("/")[0]), a.args[0].split("/")[1]
            q = {"labelSelector": a.selector} if a.selector else None
            if name:
                _print(k.get(k.k8s(f"/api/v1/nodes/{name}" if what == "node" else object_path(what, name, ns))), a.output or "yaml")
                return 0
            if what == "node":
                items = k.get(k.k8s("/api/v1/nodes"), query=q)["items"]
            elif a.all_namespaces:
                path = {"pod": "/api/v1/pods", "event": "/api/v1/events", "daemonset": "/apis/apps/v1/daemonsets",
                        "job": "/apis/batch/v1/jobs"}.get(what)
                items = k.get(k.k8s(path), query=q)["items"] if path else []
            else:
                items = k.get(k.k8s(collection_path(what, ns)), query=q)["items"]
            if a.output in ("json", "yaml"):
                _print({"apiVersion": "v1", "kind": "List", "items": items}, a.output)
            elif what == "node":
                print(fmt_nodes(items, a.output == "wide"))
            elif what == "pod":
                print(fmt_pods(items, a.output == "wide", a.all_namespaces))
            else:
                print(fmt_generic(what, items, a.all_namespaces))
        elif a.verb == "describe":
            what, name = kind_key(a.args[0]), a.args[1]
            o = k.get(k.k8s(f"/api/v1/nodes/{name}" if what == "node" else object_path(what, name, ns)))
            print(f"Name:         {o['metadata']['name']}")
            print(f"Labels:       {', '.join(f'{x}={y}' for x, y in o['metadata'].get('labels', {}).items())}")
            print(f"Annotations:  {', '.join(f'{x}={y}' for x, y in o['metadata'].get('annotations', {}).items())}")
            st = o.get("status", {})
            if what == "node":
                print("Capacity:\n" + "\n".join(f"  {x}: {y}" for x, y in st.get("capacity", {}).items()))
                print("Allocatable:\n" + "\n".join(f"  {x}: {y}" for x, y in st.get("allocatable", {}).items()))
                print("Devices:\n" + "\n".join(_device_line(d) for d in st.get("devices", [])))
            print("Conditions:\n" + "\n".join(f"  {c['type']:<18} {c['status']:<8} {c.get('reason', '')}  {c.get('message', '')}"
                                              for c in st.get("conditions", [])))
            if what == "pod":
                print(f"Node:         {o['spec'].get('nodeName')}\nStatus:       {st.get('phase')}")
        elif a.verb in ("create", "apply"):
            res = apply_objects(k, load_manifests(a.filename))
            for r in res:
                print(f"{r['kind'].lower()}/{r['name']} {'created' if r['created'] else 'unchanged'}")
        elif a.verb == "delete":
            if a.filename:
                n = delete_objects(k, load_manifests(a.filename))
            else:
                what, name = kind_key(a.args[0]), a.args[1]
                k.delete(k.k8s(f"/api/v1/nodes/{name}" if what == "node" else object_path(what, name, ns)))
                n = 1
            print(f"{n} object(s) deleted")
        elif a.verb == "logs":
            print(k.get(k.k8s(object_path("pod", a.args[0], ns) + "/log"), query={"tailLines": a.tail or None}, raw=True), end="")
        elif a.verb in ("cordon", "uncordon"):
            k.request("PATCH", k.k8s(f"/api/v1/nodes/{a.args[0]}"), body={"spec": {"unschedulable": a.verb == "cordon"}})
            print(f"node/{a.args[0]} {a.verb}ed")
        elif a.verb == "wait":
            what, name = a.args[0].split("/", 1)
            if kind_key(what) != "job":
                raise SystemExit("only job/NAME is supported by wait")
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
