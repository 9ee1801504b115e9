"""Kubernetes object helpers shared by kubectl, the playbook's tk8s_kube module and setup.

Maps kinds to API paths, loads (templated) multi-document manifests, applies/deletes objects and
waits for conditions with the control plane's long-poll watch (no sleep loops).
"""
from __future__ import annotations

import time
from pathlib import Path

from . import templating
from .controlplane.client import ApiError, Client
from .utils import yamlio

KINDS = {
    "pod": ("Pod", "/api/v1", "pods"),
    "service": ("Service", "/api/v1", "services"),
    "event": ("Event", "/api/v1", "events"),
    "daemonset": ("DaemonSet", "/apis/apps/v1", "daemonsets"),
    "deployment": ("Deployment", "/apis/apps/v1", "deployments"),
    "job": ("Job", "/apis/batch/v1", "jobs"),
}
ALIASES = {"po": "pod", "pods": "pod", "svc": "service", "services": "service", "ds": "daemonset",
           "daemonsets": "daemonset", "deploy": "deployment", "deployments": "deployment", "jobs": "job",
           "ev": "event", "events": "event", "no": "node", "nodes": "node"}


def kind_key(kind: str) -> str:
    k = kind.lower()
    return ALIASES.get(k, k)


def collection_path(kind: str, ns: str = "default") -> str:
    k = kind_key(kind)
    if k == "node":
        return "/api/v1/nodes"
    if k not in KINDS:
        raise ValueError(f"unsupported kind {kind!r}")
    _, group, plural = KINDS[k]
    return f"{group}/namespaces/{ns}/{plural}"


def object_path(kind: str, name: str, ns: str = "default") -> str:
    return f"{collection_path(kind, ns)}/{name}"


def load_manifests(path: str | Path, variables: dict | None = None) -> list[dict]:
    docs = [d for d in yamlio.load_all(Path(path).read_text()) if d]
    if variables:
        docs = templating.render(docs, variables)
    out = []
    for d in docs:
        if d.get("kind") == "List":
            out += d.get("items", [])
        else:
            out.append(d)
    return out


def apply_objects(k: Client, objs: list[dict]) -> list[dict]:
    res = []
    for o in objs:
        kind = o.get("kind", "")
        if kind.lower() == "namespace":
            res.append({"kind": kind, "name": o["metadata"]["name"], "created": False})
            continue
        ns = o.get("metadata", {}).get("namespace", "default")
        try:
            k.post(k.k8s(collection_path(kind, ns)), o)
            res.append({"kind": kind, "name": o["metadata"].get("name"), "created": True})
        except ApiError as e:
            if e.status != 409:
                raise
            res.append({"kind": kind, "name": o["metadata"].get("name"), "created": False})
    return res


def delete_objects(k: Client, objs: list[dict]) -> int:
    n = 0
    for o in objs:
        kind = o.get("kind", "")
        if kind.lower() == "namespace":
            continue
        ns = o.get("metadata", {}).get("namespace", "default")
        try:
            k.delete(k.k8s(object_path(kind, o["metadata"]["name"], ns)))
            n += 1
        except ApiError as e:
            if e.status != 404:
                raise
    return n


def job_state(job: dict) -> str:
    for c in job.get("status", {}).get("conditions", []):
        if c.get("type") in ("Complete", "Failed") and c.get("status") == "True":
            return c["type"]
    return "Running"


def wait_job(k: Client, name: str, ns: str = "default", timeout: float = 300.0) -> dict:
    """Block (long-poll watch) until the Job is Complete or Failed; returns the Job."""
    deadline = time.monotonic() + timeout
    path = k.k8s(collection_path("job", ns))
    rv = 0
    while True:
        job = k.get(k.k8s(object_path("job", name, ns)))
        if job_state(job) != "Running":
            return job
        left = deadline - time.monotonic()
        if left <= 0:
            raise TimeoutError(f"job {ns}/{name} not finished after {timeout}s")
        rv = max(rv, int(job["metadata"]["resourceVersion"]))
        rv, _ = k.watch(path, rv, timeout=min(left, 20.0))


def pods_of(k: Client, label_selector: str, ns: str = "default") -> list[dict]:
    return k.get(k.k8s(collection_path("pod", ns)), query={"labelSelector": label_selector})["items"]
