"""The pod scheduler of the control plane: binds pending pods to Ready nodes with room, counting
the extended resource amd.com/gpu (validated nodes only), the way the AMD k8s-device-plugin
exposes it. A mixin of server.ControlPlane.

Host-scoped GPU pods (``tk8s.amd.com/gpu-scope: host``, the cluster's own RCCL fabric Job only,
objects._admit_gpu_visibility): in the default layout every worker is a one-GPU slice of the same
8x MI355X host, and an all-reduce over them wants ONE process driving all of the host's GPUs
(one runtime start, one ncclCommInitAll) rather than one rank process per node. Such a pod asks
for N amd.com/gpu; the scheduler finds a host (node label ``tk8s.amd.com/host``) whose whole,
idle GPU nodes add up to exactly N, binds the pod to one of them (the leader, whose agent runs it)
and records the claim on the others in the pod's annotations -- ``host-claims`` (GPUs counted
against each node, so nothing else lands there meanwhile) and ``host-devices`` (which devices of
the other nodes the leader's process may open).
"""
from __future__ import annotations

import json

from .objects import (
    GPU, QUOTA_BLOCKED, TERMINAL, _key, _cond, _set_cond, node_ready, node_validated, pod_gpus, labels_match,
)

GPU_SCOPE = "tk8s.amd.com/gpu-scope"
HOST_LABEL = "tk8s.amd.com/host"
HOST_CLAIMS = "tk8s.amd.com/host-claims"
HOST_DEVICES = "tk8s.amd.com/host-devices"
SELECTED_NODE = "volume.kubernetes.io/selected-node"


def pod_claims(o: dict) -> dict[str, int]:
    """amd.com/gpu a bound pod holds per node: its node's share, or a host-scoped pod's claims."""
    ann = o["metadata"].get("annotations") or {}
    if ann.get(HOST_CLAIMS):
        try:
            return {k: int(v) for k, v in json.loads(ann[HOST_CLAIMS]).items()}
        except (ValueError, AttributeError):
            pass
    nn = o["spec"].get("nodeName")
    return {nn: pod_gpus(o)} if nn else {}


class Scheduler:
    def _scheduler(self, pid: str) -> None:
        pending = [o for o in self.store.list("pods", lambda o: self._in(pid, o))
                   if not o["spec"].get("nodeName") and o.get("status", {}).get("phase") == "Pending"]
        if not pending:
            return
        nodes = [n for n in self.store.list("nodes", lambda n: self._in(pid, n))
                 if node_ready(n) and not n["spec"].get("unschedulable")]
        used: dict[str, int] = {}
        count: dict[str, int] = {}
        reqs: dict[str, list[float]] = {}  # node -> [cpu, memory] requested by its pods
        from .objects import pod_usage
        from ..utils import quantity

        for o in self.store.list("pods", lambda o: self._in(pid, o)):
            nn = o["spec"].get("nodeName")
            if nn and o.get("status", {}).get("phase") not in TERMINAL:
                for cn, g in pod_claims(o).items():
                    used[cn] = used.get(cn, 0) + g
                    count[cn] = count.get(cn, 0) + 1
                u = pod_usage(o)
                r = reqs.setdefault(nn, [0.0, 0.0])
                r[0] += u.get("requests.cpu", 0.0)
                r[1] += u.get("requests.memory", 0.0)
        # taints, node affinity, inter-pod (anti-)affinity (placement.py): only when something asks
        rules = any((n.get("spec") or {}).get("taints") for n in nodes) or any(
            p["spec"].get("affinity") or p["spec"].get("tolerations") or p["spec"].get("topologySpreadConstraints")
            for p in pending)
        by_name = {n["metadata"]["name"]: n for n in nodes}
        bound = [o for o in self.store.list("pods", lambda o: self._in(pid, o))
                 if o["spec"].get("nodeName") and o.get("status", {}).get("phase") not in TERMINAL] if rules else []
        # highest priority first (priority.py), then by name
        for pod in sorted(pending, key=lambda o: (-int(o["spec"].get("priority") or 0), o["metadata"]["name"])):
            need = pod_gpus(pod)
            sel = pod["spec"].get("nodeSelector")
            key = _key(pid, pod["metadata"]["namespace"], pod["metadata"]["name"])
            if (pod["metadata"].get("annotations") or {}).get(QUOTA_BLOCKED):
                why = self._quota_block(pid, pod["metadata"]["namespace"], pod["metadata"]["name"], pod)
                if why:
                    continue  # still over its namespace's quota
                self.store.patch("pods", key, lambda o: o["metadata"]["annotations"].pop(QUOTA_BLOCKED, None))
            claims, pinned, missing = self._pod_claims_nodes(pid, pod)
            if missing:
                self._unschedulable(pod, key, f'persistentvolumeclaim "{missing}" not found')
                continue
            if pinned:  # a claim's data lives on one node
                sel = {**(sel or {}), "kubernetes.io/hostname": pinned}
            if (pod["metadata"].get("annotations") or {}).get(GPU_SCOPE) == "host" and need > 0:
                self._schedule_host_scoped(pid, pod, key, need, sel, nodes, used, count)
                continue
            best = None
            why: dict[str, int] = {}
            mine = pod_usage(pod)
            for n in nodes:
                nn = n["metadata"]["name"]
                free = int(n["status"]["allocatable"].get(GPU, 0)) - used.get(nn, 0)
                if need > free or not labels_match(sel, n["metadata"].get("labels")):
                    continue
                if need and not node_validated(n):
                    continue  # GPU pods only land on validated nodes
                alloc = n["status"]["allocatable"]
                short = next((res for i, res in enumerate(("cpu", "memory"))
                              if alloc.get(res) and mine.get(f"requests.{res}", 0.0)
                              and reqs.get(nn, [0.0, 0.0])[i] + mine[f"requests.{res}"] > quantity.parse(alloc[res]) + 1e-9),
                             None)
                if short is None and alloc.get("pods") and count.get(nn, 0) >= int(alloc["pods"]):
                    short = "pods"
                if short is not None:  # the pods' requests do not fit the node's allocatable cpu/memory/pods
                    reason = "Too many pods" if short == "pods" else f"Insufficient {short}"
                    why[reason] = why.get(reason, 0) + 1
                    continue
                pref = 0
                if rules:
                    from . import placement

                    no = placement.feasible(pod, n, by_name, bound)
                    if no:
                        why[no] = why.get(no, 0) + 1
                        continue
                    pref = placement.score(pod, n, by_name, bound)
                score = (-pref, count.get(nn, 0), -free, nn)
                if best is None or score < best[0]:
                    best = (score, nn, free)
            if best is None and not why and int(pod["spec"].get("priority") or 0) > 0:
                nn = self._preempt(pid, pod, key, need, sel, nodes, used)
                if nn is not None:
                    best = (None, nn, 0)
            if best is None:
                extra = "".join(f", {c} node(s) excluded by {w}" for w, c in sorted(why.items()))
                self._unschedulable(pod, key, f"0/{len(nodes)} nodes available: need {need} {GPU}{extra}")
                continue
            nn = best[1]
            used[nn] = used.get(nn, 0) + need
            count[nn] = count.get(nn, 0) + 1
            r = reqs.setdefault(nn, [0.0, 0.0])
            r[0] += mine.get("requests.cpu", 0.0)
            r[1] += mine.get("requests.memory", 0.0)
            if rules:  # what the next pods of this pass see (anti-affinity spreads replicas at once)
                bound.append({**pod, "spec": {**pod["spec"], "nodeName": nn}})
            for c in claims:  # WaitForFirstConsumer: the first pod's node holds the claim's data
                ckey = _key(pid, pod["metadata"]["namespace"], c)
                if SELECTED_NODE not in ((self.store.get("persistentvolumeclaims", ckey) or {}).get("metadata", {})
                                         .get("annotations") or {}):
                    pvc = self.store.patch("persistentvolumeclaims", ckey, lambda o, nn=nn: o["metadata"].setdefault(
                        "annotations", {}).__setitem__(SELECTED_NODE, nn))
                    self._provision_pv(pid, pod["metadata"]["namespace"], pvc, node=nn)
            self._bind(pid, pod, key, nn)

    def _pod_claims_nodes(self, pid: str, pod: dict) -> tuple[list[str], str | None, str | None]:
        """(claims the pod mounts, the node they pin it to, a claim that does not exist)."""
        ns = pod["metadata"]["namespace"]
        claims, pinned = [], None
        for v in pod["spec"].get("volumes") or []:
            c = (v.get("persistentVolumeClaim") or {}).get("claimName")
            if not c:
                continue
            pvc = self.store.get("persistentvolumeclaims", _key(pid, ns, c))
            if pvc is None:
                return claims, pinned, c
            claims.append(c)
            pinned = pinned or (pvc["metadata"].get("annotations") or {}).get(SELECTED_NODE)
        return claims, pinned, None

    def _unschedulable(self, pod: dict, key: str, msg: str) -> None:
        c = _cond(pod, "PodScheduled")
        if not c or c["status"] != "False" or c.get("message") != msg:
            self.store.patch("pods", key, lambda o: _set_cond(o, "PodScheduled", "False", "Unschedulable", msg))

    def _bind(self, pid: str, pod: dict, key: str, nn: str, annotations: dict | None = None) -> None:
        def bind(o, nn=nn):
            o["spec"]["nodeName"] = nn
            if annotations:
                o["metadata"].setdefault("annotations", {}).update(annotations)
            _set_cond(o, "PodScheduled", "True", "Scheduled", f"assigned to {nn}")

        self.store.patch("pods", key, bind)
        self._event(pid, pod["metadata"]["namespace"], {"kind": "Pod", "name": pod["metadata"]["name"]},
                    "Scheduled", f"Successfully assigned {pod['metadata']['name']} to {nn}")

    def _schedule_host_scoped(self, pid: str, pod: dict, key: str, need: int, sel, nodes: list[dict],
                              used: dict, count: dict) -> None:
        hosts: dict[str, list[dict]] = {}
        for n in nodes:
            nn = n["metadata"]["name"]
            alloc = int(n["status"]["allocatable"].get(GPU, 0))
            # whole idle validated GPU nodes only: the leader's process opens every device of each
            if (alloc > 0 and used.get(nn, 0) == 0 and node_validated(n)
                    and labels_match(sel, n["metadata"].get("labels"))):
                hosts.setdefault((n["metadata"].get("labels") or {}).get(HOST_LABEL, f"node:{nn}"), []).append(n)
        for host in sorted(hosts):
            members = sorted(hosts[host], key=lambda n: (-int(n["status"]["allocatable"].get(GPU, 0)), n["metadata"]["name"]))
            chosen, total = [], 0
            for n in members:
                g = int(n["status"]["allocatable"].get(GPU, 0))
                if total + g <= need:
                    chosen.append(n)
                    total += g
                if total == need:
                    break
            if total != need:
                continue
            leader = chosen[0]["metadata"]["name"]
            claims = {n["metadata"]["name"]: int(n["status"]["allocatable"].get(GPU, 0)) for n in chosen}
            devices = [{"node": n["metadata"]["name"], "id": d["id"], "ordinal": d.get("ordinal"),
                        "renderMinor": d.get("renderMinor", -1)}
                       for n in chosen[1:] for d in (n.get("status", {}).get("devices") or [])
                       if d.get("health") == "Healthy"]
            for cn, g in claims.items():
                used[cn] = used.get(cn, 0) + g
                count[cn] = count.get(cn, 0) + 1
            self._bind(pid, pod, key, leader, {HOST_CLAIMS: json.dumps(claims, sort_keys=True),
                                               HOST_DEVICES: json.dumps(devices, sort_keys=True),
                                               HOST_LABEL: host})
            return
        self._unschedulable(pod, key, f"no host has idle GPU nodes adding up to {need} {GPU} "
                                      f"({GPU_SCOPE}: host)")
