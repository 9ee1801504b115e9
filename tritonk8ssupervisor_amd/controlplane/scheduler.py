"""The pod scheduler of the control plane: binds pending pods to Ready nodes with room, counting
the extended resource amd.com/gpu (validated nodes only), the way the AMD k8s-device-plugin
exposes it. A mixin of server.ControlPlane.
"""
from __future__ import annotations

from .objects import GPU, TERMINAL, _key, _cond, _set_cond, node_ready, node_validated, pod_gpus, labels_match


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

