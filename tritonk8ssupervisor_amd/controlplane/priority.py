"""Pod priority and preemption: PriorityClasses (scheduling.k8s.io/v1, cluster-scoped) and the
scheduler's preemption of lower-priority pods. A mixin of server.ControlPlane.

A pod's ``spec.priorityClassName`` resolves at admission -- for a client's pod and for a
controller's alike -- into ``spec.priority`` and ``spec.preemptionPolicy``; a pod without one gets
the class marked ``globalDefault`` or priority 0. An unknown class is refused (403), as Kubernetes'
Priority admission plugin does. ``system-cluster-critical`` (2000000000) and
``system-node-critical`` (2000001000) always exist; user classes stay at or below 1000000000 and
may not take the ``system-`` prefix.

The scheduler takes pending pods highest priority first. A GPU pod that fits nowhere and may
preempt (``preemptionPolicy`` not ``Never``) looks for the node where deleting the fewest,
lowest-priority pods frees enough ``amd.com/gpu`` -- only pods of strictly lower priority,
those a PodDisruptionBudget still allows to go before the others -- deletes them (event
``Preempted`` on each, ``status.nominatedNodeName`` on the preemptor) and binds it there: how a
production training job takes the MI355X GPUs of a best-effort sweep.
"""
from __future__ import annotations

from .httpserver import HttpError
from .objects import GPU, TERMINAL, _key, labels_match, node_validated, pod_gpus

PC = "priorityclasses"
BUILTIN = {"system-cluster-critical": 2000000000, "system-node-critical": 2000001000}
USER_MAX = 1000000000


def priority(pod: dict) -> int:
    return int(pod.get("spec", {}).get("priority") or 0)


class Priority:
    def _admit_priority_class(self, pid: str, name: str, body: dict) -> None:
        v = body.get("value")
        if not isinstance(v, int) or isinstance(v, bool):
            raise HttpError(422, f'PriorityClass.scheduling.k8s.io "{name}" is invalid: value: Required value')
        if name.startswith("system-") or v > USER_MAX:
            raise HttpError(422, f'PriorityClass.scheduling.k8s.io "{name}" is invalid: only system classes may use '
                                 f'the "system-" prefix or a value above {USER_MAX}')
        if body.get("preemptionPolicy", "PreemptLowerPriority") not in ("PreemptLowerPriority", "Never"):
            raise HttpError(422, f"preemptionPolicy: Unsupported value: {body['preemptionPolicy']!r}")
        if body.get("globalDefault"):
            other = next((c["metadata"]["name"] for c in self.store.list(PC, lambda o: self._in(pid, o))
                          if c.get("globalDefault") and c["metadata"]["name"] != name), None)
            if other:
                raise HttpError(422, f'PriorityClass.scheduling.k8s.io "{name}" is invalid: globalDefault: '
                                     f'Invalid value: PriorityClass "{other}" is already marked as default')

    def _resolve_priority(self, pid: str, spec: dict) -> None:
        """``priorityClassName`` -> ``priority`` + ``preemptionPolicy`` on a pod spec (in place)."""
        name = spec.get("priorityClassName")
        if name:
            if name in BUILTIN:
                value, policy = BUILTIN[name], "PreemptLowerPriority"
            else:
                pc = self.store.get(PC, _key(pid, "", name))
                if pc is None:
                    raise HttpError(403, f'pods is forbidden: no PriorityClass with name {name} was found')
                value, policy = int(pc["value"]), pc.get("preemptionPolicy", "PreemptLowerPriority")
        else:
            pc = next((c for c in self.store.list(PC, lambda o: self._in(pid, o)) if c.get("globalDefault")), None) \
                if self.store.keys(PC) else None
            if pc is None:
                spec.setdefault("priority", 0)
                return
            spec["priorityClassName"] = pc["metadata"]["name"]
            value, policy = int(pc["value"]), pc.get("preemptionPolicy", "PreemptLowerPriority")
        if spec.get("priority") not in (None, value):
            raise HttpError(403, "the integer value of priority must not be provided in pod spec; the priority "
                                 "admission controller computes it from the given PriorityClass name")
        spec["priority"], spec["preemptionPolicy"] = value, policy

    def _preempt(self, pid: str, pod: dict, key: str, need: int, sel, nodes: list[dict], used: dict) -> str | None:
        """Free ``need`` GPUs for ``pod`` by deleting lower-priority pods on one node; the node, or None."""
        prio = priority(pod)
        if need <= 0 or pod["spec"].get("preemptionPolicy") == "Never":
            return None
        live = [o for o in self.store.list("pods", lambda o: self._in(pid, o))
                if o["spec"].get("nodeName") and o.get("status", {}).get("phase") not in TERMINAL
                and not o["metadata"].get("deletionTimestamp")]
        protected = self._pdb_protected(pid) if self.store.keys("poddisruptionbudgets") else set()
        best = None
        for n in nodes:
            nn = n["metadata"]["name"]
            if not labels_match(sel, n["metadata"].get("labels")) or not node_validated(n):
                continue
            free = int(n["status"]["allocatable"].get(GPU, 0)) - used.get(nn, 0)
            cands = sorted((o for o in live if o["spec"]["nodeName"] == nn and priority(o) < prio and pod_gpus(o) > 0),
                           key=lambda o: (o["metadata"]["name"] in protected, priority(o),
                                          -int(o["metadata"].get("resourceVersion", 0) or 0)))
            victims = []
            for o in cands:
                if free >= need:
                    break
                victims.append(o)
                free += pod_gpus(o)
            if free < need:
                continue
            cost = (sum(o["metadata"]["name"] in protected for o in victims),
                    max((priority(o) for o in victims), default=-(1 << 62)), len(victims), nn)
            if best is None or cost < best[0]:
                best = (cost, nn, victims)
        if best is None:
            return None
        _cost, nn, victims = best
        ns, name = pod["metadata"]["namespace"], pod["metadata"]["name"]
        for o in victims:
            vns, vname = o["metadata"]["namespace"], o["metadata"]["name"]
            self._delete_pod(pid, vns, vname, disruption="PreemptionByScheduler")  # (its GPUs: the agent starts the preemptor once they are free)
            used[nn] = used.get(nn, 0) - pod_gpus(o)
            self._event(pid, vns, {"kind": "Pod", "name": vname}, "Preempted",
                        f"Preempted by pod {ns}/{name} (priority {priority(pod)}) on node {nn}", "Normal")
        self.store.patch("pods", key, lambda o: o.setdefault("status", {}).__setitem__("nominatedNodeName", nn))
        self._again = True  # the victims' controllers replace them in this reconcile
        return nn

    def _pdb_protected(self, pid: str) -> set[str]:
        """Pods a PodDisruptionBudget would not let go now (preempted last)."""
        out = set()
        for b in self.store.list("poddisruptionbudgets", lambda o: self._in(pid, o)):
            if (b.get("status") or {}).get("disruptionsAllowed", 0) <= 0:
                out |= {o["metadata"]["name"] for o in self._pdb_pods(pid, b)}
        return out
