"""The resource metrics API (``metrics.k8s.io/v1beta1``: what metrics-server serves, and what
``kubectl top`` and the HorizontalPodAutoscaler read) and the HPA controller
(``autoscaling/v2`` HorizontalPodAutoscaler). A mixin of server.ControlPlane.

Node agents sample their node's and pods' CPU and memory (agent/usage.py) and send them with
their heartbeat; the latest sample of each node is kept in memory (``self.metrics``), not in
the store: metrics are not objects and are not persisted, as with metrics-server.

HPA: every ``HPA_PERIOD`` seconds (15, the controller-manager's default) each autoscaler reads
its target's pods' usage and requests, and scales the target's ``replicas`` to
``ceil(current * utilization / target)`` -- for ``Resource`` metrics ``cpu``/``memory`` with
``Utilization`` (percent of requests) or ``AverageValue`` targets, and ``amd.com/gpu`` with a
``Utilization`` target: the average GFX busy percent of the pods' GPUs (AMD SMI, sampled by the
node agents) -- within
[minReplicas, maxReplicas], ignoring changes inside a 10 % tolerance, and keeping the highest
recommendation of the scale-down stabilization window (``behavior.scaleDown.
stabilizationWindowSeconds``, default 300), and moving no further than ``behavior``'s policies
allow within each policy's ``periodSeconds`` (the controller keeps its own scale events). Pods that are not Running or have no sample yet
are left out, as Kubernetes does for unready pods.
"""
from __future__ import annotations

import math
import time

from .httpserver import HttpError, Request
from .objects import _key, _set_cond, labels_match

METRICS_GV = "metrics.k8s.io/v1beta1"
HPA_PERIOD = 15.0
TOLERANCE = 0.1
_TARGET_KIND = {"Deployment": "deployments", "StatefulSet": "statefulsets", "ReplicaSet": "replicasets"}


def resource_list() -> dict:
    return {"kind": "APIResourceList", "apiVersion": "v1", "groupVersion": METRICS_GV, "resources": [
        {"name": "nodes", "singularName": "", "namespaced": False, "kind": "NodeMetrics", "verbs": ["get", "list"]},
        {"name": "pods", "singularName": "", "namespaced": True, "kind": "PodMetrics", "verbs": ["get", "list"]}]}


def _rate_limit(behavior: dict, current: int, desired: int, events=(), now: float = 0.0) -> int:
    """The HPA's scaling policies: how far the target may move within each policy's window
    (``behavior.scaleUp|scaleDown``: ``policies`` of ``Pods``/``Percent`` per ``periodSeconds``,
    ``selectPolicy`` Max|Min|Disabled). ``events`` are this autoscaler's past changes as
    ``(time, replica delta)``: a policy's budget is counted from the replica count at
    the start of its window, so two quick steps cannot add up to more than one policy allows.
    Defaults as Kubernetes': up by max(100 %, 4 pods) per 15 s, down by up to 100 % per 15 s."""
    up = desired > current
    rules = behavior.get("scaleUp" if up else "scaleDown") or {}
    if rules.get("selectPolicy") == "Disabled":
        return current
    pols = rules.get("policies") or ([{"type": "Percent", "value": 100, "periodSeconds": 15},
                                      {"type": "Pods", "value": 4, "periodSeconds": 15}] if up
                                     else [{"type": "Percent", "value": 100, "periodSeconds": 15}])
    limits = []
    for p in pols:
        v = int(p.get("value", 0))
        period = float(p.get("periodSeconds", 15))
        moved = sum(d for t, d in events if now - t < period and (d > 0) == up)
        start = current - moved  # the replica count when this policy's window opened
        step = v if p.get("type") == "Pods" else math.ceil(start * v / 100.0)
        limits.append(start + step if up else max(0, start - step))
    if not limits:
        return desired
    pick = (max if rules.get("selectPolicy", "Max") == "Max" else min) if up else \
        (min if rules.get("selectPolicy", "Max") == "Max" else max)
    bound = pick(limits)
    # a window already spent holds the target where it is, never moves it back
    return max(current, min(desired, bound)) if up else min(current, max(desired, bound))


class MetricsAPI:
    # ---- ingest ---------------------------------------------------------------------------
    def _ingest_metrics(self, pid: str, node: str, m: dict) -> None:
        if not isinstance(m, dict):
            return
        if not hasattr(self, "metrics"):
            self.metrics = {}
        self.metrics[(pid, node)] = {**m, "_received": time.monotonic()}

    def _node_samples(self, pid: str) -> dict[str, dict]:
        return {n: m for (p, n), m in getattr(self, "metrics", {}).items() if p == pid}

    def _pod_samples(self, pid: str) -> dict[str, tuple[str, list[dict]]]:
        """pod key ns/name -> (timestamp, containers)."""
        out = {}
        for m in self._node_samples(pid).values():
            for key, cs in (m.get("pods") or {}).items():
                out[key] = (m.get("timestamp", ""), cs)
        return out

    # ---- metrics.k8s.io -------------------------------------------------------------------
    async def h_metrics_resources(self, req: Request, pid: str | None = None):
        return resource_list()

    async def h_node_metrics(self, req: Request, name: str | None = None, pid: str | None = None):
        from ..utils import quantity

        p = self._pid(pid, req)
        items = []
        for node, m in sorted(self._node_samples(p).items()):
            if name and node != name:
                continue
            n = m.get("node") or {}
            items.append({"kind": "NodeMetrics", "apiVersion": METRICS_GV,
                          "metadata": {"name": node, "labels": (self.store.get("nodes", _key(p, node)) or {}).get(
                              "metadata", {}).get("labels", {})},
                          "timestamp": m.get("timestamp", ""), "window": m.get("window", "10s"),
                          "usage": {"cpu": quantity.cpu(n.get("cpu_cores", 0)),
                                    "memory": quantity.memory(n.get("memory_bytes", 0))}})
        if name:
            if not items:
                raise HttpError(404, f'nodemetrics.metrics.k8s.io "{name}" not found')
            return items[0]
        return {"kind": "NodeMetricsList", "apiVersion": METRICS_GV, "metadata": {}, "items": items}

    async def h_pod_metrics(self, req: Request, ns: str | None = None, name: str | None = None,
                            pid: str | None = None):
        from ..utils import quantity

        p = self._pid(pid, req)
        sel = req.q("labelSelector")
        from .objects import _parse_selector

        want = _parse_selector(sel)
        items = []
        for key, (ts, cs) in sorted(self._pod_samples(p).items()):
            pns, pname = key.split("/", 1)
            if (ns and pns != ns) or (name and pname != name):
                continue
            pod = self.store.get("pods", _key(p, pns, pname))
            if pod is None or not labels_match(want, pod["metadata"].get("labels")):
                continue
            items.append({"kind": "PodMetrics", "apiVersion": METRICS_GV,
                          "metadata": {"name": pname, "namespace": pns, "labels": pod["metadata"].get("labels", {})},
                          "timestamp": ts, "window": "10s",
                          "containers": [{"name": c["name"], "usage": {
                              "cpu": quantity.cpu(c.get("cpu_cores", 0)), "memory": quantity.memory(c.get("memory_bytes", 0)),
                              **({"amd.com/gpu-utilization": f"{c['gpu_pct']:.0f}"} if c.get("gpu_pct") is not None else {})}}
                                         for c in cs]})
        if name:
            if not items:
                raise HttpError(404, f'podmetrics.metrics.k8s.io "{ns}/{name}" not found')
            return items[0]
        return {"kind": "PodMetricsList", "apiVersion": METRICS_GV, "metadata": {}, "items": items}

    # ---- HorizontalPodAutoscaler ------------------------------------------------------------
    def _ctl_hpas(self, pid: str, now: float | None = None) -> None:
        from ..utils import quantity

        now = time.time() if now is None else now
        samples = self._pod_samples(pid)
        if not hasattr(self, "_hpa_recs"):
            self._hpa_recs, self._hpa_events = {}, {}
        for hpa in self.store.list("horizontalpodautoscalers", lambda o: self._in(pid, o)):
            ns, name = hpa["metadata"]["namespace"], hpa["metadata"]["name"]
            spec = hpa["spec"]
            ref = spec.get("scaleTargetRef") or {}
            plural = _TARGET_KIND.get(ref.get("kind", ""))
            target = self.store.get(plural, _key(pid, ns, ref.get("name", ""))) if plural else None
            st = dict(hpa.get("status") or {})
            holder = {"status": {"conditions": list(st.get("conditions") or [])}}  # what _set_cond edits
            conds = holder["status"]
            if target is None:
                _set_cond(holder, "AbleToScale", "False", "FailedGetScale",
                          f"the HPA controller was unable to get the target's current scale: {ref.get('kind')}/{ref.get('name')}")
                self._hpa_status(pid, ns, name, hpa, {**st, "conditions": conds["conditions"]})
                continue
            _set_cond(holder, "AbleToScale", "True", "SucceededGetScale", "the HPA controller was able to get the target's current scale")
            current = int(target["spec"].get("replicas", 1))
            sel = (target["spec"].get("selector") or {}).get("matchLabels") or {}
            pods = [o for o in self.store.list("pods", lambda o: self._in(pid, o) and o["metadata"].get("namespace") == ns
                                               and labels_match(sel, o["metadata"].get("labels")))
                    if o.get("status", {}).get("phase") == "Running"]
            desired, current_metrics, why = None, [], ""
            for metric in spec.get("metrics") or [{"type": "Resource", "resource": {
                    "name": "cpu", "target": {"type": "Utilization", "averageUtilization": 80}}}]:
                if metric.get("type") != "Resource":
                    why = f"metric type {metric.get('type')} is not supported (Resource cpu/memory only)"
                    continue
                res = metric["resource"].get("name")
                tgt = metric["resource"].get("target") or {}
                if res == "amd.com/gpu":  # GPU busy %, averaged over the pods that report it
                    vals = [c["gpu_pct"] for o in pods for c in samples.get(f"{ns}/{o['metadata']['name']}", ("", []))[1]
                            if c.get("gpu_pct") is not None]
                    if not vals:
                        why = "no GPU activity samples for the target's pods yet (AMD SMI)"
                        continue
                    util = sum(vals) / len(vals)
                    ratio = util / float(tgt.get("averageUtilization", 80))
                    current_metrics.append({"type": "Resource", "resource": {"name": res, "current": {
                        "averageUtilization": int(round(util))}}})
                    want = current if abs(ratio - 1.0) <= TOLERANCE else math.ceil(len(vals) * ratio)
                    desired = want if desired is None else max(desired, want)
                    continue
                usage, requests, n = 0.0, 0.0, 0
                for o in pods:
                    key = f"{ns}/{o['metadata']['name']}"
                    if key not in samples:
                        continue
                    n += 1
                    usage += sum(c.get("cpu_cores" if res == "cpu" else "memory_bytes", 0) for c in samples[key][1])
                    for c in o["spec"].get("containers") or []:
                        r = ((c.get("resources") or {}).get("requests") or {}).get(res)
                        if r is not None:
                            requests += quantity.parse(r)
                if not n:
                    why = "no metrics for the target's pods yet"
                    continue
                if tgt.get("type", "Utilization") == "Utilization":
                    if not requests:
                        why = f"missing request for {res} on the target's pods"
                        continue
                    util = 100.0 * usage / requests
                    ratio = util / float(tgt.get("averageUtilization", 80))
                    current_metrics.append({"type": "Resource", "resource": {"name": res, "current": {
                        "averageUtilization": int(round(util)),
                        "averageValue": quantity.cpu(usage / n) if res == "cpu" else quantity.memory(usage / n)}}})
                else:
                    ratio = (usage / n) / quantity.parse(tgt.get("averageValue", "1"))
                    current_metrics.append({"type": "Resource", "resource": {"name": res, "current": {
                        "averageValue": quantity.cpu(usage / n) if res == "cpu" else quantity.memory(usage / n)}}})
                want = current if abs(ratio - 1.0) <= TOLERANCE else math.ceil(n * ratio)
                desired = want if desired is None else max(desired, want)
            lo, hi = int(spec.get("minReplicas", 1)), int(spec.get("maxReplicas", current))
            if desired is None:
                _set_cond(holder, "ScalingActive", "False", "FailedGetResourceMetric", why)
                self._hpa_status(pid, ns, name, hpa, {**st, "currentReplicas": current, "desiredReplicas": current,
                                                      "conditions": conds["conditions"]})
                continue
            _set_cond(holder, "ScalingActive", "True", "ValidMetricFound", "the HPA was able to compute the replica count")
            desired = min(hi, max(lo, desired))
            # stabilization: scaling down takes the highest recommendation of its window (300 s by
            # default), scaling up the lowest of its own (0 s by default)
            beh = spec.get("behavior") or {}
            down_w = float((beh.get("scaleDown") or {}).get("stabilizationWindowSeconds", 300))
            up_w = float((beh.get("scaleUp") or {}).get("stabilizationWindowSeconds", 0))
            recs = [(t, r) for t, r in self._hpa_recs.get((pid, ns, name), []) if now - t <= max(down_w, up_w)]
            recs.append((now, desired))
            self._hpa_recs[(pid, ns, name)] = recs
            if desired < current:
                desired = min(current, max(r for t, r in recs if now - t <= down_w))
            elif desired > current:
                desired = max(current, min(r for t, r in recs if now - t <= up_w))
            events = [(t, d) for t, d in self._hpa_events.get((pid, ns, name), []) if now - t < 1800]
            desired = min(hi, max(lo, _rate_limit(beh, current, desired, events, now)))
            status = {**st, "currentReplicas": current, "desiredReplicas": desired, "currentMetrics": current_metrics,
                      "conditions": conds["conditions"]}
            if desired != current:
                self._hpa_events[(pid, ns, name)] = events + [(now, desired - current)]
                self.replace(pid, plural, ns, ref["name"], {"spec": {"replicas": desired}}, merge=True,
                             manager="horizontal-pod-autoscaler", subresource="scale")
                status["lastScaleTime"] = time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime(now))
                self._event(pid, ns, {"kind": "HorizontalPodAutoscaler", "name": name}, "SuccessfulRescale",
                            f"New size: {desired}; reason: {current_metrics[0]['resource']['name'] if current_metrics else ''} "
                            f"resource utilization above target" if desired > current else
                            f"New size: {desired}; reason: All metrics below target")
            self._hpa_status(pid, ns, name, hpa, status)

    def _hpa_status(self, pid: str, ns: str, name: str, hpa: dict, status: dict) -> None:
        status["observedGeneration"] = int(hpa["metadata"].get("generation", 1))
        if status != hpa.get("status"):
            self.store.patch("horizontalpodautoscalers", _key(pid, ns, name), lambda o, s=status: o.__setitem__("status", s))

    async def hpa_loop(self) -> None:
        import asyncio

        while True:
            await asyncio.sleep(float(getattr(self, "hpa_period", HPA_PERIOD)))
            if not self.store.keys("horizontalpodautoscalers"):
                continue
            for p in self.store.list("projects"):
                self._ctl_hpas(p["id"])
