"""Voluntary disruptions: PodDisruptionBudgets (policy/v1) and the Eviction API
(``POST .../pods/<name>/eviction``). A mixin of server.ControlPlane.

A budget selects pods by label in its namespace and says how many must stay healthy
(``minAvailable``) or may be down (``maxUnavailable``), as a count or a percentage of the pods it
expects. Its status (``currentHealthy``, ``desiredHealthy``, ``expectedPods``,
``disruptionsAllowed``, condition ``DisruptionAllowed``) is kept by ``_ctl_pdbs``. An eviction is
a delete that asks first: while a budget covering the pod allows no disruption the API answers
429 TooManyRequests ("would violate the pod's disruption budget") and the pod stays; otherwise
the pod is deleted and the budget's allowance drops at once (``status.disruptedPods`` holds the
pod until it is gone, so two evictions cannot both spend the last allowance). ``kubectl drain``
evicts through this API and retries a 429 until its timeout -- how a GPU node goes into
maintenance without taking a serving Deployment below its floor.

``expectedPods`` is what the budget's pods' controllers want (a Deployment/StatefulSet/ReplicaSet's
``replicas``, a Job's ``parallelism``), else the number of matching pods; a percentage
``minAvailable`` rounds up, a percentage ``maxUnavailable`` rounds up as well (Kubernetes'
rounding). "Healthy" means Running and not NotReady.
"""
from __future__ import annotations

import math

from .httpserver import HttpError, Request, Response
from .objects import TERMINAL, _key
from .store import now_iso

PDB = "poddisruptionbudgets"
_OWNER_KINDS = {"Deployment": "deployments", "StatefulSet": "statefulsets", "ReplicaSet": "replicasets", "Job": "jobs"}


def _amount(v, total: int) -> int:
    if isinstance(v, str) and v.endswith("%"):
        return math.ceil(total * float(v[:-1]) / 100.0)
    return int(v)


def _healthy(pod: dict) -> bool:
    st = pod.get("status") or {}
    return st.get("phase") == "Running" and not (pod.get("metadata") or {}).get("deletionTimestamp") and not any(
        c.get("type") == "Ready" and c.get("status") == "False" for c in st.get("conditions") or [])


class Disruption:
    def _pdb_pods(self, pid: str, pdb: dict) -> list[dict]:
        ns, sel = pdb["metadata"]["namespace"], (pdb.get("spec") or {}).get("selector")
        return [o for o in self.store.list("pods", lambda o: self._in(pid, o) and o["metadata"].get("namespace") == ns)
                if o.get("status", {}).get("phase") not in TERMINAL and _sel(sel, o["metadata"].get("labels"))]

    def _expected(self, pid: str, pods: list[dict]) -> int:
        """What the pods' controllers want, counted once per controller; uncontrolled pods count themselves."""
        total, seen = 0, set()
        for o in pods:
            ref = next((r for r in o["metadata"].get("ownerReferences") or [] if r.get("controller", True)), None)
            kind = _OWNER_KINDS.get((ref or {}).get("kind"))
            if kind is None:
                total += 1
                continue
            if ref["uid"] in seen:
                continue
            seen.add(ref["uid"])
            owner = self.store.get(kind, _key(pid, o["metadata"]["namespace"], ref["name"]))
            spec = (owner or {}).get("spec") or {}
            total += int(spec.get("parallelism", spec.get("completions", 1)) if kind == "jobs" else spec.get("replicas", 1))
        return total

    def _pdb_status(self, pid: str, pdb: dict) -> dict:
        spec = pdb.get("spec") or {}
        pods = self._pdb_pods(pid, pdb)
        expected = self._expected(pid, pods)
        names = {o["metadata"]["name"] for o in pods}
        # an eviction in flight still counts against the budget until its pod is gone
        disrupted = {n: t for n, t in ((pdb.get("status") or {}).get("disruptedPods") or {}).items() if n in names}
        healthy = sum(1 for o in pods if _healthy(o) and o["metadata"]["name"] not in disrupted)
        if "minAvailable" in spec:
            desired = _amount(spec["minAvailable"], expected)
        else:
            desired = max(0, expected - _amount(spec.get("maxUnavailable", 0), expected))
        allowed = max(0, healthy - desired)
        st = {"observedGeneration": int(pdb["metadata"].get("generation", 1)), "currentHealthy": healthy,
              "desiredHealthy": desired, "expectedPods": expected, "disruptionsAllowed": allowed}
        if disrupted:
            st["disruptedPods"] = disrupted
        old = next((c for c in (pdb.get("status") or {}).get("conditions") or [] if c.get("type") == "DisruptionAllowed"), None)
        want = ("True", "SufficientPods") if allowed > 0 else ("False", "InsufficientPods")
        if old and (old.get("status"), old.get("reason")) == want:
            st["conditions"] = [old]
        else:
            st["conditions"] = [{"type": "DisruptionAllowed", "status": want[0], "reason": want[1],
                                 "observedGeneration": st["observedGeneration"], "lastTransitionTime": now_iso(),
                                 "message": ""}]
        return st

    def _ctl_pdbs(self, pid: str) -> None:
        for pdb in self.store.list(PDB, lambda o: self._in(pid, o)):
            st = self._pdb_status(pid, pdb)
            if pdb.get("status") != st:
                self.store.patch(PDB, _key(pid, pdb["metadata"]["namespace"], pdb["metadata"]["name"]),
                                 lambda o, s=st: o.__setitem__("status", s))

    @staticmethod
    def _admit_pdb(name: str, body: dict) -> None:
        spec = body.get("spec") or {}
        if ("minAvailable" in spec) == ("maxUnavailable" in spec):
            raise HttpError(422, f'PodDisruptionBudget.policy "{name}" is invalid: spec: Invalid value: '
                                 "minAvailable and maxUnavailable cannot be both set (and one is required)")
        for f in ("minAvailable", "maxUnavailable"):
            v = spec.get(f)
            if v is None:
                continue
            ok = (isinstance(v, int) and v >= 0) or (isinstance(v, str) and v.endswith("%") and v[:-1].isdigit()
                                                    and 0 <= int(v[:-1]) <= 100)
            if not ok:
                raise HttpError(422, f'PodDisruptionBudget.policy "{name}" is invalid: spec.{f}: Invalid value: {v!r}: '
                                     "must be a non-negative integer or a percentage")
        body.setdefault("status", {})

    def evict(self, pid: str, ns: str, name: str, dry_run: bool = False) -> None:
        """Delete ``ns/name`` unless that would break a disruption budget (HttpError 429)."""
        pod = self.store.get("pods", _key(pid, ns, name))
        if pod is None:
            raise HttpError(404, f'pods "{name}" not found')
        budgets = [b for b in self.store.list(PDB, lambda o: self._in(pid, o) and o["metadata"]["namespace"] == ns)
                   if _sel((b.get("spec") or {}).get("selector"), pod["metadata"].get("labels"))]
        if len(budgets) > 1:
            raise HttpError(500, "This pod has more than one PodDisruptionBudget, which the eviction subresource "
                                 "does not support.")
        # a pod that is not healthy anyway (Pending, NotReady) or already done may always go
        if budgets and pod.get("status", {}).get("phase") not in TERMINAL and _healthy(pod):
            b = budgets[0]
            st = self._pdb_status(pid, b)
            if st["disruptionsAllowed"] <= 0:
                raise HttpError(429, "Cannot evict pod as it would violate the pod's disruption budget.",
                                body={"kind": "Status", "apiVersion": "v1", "metadata": {}, "status": "Failure",
                                      "message": "Cannot evict pod as it would violate the pod's disruption budget.",
                                      "reason": "TooManyRequests", "code": 429,
                                      "details": {"causes": [{"reason": "DisruptionBudget", "message":
                                                              f"The disruption budget {b['metadata']['name']} needs "
                                                              f"{st['desiredHealthy']} healthy pods and has "
                                                              f"{st['currentHealthy']} currently"}]}})
            if dry_run:
                return
            self.store.patch(PDB, _key(pid, ns, b["metadata"]["name"]), lambda o: o.setdefault("status", {}).setdefault(
                "disruptedPods", {}).__setitem__(name, now_iso()))
        if dry_run:
            return
        self._delete_pod(pid, ns, name, disruption="EvictionByEvictionAPI")
        self._event(pid, ns, {"kind": "Pod", "name": name}, "Evicted", "Evicted through the eviction API", "Normal")
        self.reconcile()

    async def h_pod_eviction(self, req: Request, ns: str, name: str, pid: str | None = None):
        """``POST /api/v1/namespaces/<ns>/pods/<name>/eviction`` with a policy/v1 Eviction."""
        p = self._pid(pid, req)
        self._auth(req, self.project(p))
        body = req.json() or {}
        if body.get("kind") not in (None, "Eviction") or (body.get("metadata") or {}).get("name", name) != name:
            raise HttpError(400, "the body must be a policy/v1 Eviction of this pod")
        dry = self._dry_run(req) or bool((body.get("deleteOptions") or {}).get("dryRun"))
        self.evict(p, ns, name, dry_run=dry)
        return Response(201, {"kind": "Status", "apiVersion": "v1", "metadata": {}, "status": "Success", "code": 201})


def _sel(sel, labels) -> bool:
    from .placement import selector_matches  # (lazy: off the control plane's start-up imports)

    return selector_matches(sel, labels)
