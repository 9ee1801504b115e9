"""Workload controllers beyond DaemonSets/Jobs/Deployments (controllers.py): StatefulSets,
ReplicaSets and CronJobs. A mixin of server.ControlPlane, run by reconcile().

* **StatefulSet** -- pods ``<name>-0 .. <name>-(n-1)`` with stable names and DNS
  (``<pod>.<serviceName>.<ns>.svc.cluster.local`` through a headless Service), hostname and
  subdomain set, labels ``statefulset.kubernetes.io/pod-name`` and ``apps.kubernetes.io/pod-index``.
  ``OrderedReady`` (default) creates ordinal i only once 0..i-1 run and removes from the highest
  ordinal one at a time; ``Parallel`` does both at once. ``RollingUpdate`` (default) replaces pods
  whose ``controller-revision-hash`` is stale from the highest ordinal down, one at a time, each
  after the others run (``partition`` keeps ordinals below it); ``OnDelete`` replaces only pods
  the user deletes. A stable name is what a multi-node GPU job keys its ranks on (rank = ordinal,
  ``MASTER_ADDR`` = ``<name>-0.<service>``).
  ``volumeClaimTemplates`` give each ordinal its own claim ``<template>-<name>-<ordinal>``,
  which outlives the pod (and the StatefulSet), as in Kubernetes.
* **ReplicaSet** -- ``replicas`` pods from the template (no rollout: that is the Deployment's).
* **CronJob** -- a Job from ``jobTemplate`` at each scheduled time (cron.py), named
  ``<name>-<scheduled minute>``; ``concurrencyPolicy`` Allow/Forbid/Replace, ``suspend``,
  ``startingDeadlineSeconds``, ``successfulJobsHistoryLimit`` (3) / ``failedJobsHistoryLimit`` (1),
  status ``active``/``lastScheduleTime``/``lastSuccessfulTime``. The control plane's clock loop
  (server.cron_loop) runs it every second.

The reference's Kubernetes (1.5, through Rancher) had these controllers in kube-controller-manager
(SURVEY.md §2.4 P3); there is no code of the reference behind this module.
"""
from __future__ import annotations

import copy
import time

from .objects import TERMINAL, _key, template_hash

STS_POD_NAME = "statefulset.kubernetes.io/pod-name"
POD_INDEX = "apps.kubernetes.io/pod-index"
REVISION = "controller-revision-hash"
SCHEDULED_AT = "batch.kubernetes.io/cronjob-scheduled-timestamp"


def _ts(iso: str | None):
    from datetime import datetime, timezone  # (off the control plane's start-up path)

    if not iso:
        return None
    try:
        return datetime.strptime(iso, "%Y-%m-%dT%H:%M:%SZ").replace(tzinfo=timezone.utc)
    except ValueError:
        return None


def _iso(t) -> str:
    from datetime import timezone

    return t.astimezone(timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")


def job_finished(job: dict) -> str | None:
    for c in (job.get("status") or {}).get("conditions") or []:
        if c.get("type") in ("Complete", "Failed") and c.get("status") == "True":
            return c["type"]
    return None


class Workloads:
    # ---- StatefulSets ---------------------------------------------------------------------
    def _ctl_statefulsets(self, pid: str) -> None:
        for s in self.store.list("statefulsets", lambda o: self._in(pid, o)):
            ns, name = s["metadata"]["namespace"], s["metadata"]["name"]
            spec = s["spec"]
            want = int(spec.get("replicas", 1))
            parallel = spec.get("podManagementPolicy") == "Parallel"
            upd = spec.get("updateStrategy") or {}
            rolling = upd.get("type", "RollingUpdate") == "RollingUpdate"
            partition = int((upd.get("rollingUpdate") or {}).get("partition", 0))
            h = template_hash(spec["template"])
            match = (spec.get("selector") or {}).get("matchLabels") or {}
            pods: dict[int, dict] = {}
            for o in self._owned(pid, s):
                try:
                    pods[int(o["metadata"].get("labels", {}).get(POD_INDEX, -1))] = o
                except ValueError:
                    continue

            def running(o):
                return o.get("status", {}).get("phase") == "Running" and not o["metadata"].get("deletionTimestamp")

            # a pod of a StatefulSet that ended (restartPolicy is Always, so only a failure) is
            # replaced under the same name
            for i, o in list(pods.items()):
                if o.get("status", {}).get("phase") in TERMINAL:
                    self._delete_pod(pid, ns, o["metadata"]["name"])
                    del pods[i]
            # scale up, in order unless Parallel
            for i in range(want):
                if i in pods:
                    continue
                if not parallel and not all(running(pods[j]) for j in range(i) if j in pods):
                    break
                tmpl = copy.deepcopy(spec["template"])
                tspec = tmpl.setdefault("spec", {})
                tspec["hostname"] = f"{name}-{i}"
                if spec.get("serviceName"):
                    tspec["subdomain"] = spec["serviceName"]
                # volumeClaimTemplates: one claim per ordinal, kept when the pod goes, so the
                # ordinal's replacement mounts the same data
                for vct in spec.get("volumeClaimTemplates") or []:
                    vname = (vct.get("metadata") or {}).get("name", "data")
                    claim = f"{vname}-{name}-{i}"
                    if self.store.get("persistentvolumeclaims", _key(pid, ns, claim)) is None:
                        self.create(pid, "persistentvolumeclaims", ns, {
                            "apiVersion": "v1", "kind": "PersistentVolumeClaim",
                            "metadata": {"name": claim, "labels": dict(match)}, "spec": copy.deepcopy(vct.get("spec") or {})})
                    vols = [v for v in tspec.get("volumes") or [] if v.get("name") != vname]
                    tspec["volumes"] = vols + [{"name": vname, "persistentVolumeClaim": {"claimName": claim}}]
                # (no ControllerRevision history here: a pod is always created from the current
                # template, below a rolling-update partition too)
                pods[i] = self._new_pod(pid, ns, f"{name}-{i}", s, "StatefulSet", tmpl,
                                        labels={**match, STS_POD_NAME: f"{name}-{i}", POD_INDEX: str(i), REVISION: h})
                if not parallel:
                    break
            # scale down from the highest ordinal
            extra = sorted((i for i in pods if i >= want), reverse=True)
            for i in extra[: len(extra) if parallel else 1]:
                if parallel or all(running(pods[j]) for j in pods if j < want):
                    self._delete_pod(pid, ns, pods.pop(i)["metadata"]["name"])
            # rolling update: one stale pod at a time, highest ordinal first, once all others run
            if rolling and len(pods) == want and all(running(o) for o in pods.values()):
                stale = [i for i, o in pods.items() if i >= partition and o["metadata"]["labels"].get(REVISION) != h]
                if stale:
                    i = max(stale)
                    self._delete_pod(pid, ns, pods.pop(i)["metadata"]["name"])
                    self._again = True  # the next pass re-creates it from the new template
            ready = sum(1 for o in pods.values() if running(o))
            updated = sum(1 for o in pods.values() if o["metadata"]["labels"].get(REVISION) == h)
            cur_rev = (s.get("status") or {}).get("currentRevision") or h
            if updated == want and ready == want:
                cur_rev = h
            status = {"observedGeneration": int(s["metadata"].get("generation", 1)), "replicas": len(pods),
                      "readyReplicas": ready, "availableReplicas": ready, "updatedReplicas": updated,
                      "currentReplicas": sum(1 for o in pods.values() if o["metadata"]["labels"].get(REVISION) == cur_rev),
                      "currentRevision": cur_rev, "updateRevision": h}
            if s.get("status") != status:
                self.store.patch("statefulsets", _key(pid, ns, name), lambda o, st=status: o.__setitem__("status", st))

    # ---- ReplicaSets ----------------------------------------------------------------------
    def _ctl_replicasets(self, pid: str) -> None:
        for rs in self.store.list("replicasets", lambda o: self._in(pid, o) and not any(
                r.get("kind") == "Deployment" for r in o["metadata"].get("ownerReferences", []))):
            # (a Deployment's ReplicaSets are its revision history: controllers.py runs those pods)
            ns, name = rs["metadata"]["namespace"], rs["metadata"]["name"]
            spec = rs["spec"]
            want = int(spec.get("replicas", 1))
            match = (spec.get("selector") or {}).get("matchLabels") or {}
            live = [o for o in self._owned(pid, rs) if o.get("status", {}).get("phase") not in TERMINAL
                    and not o["metadata"].get("deletionTimestamp")]
            for _ in range(max(0, want - len(live))):
                self._seq += 1
                live.append(self._new_pod(pid, ns, f"{name}-{self._seq:05x}", rs, "ReplicaSet", spec["template"],
                                          labels=dict(match)))
            # scale down: pods not yet running go first, then the youngest
            order = sorted(live, key=lambda o: (o.get("status", {}).get("phase") == "Running", o["metadata"]["name"]))
            for o in order[: max(0, len(live) - want)]:
                self._delete_pod(pid, ns, o["metadata"]["name"])
                live.remove(o)
            ready = sum(1 for o in live if o.get("status", {}).get("phase") == "Running")
            status = {"observedGeneration": int(rs["metadata"].get("generation", 1)), "replicas": len(live),
                      "readyReplicas": ready, "availableReplicas": ready, "fullyLabeledReplicas": len(live)}
            if rs.get("status") != status:
                self.store.patch("replicasets", _key(pid, ns, name), lambda o, st=status: o.__setitem__("status", st))

    # ---- CronJobs -------------------------------------------------------------------------
    def _delete_job(self, pid: str, ns: str, name: str) -> None:
        job = self.store.delete("jobs", _key(pid, ns, name))
        if job is None:
            return
        for pod in self._owned(pid, job):
            self._delete_pod(pid, ns, pod["metadata"]["name"])

    def _ctl_cronjobs(self, pid: str, now=None) -> None:
        from datetime import datetime, timezone

        from . import cron

        now = now or datetime.now(timezone.utc)
        for cj in self.store.list("cronjobs", lambda o: self._in(pid, o)):
            ns, name = cj["metadata"]["namespace"], cj["metadata"]["name"]
            spec, st = cj["spec"], dict(cj.get("status") or {})
            uid = cj["metadata"]["uid"]
            jobs = self.store.list("jobs", lambda o, u=uid: self._in(pid, o) and o["metadata"].get("namespace") == ns and any(
                r.get("uid") == u for r in o["metadata"].get("ownerReferences", [])))
            active = [j for j in jobs if not job_finished(j)]
            done = sorted((j for j in jobs if job_finished(j)),
                          key=lambda j: j["metadata"].get("annotations", {}).get(SCHEDULED_AT, ""))
            for j in done:
                if job_finished(j) == "Complete":
                    t = (j.get("status") or {}).get("completionTime")
                    if t and (not st.get("lastSuccessfulTime") or t > st["lastSuccessfulTime"]):
                        st["lastSuccessfulTime"] = t
            for kind, limit in (("Complete", int(spec.get("successfulJobsHistoryLimit", 3))),
                                ("Failed", int(spec.get("failedJobsHistoryLimit", 1)))):
                mine = [j for j in done if job_finished(j) == kind]
                for j in mine[: max(0, len(mine) - limit)]:
                    self._delete_job(pid, ns, j["metadata"]["name"])
            if not spec.get("suspend"):
                try:
                    sched = cron.parse(spec.get("schedule", ""), spec.get("timeZone"))
                except cron.CronError:
                    sched = None
                earliest = _ts(st.get("lastScheduleTime")) or _ts(cj["metadata"].get("creationTimestamp")) or now
                t, _missed = cron.most_recent(sched, earliest, now) if sched else (None, 0)
                deadline = spec.get("startingDeadlineSeconds")
                if t is not None and deadline is not None and (now - t).total_seconds() > float(deadline):
                    st["lastScheduleTime"] = _iso(t)  # missed its window: skipped, as Kubernetes does
                    t = None
                policy = spec.get("concurrencyPolicy", "Allow")
                if t is not None and not (policy == "Forbid" and active):
                    if policy == "Replace":
                        for j in active:
                            self._delete_job(pid, ns, j["metadata"]["name"])
                        active = []
                    jname = f"{name}-{int(t.timestamp()) // 60}" if not sched.every else f"{name}-{int(t.timestamp())}"
                    tmpl = copy.deepcopy(spec.get("jobTemplate") or {})
                    md = tmpl.get("metadata") or {}
                    body = {"apiVersion": "batch/v1", "kind": "Job",
                            "metadata": {"name": jname, "labels": dict(md.get("labels") or {}),
                                         "annotations": {**(md.get("annotations") or {}), SCHEDULED_AT: _iso(t)},
                                         "ownerReferences": [{"apiVersion": "batch/v1", "kind": "CronJob", "name": name,
                                                              "uid": uid, "controller": True}]},
                            "spec": tmpl.get("spec") or {}}
                    if self.store.get("jobs", _key(pid, ns, jname)) is None:
                        try:
                            active.append(self.create(pid, "jobs", ns, body))
                            self._event(pid, ns, {"kind": "CronJob", "name": name}, "SuccessfulCreate", f"Created job {jname}")
                        except Exception as e:  # noqa: BLE001 - a bad template is reported, not fatal
                            self._event(pid, ns, {"kind": "CronJob", "name": name}, "FailedCreate", str(e)[:300], "Warning")
                    st["lastScheduleTime"] = _iso(t)
            st["active"] = [{"kind": "Job", "namespace": ns, "name": j["metadata"]["name"], "uid": j["metadata"]["uid"],
                             "apiVersion": "batch/v1"} for j in active]
            if not st["active"]:
                del st["active"]
            if st != (cj.get("status") or {}):
                self.store.patch("cronjobs", _key(pid, ns, name), lambda o, s2=st: o.__setitem__("status", s2))

    async def cron_loop(self) -> None:
        """The controllers that run on the clock rather than on changes, every second: CronJobs,
        and Jobs with an ``activeDeadlineSeconds`` or ``ttlSecondsAfterFinished``."""
        import asyncio

        while True:
            await asyncio.sleep(1.0 - (time.time() % 1.0) + 0.01)
            if any("activeDeadlineSeconds" in j["spec"] or "ttlSecondsAfterFinished" in j["spec"]
                   for j in self.store.list("jobs")):
                self.reconcile()
            if not self.store.keys("cronjobs"):
                continue
            for p in self.store.list("projects"):
                self._ctl_cronjobs(p["id"])
            self.reconcile()

