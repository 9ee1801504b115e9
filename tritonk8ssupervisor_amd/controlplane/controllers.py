"""Controllers of the control plane: DaemonSets, the GPU validation gate, Indexed Jobs,
Deployments (rolling updates), run by reconcile() after every change. A mixin of
server.ControlPlane.
"""
from __future__ import annotations

import copy
import time

from .httpserver import HttpError
from .store import now_iso


def _failure_action(policy: dict | None, pod: dict) -> tuple[str, str]:
    """A Job's ``podFailurePolicy`` verdict on one failed pod: (FailJob|Ignore|Count, why). The
    first rule that matches decides -- ``onExitCodes`` (``containerName``, ``In``/``NotIn``) on the
    containers' terminated exit codes, ``onPodConditions`` on the pod's conditions; none: Count.
    How a training Job fails at once on a bad-config exit code but retries a node's hardware fault."""
    if not policy:
        return "Count", ""
    st = pod.get("status") or {}
    codes = [(c.get("name"), ((c.get("state") or {}).get("terminated") or {}).get("exitCode"))
             for c in st.get("containerStatuses") or []]
    codes = [(n, int(x)) for n, x in codes if x is not None]
    if not codes and st.get("exitCode") is not None:
        codes = [(None, int(st["exitCode"]))]
    conds = {(c.get("type"), c.get("status")) for c in st.get("conditions") or []}
    for i, rule in enumerate(policy.get("rules") or []):
        ec = rule.get("onExitCodes")
        if ec:
            vals = {int(v) for v in ec.get("values") or []}
            for name, code in codes:
                if ec.get("containerName") not in (None, name) or code == 0:
                    continue
                if (code in vals) == (ec.get("operator", "In") == "In"):
                    ns, pn = pod["metadata"].get("namespace", "default"), pod["metadata"]["name"]
                    return rule.get("action", "Count"), (f"Container {name or 'main'} for pod {ns}/{pn} failed with exit code "
                                                         f"{code} matching {rule.get('action')} rule at index {i}")
        for pc in rule.get("onPodConditions") or []:
            if (pc.get("type"), pc.get("status", "True")) in conds:
                return rule.get("action", "Count"), (f"Pod {pod['metadata']['name']} has condition {pc.get('type')} "
                                                     f"matching {rule.get('action')} rule at index {i}")
    return "Count", ""


def _conditions(obj: dict, want: list[tuple[str, str, str, str]]) -> list[dict]:
    """Status conditions (type, status, reason, message), keeping an old entry's times while its
    status and reason hold, so an unchanged object is not rewritten."""
    old = {c.get("type"): c for c in (obj.get("status") or {}).get("conditions") or []}
    out = []
    for ctype, status, reason, message in want:
        c = old.get(ctype)
        if c and (c.get("status"), c.get("reason"), c.get("message")) == (status, reason, message):
            out.append(c)
        else:
            t = now_iso()
            out.append({"type": ctype, "status": status, "reason": reason, "message": message,
                        "lastUpdateTime": t, "lastTransitionTime": c["lastTransitionTime"] if c and c.get("status") == status else t})
    return out


def _epoch(iso: str | None) -> float:
    """Seconds since the epoch of an RFC 3339 ``...Z`` timestamp (now if missing or malformed)."""
    import calendar

    try:
        return float(calendar.timegm(time.strptime(iso or "", "%Y-%m-%dT%H:%M:%SZ")))
    except ValueError:
        return time.time()

REVISION = "deployment.kubernetes.io/revision"
from .objects import (
    VALIDATION_LABEL, TERMINAL, _key, _cond, _set_cond, _set_ready, _xgmi_view, template_hash, labels_match, node_ready,
    strip_owned,
)


class Controllers:
    # ---- controllers ------------------------------------------------------------------
    def reconcile(self) -> None:
        """Run every controller once (cheap at this scale; called after each mutation)."""
        if getattr(self, "_reconciling", False):
            self._again = True
            return
        self._reconciling = True
        try:
            for _ in range(8):
                self._again = False
                for p in self.store.list("projects"):
                    pid = p["id"]
                    self._ctl_daemonsets(pid)
                    self._ctl_jobs(pid)
                    self._ctl_deployments(pid)
                    self._ctl_statefulsets(pid)
                    self._ctl_replicasets(pid)
                    self._ctl_endpoints(pid)
                    self._ctl_quotas(pid)
                    self._ctl_pdbs(pid)
                    self._ctl_validation(pid)
                    self._scheduler(pid)
                if not self._again:
                    break
        finally:
            self._reconciling = False

    def _new_pod(self, pid: str, ns: str, name: str, owner: dict, owner_kind: str, template: dict,
                 node: str | None = None, extra_env: dict | None = None, labels: dict | None = None,
                 annotations: dict | None = None) -> dict:
        spec = copy.deepcopy(template.get("spec", {}))
        if extra_env:
            for c in spec.get("containers", []):
                c.setdefault("env", []).extend({"name": k, "value": str(v)} for k, v in extra_env.items())
        if node:
            spec["nodeName"] = node
        md = copy.deepcopy(template.get("metadata", {}))
        if md.get("annotations"):  # (admission refuses them in templates; a restored old object may have them)
            md["annotations"] = strip_owned(md["annotations"])
        md.update(name=name, namespace=ns)
        md.setdefault("labels", {}).update(labels or {})
        md.setdefault("annotations", {}).update(annotations or {})
        md["ownerReferences"] = [{"kind": owner_kind, "name": owner["metadata"]["name"], "uid": owner["metadata"]["uid"]}]
        pod = {"kind": "Pod", "apiVersion": "v1", "metadata": md, "spec": spec, "_project": pid,
               "status": {"phase": "Pending", "conditions": []}}
        spec.setdefault("restartPolicy", "Always")
        try:
            self._resolve_priority(pid, spec)
            self._pod_security(pid, ns, name, pod)
            self._admit_limit_ranges(pid, ns, name, pod)
        except HttpError as e:  # as the ReplicaSet controller's FailedCreate: nothing is created
            self._event(pid, ns, {"kind": owner_kind, "name": owner["metadata"]["name"]}, "FailedCreate",
                        f'Error creating: pods "{name}" is forbidden: {e.message}', "Warning")
            return pod
        why = self._quota_block(pid, ns, name, pod)
        if why:  # as the ReplicaSet controller's 403: the pod waits (unscheduled) until the quota allows it
            from .objects import QUOTA_BLOCKED

            md.setdefault("annotations", {})[QUOTA_BLOCKED] = "true"
            _set_cond(pod, "PodScheduled", "False", "ExceededQuota", why)
            self._event(pid, ns, {"kind": owner_kind, "name": owner["metadata"]["name"]}, "FailedCreate",
                        f"Error creating: pods \"{name}\" is forbidden: {why}", "Warning")
        return self.store.put("pods", _key(pid, ns, name), pod)

    def _delete_pod(self, pid: str, ns: str, name: str, grace: float | None = None, force: bool = False,
                    disruption: str | None = None) -> dict | None:
        """Delete a pod gracefully, as the API server does: a pod running on a node whose agent is
        alive gets ``metadata.deletionTimestamp`` (now + grace, ``terminationGracePeriodSeconds``
        by default) and stays, Terminating, until that agent has stopped it (preStop hook, SIGTERM,
        SIGKILL at the deadline) and confirms with a forced delete; controllers stop counting it at
        once and the scheduler keeps counting its GPUs. Any other pod -- not started, finished, on
        a node no agent answers for -- or ``force``/``grace == 0`` goes at once. The lease loop
        force-deletes a Terminating pod whose agent never confirmed (``_pod_gc``). ``disruption``:
        the ``DisruptionTarget`` condition's reason (EvictionByEvictionAPI, PreemptionByScheduler,
        DeletionByTaintManager), what a Job's podFailurePolicy ``onPodConditions`` can match."""
        key = _key(pid, ns, name)
        pod = self.store.get("pods", key)
        if pod is None:
            return None
        nn = pod["spec"].get("nodeName")
        if grace is None:
            grace = float(pod["spec"].get("terminationGracePeriodSeconds", 30))
        graceful = (not force and grace > 0 and nn and pod.get("status", {}).get("phase") == "Running"
                    and _key(pid, nn) in getattr(self, "leases", {}) and node_ready(self.store.get("nodes", _key(pid, nn)) or {}))
        if not graceful:
            return self.store.delete("pods", key)
        if pod["metadata"].get("deletionTimestamp"):
            return pod  # already terminating (a second delete may only shorten it; not modelled)

        def mark(o):
            o["metadata"]["deletionTimestamp"] = time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime(time.time() + grace))
            o["metadata"]["deletionGracePeriodSeconds"] = int(grace)
            if disruption:
                _set_cond(o, "DisruptionTarget", "True", disruption, "the pod is being deleted for a disruption")
        self._again = True  # controllers replace it now
        return self.store.patch("pods", key, mark)

    def _owned(self, pid: str, owner: dict) -> list[dict]:
        uid = owner["metadata"]["uid"]
        return self.store.list("pods", lambda o: self._in(pid, o) and any(
            r.get("uid") == uid for r in o["metadata"].get("ownerReferences", [])))

    def _ctl_daemonsets(self, pid: str) -> None:
        nodes = self.store.list("nodes", lambda n: self._in(pid, n))
        for ds in self.store.list("daemonsets", lambda o: self._in(pid, o)):
            ns = ds["metadata"]["namespace"]
            tmpl = ds["spec"]["template"]
            sel = tmpl.get("spec", {}).get("nodeSelector")
            pods = {o["spec"].get("nodeName"): o for o in self._owned(pid, ds)}
            eligible = [n for n in nodes if labels_match(sel, n["metadata"].get("labels"))
                        and not n["spec"].get("unschedulable")]
            hc = self.__dict__.setdefault("_ds_hash", {})  # (uid, resourceVersion) -> template hash
            ck = (ds["metadata"].get("uid"), ds["metadata"].get("resourceVersion"))
            h = hc.get(ck)
            if h is None:
                if len(hc) > 1000:
                    hc.clear()
                h = hc[ck] = template_hash(tmpl)
            for n in eligible:
                nn = n["metadata"]["name"]
                if nn not in pods:
                    pods[nn] = self._new_pod(pid, ns, f"{ds['metadata']['name']}-{nn}", ds, "DaemonSet", tmpl, node=nn,
                                             labels={**(ds["spec"].get("selector", {}).get("matchLabels") or {}),
                                                     "controller-revision-hash": h,
                                                     # the validation DaemonSet's pods say so (the agent
                                                     # lets them read their machine's burn-in result)
                                                     **({VALIDATION_LABEL: "true"} if (ds["metadata"].get("labels")
                                                        or {}).get(VALIDATION_LABEL) == "true" else {})})
            # RollingUpdate (the default; OnDelete leaves it to the user): a changed template replaces
            # the running pods node by node, at most maxUnavailable (1) at a time
            upd = ds["spec"].get("updateStrategy") or {}
            if upd.get("type", "RollingUpdate") == "RollingUpdate":
                budget = int((upd.get("rollingUpdate") or {}).get("maxUnavailable", 1) or 1)
                down = sum(1 for o in pods.values() if o["metadata"].get("deletionTimestamp")
                           or o.get("status", {}).get("phase") == "Pending")
                for nn, o in sorted(pods.items()):
                    if down >= budget:
                        break
                    stale = (o["metadata"].get("labels") or {}).get("controller-revision-hash") not in (None, h)
                    if stale and o.get("status", {}).get("phase") == "Running" and not o["metadata"].get("deletionTimestamp"):
                        self._delete_pod(pid, ns, o["metadata"]["name"])
                        self._again = True  # its node gets the new template's pod once it is gone
                        down += 1
            phases = [o.get("status", {}).get("phase") for o in pods.values()]
            status = {"desiredNumberScheduled": len(eligible), "currentNumberScheduled": len(pods),
                      "numberReady": phases.count("Running") + phases.count("Succeeded"),
                      "numberSucceeded": phases.count("Succeeded"), "numberFailed": phases.count("Failed"),
                      "updatedNumberScheduled": sum(1 for o in pods.values() if (o["metadata"].get("labels") or {}).get(
                          "controller-revision-hash") == h)}
            if ds.get("status") != status:
                self.store.patch("daemonsets", _key(pid, ns, ds["metadata"]["name"]), lambda o, s=status: o.__setitem__("status", s))

    def _ctl_validation(self, pid: str) -> None:
        """Node condition AMDGPUValidated from the validation DaemonSet's pod on that node."""
        for ds in self.store.list("daemonsets", lambda o: self._in(pid, o) and o["metadata"].get("labels", {}).get(VALIDATION_LABEL) == "true"):
            for pod in self._owned(pid, ds):
                nn = pod["spec"].get("nodeName")
                phase = pod.get("status", {}).get("phase")
                if not nn or phase not in TERMINAL:
                    continue
                key = _key(pid, nn)
                n = self.store.get("nodes", key)
                if n is None:
                    continue
                result = pod.get("status", {}).get("result") or {}
                view = _xgmi_view(result)
                want = ("True", "ProbesPassed") if phase == "Succeeded" else ("False", "ProbesFailed")
                if want[0] == "True" and view is not None and not view["healthy"]:
                    want = ("False", "XGMILinkDegraded")
                c = _cond(n, "AMDGPUValidated")
                if c and (c["status"], c["reason"]) == want:
                    continue

                def fn(node, want=want, result=result, pod=pod, view=view):
                    from .. import xgmi

                    msg = xgmi.message(view) if want[1] == "XGMILinkDegraded" else pod.get("status", {}).get("message", "")
                    _set_cond(node, "AMDGPUValidated", want[0], want[1], msg[:500])
                    ann = node["metadata"].setdefault("annotations", {})
                    if view is not None:
                        ann.update(xgmi.annotations(view))
                        if view["healthy"]:
                            _set_cond(node, "XGMILinksHealthy", "True", "LinksHealthy",
                                      f"{view['pulls']} pulls >= {view.get('min_fraction')} x median {view.get('median_gbps')} GB/s")
                        else:
                            _set_cond(node, "XGMILinksHealthy", "False", "XGMILinkDegraded", xgmi.message(view))
                        _set_ready(node)
                    for k, path in (("hbm-write-gbps", ("hbm", "gbps")), ("hbm-read-gbps", ("hbm", "read_gbps")),
                                    ("md5-mbps", ("md5", "mbps")),
                                    ("copy-gbps", ("copy", "kernel_gbps")), ("probe-ms", ("timings_ms", "total")),
                                    ("hip-init-ms", ("timings_ms", "hip_init"))):
                        v = result.get(path[0], {}).get(path[1]) if isinstance(result.get(path[0]), dict) else None
                        if k.endswith(("gbps", "mbps")) and (result.get("hbm") or {}).get("timing") == "implausible":
                            ann["tk8s.amd.com/probe-timing"] = "implausible (GPU timestamps above the HBM peak)"
                            continue
                        if v is not None:
                            ann[f"tk8s.amd.com/{k}"] = f"{v:.1f}"

                self.store.patch("nodes", key, fn)
                if want[1] == "XGMILinkDegraded":
                    from .. import xgmi

                    self._event(pid, "default", {"kind": "Node", "name": nn}, "XGMILinkDegraded", xgmi.message(view),
                                "Warning")

    def _ctl_jobs(self, pid: str) -> None:
        """Job controller: ``completions``/``parallelism``, ``completionMode: Indexed`` (ranks get
        JOB_COMPLETION_INDEX), ``backoffLimit``; ``suspend`` stops the active pods and holds new
        ones back; ``activeDeadlineSeconds`` fails a job that ran too long (DeadlineExceeded) and
        ``ttlSecondsAfterFinished`` deletes a finished one with its pods (cron_loop keeps time)."""
        now = time.time()
        for job in self.store.list("jobs", lambda o: self._in(pid, o)):
            ns, jname = job["metadata"]["namespace"], job["metadata"]["name"]
            spec = job["spec"]
            st0 = job.get("status") or {}
            fin = next((c for c in st0.get("conditions", []) if c["type"] in ("Complete", "Failed") and c["status"] == "True"), None)
            ttl = spec.get("ttlSecondsAfterFinished")
            if fin is not None and ttl is not None and now - _epoch(fin.get("lastTransitionTime")) >= float(ttl):
                self._delete_job(pid, ns, jname)
                continue
            completions = int(spec.get("completions", 1))
            parallelism = int(spec.get("parallelism", completions))
            backoff = int(spec.get("backoffLimit", 6))
            indexed = spec.get("completionMode") == "Indexed"
            pods = self._owned(pid, job)
            succeeded_idx, active, failed = set(), 0, 0
            fail_job = None  # (message) of a podFailurePolicy FailJob match
            for o in pods:
                ph = o.get("status", {}).get("phase")
                idx = int(o["metadata"].get("annotations", {}).get("batch.kubernetes.io/job-completion-index", -1))
                if ph == "Succeeded":
                    succeeded_idx.add(idx if indexed else o["metadata"]["name"])
                elif o["metadata"].get("deletionTimestamp"):
                    continue  # terminating: neither active nor failed (its replacement may start)
                elif ph == "Failed":
                    action, why = _failure_action(spec.get("podFailurePolicy"), o)
                    if action == "FailJob" and fail_job is None:
                        fail_job = why
                    if action != "Ignore":  # Ignore: not counted, the pod is replaced
                        failed += 1
                else:
                    active += 1
            done = fin is not None
            suspended = bool(spec.get("suspend"))
            deadline = spec.get("activeDeadlineSeconds")
            started = st0.get("startTime") if not suspended else None
            over = (not done and not suspended and started is not None and deadline is not None
                    and now - _epoch(started) >= float(deadline))
            if not done and (failed > backoff or over or suspended or fail_job):
                for o in pods:  # stop the rest (a gang job cannot finish without all ranks)
                    if o.get("status", {}).get("phase") not in TERMINAL and not o["metadata"].get("deletionTimestamp"):
                        self._delete_pod(pid, ns, o["metadata"]["name"])
                        active -= 1
            elif not done:
                running_idx = {int(o["metadata"].get("annotations", {}).get("batch.kubernetes.io/job-completion-index", -1))
                               for o in pods if o.get("status", {}).get("phase") not in TERMINAL}
                need = [i for i in range(completions) if i not in succeeded_idx and i not in running_idx] if indexed \
                    else list(range(max(0, completions - len(succeeded_idx) - active)))
                for i in need[: max(0, parallelism - active)]:
                    self._seq += 1
                    name = f"{jname}-{i}-{self._seq:x}" if indexed else f"{jname}-{self._seq:x}"
                    env = {"JOB_COMPLETION_INDEX": i, "JOB_COMPLETIONS": completions, "JOB_NAME": jname} if indexed else {"JOB_NAME": jname}
                    self._new_pod(pid, ns, name, job, "Job", spec["template"], extra_env=env,
                                  labels={"job-name": jname},
                                  annotations={"batch.kubernetes.io/job-completion-index": str(i)} if indexed else None)
                    active += 1
            status = dict(job.get("status", {}))
            status.update(active=active, succeeded=len(succeeded_idx), failed=failed)
            conds = [c for c in status.get("conditions", [])]
            sus = next((c for c in conds if c["type"] == "Suspended"), None)
            if not done:
                if suspended and (sus is None or sus["status"] != "True"):
                    conds = [c for c in conds if c is not sus] + [{"type": "Suspended", "status": "True", "reason": "JobSuspended",
                                                                   "message": "Job suspended", "lastTransitionTime": now_iso()}]
                    status.pop("startTime", None)
                elif not suspended and sus is not None and sus["status"] == "True":
                    conds = [c for c in conds if c is not sus] + [{"type": "Suspended", "status": "False", "reason": "JobResumed",
                                                                   "message": "Job resumed", "lastTransitionTime": now_iso()}]
                if not suspended and "startTime" not in status:
                    status["startTime"] = now_iso()
                if len(succeeded_idx) >= completions:
                    conds.append({"type": "Complete", "status": "True", "lastTransitionTime": now_iso()})
                    status["completionTime"] = now_iso()
                elif fail_job:
                    conds.append({"type": "Failed", "status": "True", "reason": "PodFailurePolicy", "message": fail_job,
                                  "lastTransitionTime": now_iso()})
                elif failed > backoff:
                    conds.append({"type": "Failed", "status": "True", "reason": "BackoffLimitExceeded",
                                  "lastTransitionTime": now_iso()})
                elif over:
                    conds.append({"type": "Failed", "status": "True", "reason": "DeadlineExceeded",
                                  "message": "Job was active longer than specified deadline", "lastTransitionTime": now_iso()})
                    self._event(pid, ns, {"kind": "Job", "name": jname}, "DeadlineExceeded",
                                "Job was active longer than specified deadline", "Warning")
            status["conditions"] = conds
            if status != job.get("status"):
                self.store.patch("jobs", _key(pid, ns, jname), lambda o, s=status: o.__setitem__("status", s))

    def _ctl_deployments(self, pid: str) -> None:
        """Deployment controller with ReplicaSet-style generations: pods carry the
        ``pod-template-hash`` of the template they came from. A changed template rolls out with
        the RollingUpdate defaults (maxSurge 25 % rounded up, maxUnavailable 25 % rounded down;
        an old pod goes only when a new one runs), ``strategy: Recreate`` drops the old pods first.
        ``spec.paused`` (``kubectl rollout pause``) holds template changes back: the newest
        ReplicaSet's template keeps being scaled until the rollout is resumed."""
        for d in self.store.list("deployments", lambda o: self._in(pid, o)):
            ns, dname = d["metadata"]["namespace"], d["metadata"]["name"]
            spec = d["spec"]
            want = int(spec.get("replicas", 1))
            h = template_hash(spec["template"])
            tmpl = spec["template"]
            if spec.get("paused"):
                newest = max((rs for rs in self.store.list("replicasets", lambda o: self._in(pid, o) and any(
                    r.get("uid") == d["metadata"]["uid"] for r in o["metadata"].get("ownerReferences", [])))),
                    key=lambda rs: int((rs["metadata"].get("annotations") or {}).get(REVISION, "0") or 0), default=None)
                if newest is not None:
                    h = newest["metadata"]["labels"]["pod-template-hash"]
                    tmpl = newest["spec"]["template"]
            match = (spec.get("selector") or {}).get("matchLabels") or {}

            def live():
                return [o for o in self._owned(pid, d) if o.get("status", {}).get("phase") not in TERMINAL
                        and not o["metadata"].get("deletionTimestamp")]

            unavailable = want // 4
            for _ in range(2):  # scale down old -> room to surge again, in the same pass
                pods = live()
                new = [o for o in pods if o["metadata"].get("labels", {}).get("pod-template-hash") == h]
                old = [o for o in pods if o not in new]
                if (spec.get("strategy") or {}).get("type") == "Recreate" and old:
                    for o in old:
                        self._delete_pod(pid, ns, o["metadata"]["name"])
                    pods, old = new, []
                surge = max(1, -(-want // 4)) if old else 0
                for _ in range(max(0, min(want - len(new), want + surge - len(pods)))):
                    self._seq += 1
                    new.append(self._new_pod(pid, ns, f"{dname}-{h[:8]}-{self._seq:x}", d, "Deployment",
                                             tmpl, labels={**match, "pod-template-hash": h}))
                ready_new = sum(1 for o in new if o.get("status", {}).get("phase") == "Running")
                keep_old = max(0, want - unavailable - ready_new)
                for o in sorted(old, key=lambda o: o["metadata"]["name"])[keep_old:]:
                    self._delete_pod(pid, ns, o["metadata"]["name"])
                for o in sorted(new, key=lambda o: o["metadata"]["name"])[want:]:
                    self._delete_pod(pid, ns, o["metadata"]["name"])
            pods = live()
            self._sync_deployment_revisions(pid, d, h, pods, tmpl)
            running = sum(1 for o in pods if o.get("status", {}).get("phase") == "Running")
            status = {"observedGeneration": int(d["metadata"].get("generation", 1)), "replicas": len(pods),
                      "updatedReplicas": sum(1 for o in pods if o["metadata"].get("labels", {}).get("pod-template-hash") == h),
                      "readyReplicas": running, "availableReplicas": running,
                      "unavailableReplicas": max(0, want - running)}
            done = status["updatedReplicas"] == want == running and status["replicas"] == want
            status["conditions"] = _conditions(d, [
                ("Available", *(("True", "MinimumReplicasAvailable", "Deployment has minimum availability.")
                                if running >= want - unavailable else
                                ("False", "MinimumReplicasUnavailable", "Deployment does not have minimum availability."))),
                ("Progressing", "Unknown", "DeploymentPaused", "Deployment is paused") if spec.get("paused") else
                ("Progressing", "True", *(("NewReplicaSetAvailable", f'ReplicaSet "{dname}-{h}" has successfully progressed.')
                                          if done else ("ReplicaSetUpdated", f'ReplicaSet "{dname}-{h}" is progressing.')))])
            if d.get("status") != status:
                self.store.patch("deployments", _key(pid, ns, dname), lambda o, s=status: o.__setitem__("status", s))

    def _sync_deployment_revisions(self, pid: str, d: dict, h: str, pods: list[dict], template: dict | None = None) -> None:
        """A ReplicaSet per pod template the Deployment has had (``<name>-<pod-template-hash>``,
        annotation ``deployment.kubernetes.io/revision``), as Kubernetes keeps them: what
        ``kubectl get rs``, ``kubectl rollout history`` and ``kubectl rollout undo`` read. The pods
        stay the Deployment's own (this controller runs them); the ReplicaSets are its revision
        history, with replicas counted from the pods of their template, and only the newest
        ``revisionHistoryLimit`` (10) empty old ones are kept. Returning to an old template makes
        its ReplicaSet the newest revision again."""
        ns, dname, uid = d["metadata"]["namespace"], d["metadata"]["name"], d["metadata"]["uid"]
        match = (d["spec"].get("selector") or {}).get("matchLabels") or {}
        owned = {rs["metadata"].get("labels", {}).get("pod-template-hash"): rs for rs in self.store.list(
            "replicasets", lambda o: self._in(pid, o) and o["metadata"].get("namespace") == ns and any(
                r.get("uid") == uid for r in o["metadata"].get("ownerReferences", [])))}
        revs = {k: int(rs["metadata"].get("annotations", {}).get(REVISION, "0") or 0) for k, rs in owned.items()}
        counts: dict[str, int] = {}
        ready: dict[str, int] = {}
        for o in pods:
            ph = o["metadata"].get("labels", {}).get("pod-template-hash")
            counts[ph] = counts.get(ph, 0) + 1
            ready[ph] = ready.get(ph, 0) + (o.get("status", {}).get("phase") == "Running")
        top = max(revs.values(), default=0)
        want = int(d["spec"].get("replicas", 1))
        if h not in owned or revs[h] < top:  # a new template, or back to an old one: the newest revision
            revs[h] = top + 1 if (h not in owned or revs[h] < top) else revs[h]
        for ph in set(owned) | {h}:
            rs = owned.get(ph)
            n = counts.get(ph, 0)
            tmpl = copy.deepcopy(template or d["spec"]["template"]) if ph == h else (rs or {}).get("spec", {}).get("template")
            if tmpl is None:
                continue
            tmpl.setdefault("metadata", {}).setdefault("labels", {})["pod-template-hash"] = ph
            ann = {REVISION: str(revs[ph])}
            if ph == h:
                ann["deployment.kubernetes.io/desired-replicas"] = str(want)
            body = {"apiVersion": "apps/v1", "kind": "ReplicaSet",
                    "metadata": {"name": f"{dname}-{ph}", "namespace": ns, "labels": {**match, "pod-template-hash": ph},
                                 "annotations": {**((rs or {}).get("metadata", {}).get("annotations") or {}), **ann},
                                 "ownerReferences": [{"apiVersion": "apps/v1", "kind": "Deployment", "name": dname,
                                                      "uid": uid, "controller": True, "blockOwnerDeletion": True}]},
                    "spec": {"replicas": want if ph == h else n, "selector": {"matchLabels": {**match, "pod-template-hash": ph}},
                             "template": tmpl},
                    "status": {"replicas": n, "readyReplicas": ready.get(ph, 0), "availableReplicas": ready.get(ph, 0),
                               "fullyLabeledReplicas": n, "observedGeneration": 1}, "_project": pid}
            if rs is not None:
                body["metadata"]["uid"] = rs["metadata"]["uid"]
                body["metadata"]["creationTimestamp"] = rs["metadata"].get("creationTimestamp")
                if all(self._strip(rs).get(k) == body.get(k) for k in ("spec", "status")) and \
                        rs["metadata"].get("annotations") == body["metadata"]["annotations"]:
                    continue
            self.store.put("replicasets", _key(pid, ns, f"{dname}-{ph}"), body)
        limit = int(d["spec"].get("revisionHistoryLimit", 10))
        old = sorted((revs[ph], ph) for ph in owned if ph != h and not counts.get(ph))
        for _rev, ph in old[: max(0, len(old) - limit)]:
            self.store.delete("replicasets", _key(pid, ns, f"{dname}-{ph}"))
        if d["metadata"].get("annotations", {}).get(REVISION) != str(revs[h]):
            self.store.patch("deployments", _key(pid, ns, dname),
                             lambda o, r=str(revs[h]): o["metadata"].setdefault("annotations", {}).__setitem__(REVISION, r))

    def _ctl_endpoints(self, pid: str) -> None:
        """The Endpoints object of every Service with a selector: the Ready pods' IPs and the
        Service's target ports (named container ports resolved per pod), Not-Ready ones apart --
        what clients that discover backends through the API read (the proxy computes the same
        set itself, k8s_api._endpoints)."""
        services = self.store.list("services", lambda o: self._in(pid, o))
        wanted = set()
        for svc in services:
            sel = svc["spec"].get("selector") or {}
            if not sel:
                continue
            ns, name = svc["metadata"]["namespace"], svc["metadata"]["name"]
            wanted.add((ns, name))
            ready, not_ready, ports = [], [], {}
            for o in self.store.list("pods", lambda o, ns=ns: self._in(pid, o) and o["metadata"].get("namespace") == ns):
                if not labels_match(sel, o["metadata"].get("labels")) or o.get("status", {}).get("phase") != "Running":
                    continue
                ip = o["status"].get("podIP")
                if not ip:
                    continue
                addr = {"ip": ip, "nodeName": o["spec"].get("nodeName"),
                        "targetRef": {"kind": "Pod", "name": o["metadata"]["name"], "namespace": ns,
                                      "uid": o["metadata"].get("uid")}}
                is_ready = not o["metadata"].get("deletionTimestamp") and not any(
                    c.get("type") == "Ready" and c.get("status") == "False" for c in o["status"].get("conditions") or [])
                (ready if is_ready else not_ready).append(addr)
                for p in svc["spec"].get("ports") or []:
                    tp = p.get("targetPort", p.get("port"))
                    if isinstance(tp, str) and not tp.isdigit():
                        tp = next((cp.get("containerPort") for c in o["spec"].get("containers", [])
                                   for cp in c.get("ports", []) if cp.get("name") == tp), None)
                    if tp:
                        ports[p.get("name") or str(p.get("port"))] = {"name": p.get("name"), "port": int(tp),
                                                                      "protocol": p.get("protocol", "TCP")}
            subsets = []
            if ready or not_ready:
                sub = {"ports": sorted(ports.values(), key=lambda x: str(x["name"]))}
                if ready:
                    sub["addresses"] = sorted(ready, key=lambda a: a["ip"])
                if not_ready:
                    sub["notReadyAddresses"] = sorted(not_ready, key=lambda a: a["ip"])
                subsets = [sub]
            key = _key(pid, ns, name)
            cur = self.store.get("endpoints", key)
            if cur is None or cur.get("subsets") != subsets:
                self.store.put("endpoints", key, {  # (the store keeps the uid and creation time)
                    "metadata": {"name": name, "namespace": ns, "labels": dict(svc["metadata"].get("labels") or {})},
                    "subsets": subsets, "_project": pid})
        for ep in self.store.list("endpoints", lambda o: self._in(pid, o)):
            if (ep["metadata"]["namespace"], ep["metadata"]["name"]) not in wanted:
                self.store.delete("endpoints", _key(pid, ep["metadata"]["namespace"], ep["metadata"]["name"]))

    def _ctl_quotas(self, pid: str) -> None:
        """ResourceQuota status: ``hard`` echoed, ``used`` summed over the namespace's live pods."""
        quotas = self.store.list("resourcequotas", lambda o: self._in(pid, o))
        if not quotas:
            return
        from .objects import _fmt, pod_usage

        for q in quotas:
            ns = q["metadata"]["namespace"]
            used: dict[str, float] = {}
            for o in self.store.list("pods", lambda o, ns=ns: self._in(pid, o) and o["metadata"].get("namespace") == ns):
                if o.get("status", {}).get("phase") not in TERMINAL:
                    for k, v in pod_usage(o).items():
                        used[k] = used.get(k, 0.0) + v
            hard = (q.get("spec") or {}).get("hard") or {}
            status = {"hard": dict(hard), "used": {r: _fmt(used.get("pods" if r == "count/pods" else r, 0.0)) for r in hard}}
            if q.get("status") != status:
                self.store.patch("resourcequotas", _key(pid, ns, q["metadata"]["name"]),
                                 lambda o, s=status: o.__setitem__("status", s))
