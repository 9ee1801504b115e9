"""The kubeadm platform's side of the orchestrator (``--platform kubeadm``): the roles
(clusterUp-kubeadm.yml) install ROCm, amdgpu-dkms, containerd and kubeadm, init the master, join
the workers, deploy the AMD device plugin and the Kubernetes dashboard, and wait for every node
Ready with its amd.com/gpu; the orchestrator then reads readiness back from the real API server
through the master, prints ALL NODES READY, and runs the RCCL-tests Job on every GPU node (the
same order and the same meaning of "Ready" as on the tk8s platform). ``./setup.sh -c`` undoes
kubeadm on every host before the machines go. ``KubeadmPlatform`` is a mixin of orchestrator.Setup.

Single-node mode (a one-host inventory -- the one 8x MI355X node BASELINE.json names): the master
machine is the whole host and its only Kubernetes node (control plane + GPU worker, the
control-plane NoSchedule taint removed, the device plugin advertising all of the host's GPUs);
the wizard's worker count becomes GPU slots of that node (machines that claim GPUs of the host
and carry no kubelet). Reference anchors: rancher/server on the master and the rancher/agent join
(ansible/roles/ranchermaster/tasks/main.yml:6-13, ansible/roles/rancherhost/tasks/main.yml:26-34).
"""
from __future__ import annotations

import json
import os
import shlex
import time

from .executor import MachineExecutor
from .utils.pool import Pool
from .workspace import SetupError

KUBECTL = "kubectl --kubeconfig ${TK8S_SYSROOT:-}/etc/kubernetes/admin.conf"


def single_node(provider) -> bool:
    """Single-node kubeadm mode: the bare-metal inventory lists exactly one host."""
    f = getattr(provider, "single_host", None)
    return bool(f()) if callable(f) else False


class KubeadmPlatform:
    # -- kubeadm platform -------------------------------------------------------------------
    def _master_exec(self, cmd: str, timeout: float = 120, stdin: bytes | None = None) -> tuple[int, str]:
        ex = MachineExecutor(self.provider, self.engine.machines())
        return ex.exec(self.cfg.RANCHER_MASTER_HOSTNAME, cmd, timeout=timeout, stdin=stdin)

    @property
    def kubeadm_single_node(self) -> bool:
        return self.platform == "kubeadm" and single_node(self.provider)

    def kube_node_names(self) -> list[str]:
        """The Kubernetes nodes that carry the workers: one per worker machine, or -- single-node
        mode -- the master's node, which carries every GPU slot."""
        return [self.cfg.RANCHER_MASTER_HOSTNAME] if self.kubeadm_single_node else list(self.cfg.node_names())

    def _kubeadm_nodes(self) -> list[dict]:
        hv = getattr(self, "playbook_result", None)
        reg = ((hv.hostvars if hv else {}).get(self.cfg.RANCHER_MASTER_HOSTNAME) or {}).get("tk8s_nodes") or {}
        text = reg.get("stdout") or ""
        if not text:  # --resume past the playbook: ask the API server
            rc, text = self._master_exec(f"{KUBECTL} get nodes -o json")
            if rc != 0:
                raise SetupError(f"kubectl get nodes failed on the master: {text.strip()[-400:]}")
        return json.loads(text)["items"]

    def _kubeadm_ready(self) -> dict:
        """Readiness on the kubeadm platform: the kubeadmvalidate role already waited (bounded) for
        every node Ready and the expected amd.com/gpu; this reads back what the API server said."""
        items = self._kubeadm_nodes()
        want = set(self.kube_node_names())
        ready = [n for n in items if n["metadata"]["name"] in want and any(
            c.get("type") == "Ready" and c.get("status") == "True" for c in n.get("status", {}).get("conditions", []))]
        gpus = sum(int((n.get("status", {}).get("allocatable") or {}).get("amd.com/gpu", "0") or 0) for n in ready)
        out = {"ready": len(ready) == len(want) and gpus >= self.expected_gpus(), "nodes_ready": len(ready),
               "gpus_allocatable": gpus, "nodes_validated": len(ready)}
        if self.kubeadm_single_node:
            out["single_node"] = True
        if not out["ready"]:
            what = "the single node" if self.kubeadm_single_node else "workers"
            raise SetupError(f"cluster not ready: {len(ready)}/{len(want)} {what} Ready, {gpus} amd.com/gpu "
                             f"(expected {self.expected_gpus()})", code=124)
        return out

    def ready_line(self, ready: dict, t_ready: float) -> str:
        if ready.get("single_node"):
            return (f"ALL NODES READY: 1 node(s) (single-node: {self.cfg.RANCHER_MASTER_HOSTNAME} is control plane and "
                    f"GPU worker, {self.cfg.KUBERNETES_NUMBER_OF_NODES} worker slot(s)), "
                    f"{ready.get('gpus_allocatable', 0)} x amd.com/gpu allocatable after {t_ready:.3f}s")
        return (f"ALL NODES READY: {ready.get('nodes_ready', 0)} node(s), "
                f"{ready.get('gpus_allocatable', 0)} x amd.com/gpu allocatable after {t_ready:.3f}s")

    # -- the RCCL-tests Jobs -------------------------------------------------------------------
    def kubeadm_rccl(self) -> dict | None:
        """One RCCL-tests Job per GPU node (manifests/kubeadm/rccl-tests-job.yaml), after Ready.
        Done when every GPU node has exactly one pod that terminated successfully and whose JSON
        says the all-reduce was exact; a failed pod, a Job the cluster cannot place, or no
        result within the bound fails ./setup.sh with the reason. Finished pods hold no GPU."""
        from .kube import load_manifests

        if not self.validate or self.rccl is False:
            return None
        gpu_nodes = {n["metadata"]["name"]: int((n.get("status", {}).get("allocatable") or {}).get("amd.com/gpu", 0) or 0)
                     for n in self._kubeadm_nodes()}
        gpu_nodes = {k: v for k, v in gpu_nodes.items() if v > 0}
        if not gpu_nodes:
            return None
        run_id = f"{int(time.time() * 1000) % 10**9:x}"
        gv = self._kubeadm_group_vars()
        docs = []
        jobs = {}
        for node, g in sorted(gpu_nodes.items()):
            job = f"tk8s-rccl-{run_id}-{len(jobs)}"
            jobs[node] = job
            docs += load_manifests(self.ws.manifests / "kubeadm" / "rccl-tests-job.yaml", {
                "job_name": job, "run_id": run_id, "node": node, "gpus": g, "max_bytes": self.rccl_max_bytes,
                "rccl_tests_image": gv.get("rccl_tests_image", "docker.io/library/ubuntu:22.04"),
                "tk8s_install_dir": gv.get("tk8s_install_dir", "/opt/tk8s")})
        text = json.dumps({"apiVersion": "v1", "kind": "List", "items": docs}, indent=1)
        path = f"${{TK8S_SYSROOT:-}}/etc/kubernetes/tk8s/rccl-tests-{run_id}.json"
        rc, out = self._master_exec(f"mkdir -p ${{TK8S_SYSROOT:-}}/etc/kubernetes/tk8s && cat > {path} && "
                                    f"{KUBECTL} apply -f {path}", stdin=text.encode())
        if rc != 0:
            raise SetupError(f"RCCL-tests: kubectl apply failed on the master: {out.strip()[-600:]}", code=2)
        self.out(f"Running RCCL all-reduce on {len(jobs)} GPU node(s) ({sum(gpu_nodes.values())} GPU(s); "
                 f"Jobs kube-system/tk8s-rccl-{run_id}-*)")
        deadline = time.monotonic() + max(10.0, self.rccl_timeout or self.timeout)
        poll = float(os.environ.get("TK8S_RCCL_POLL", "2"))
        while True:
            rc, out = self._master_exec(f"{KUBECTL} -n kube-system get pods -l tk8s.amd.com/rccl-run={run_id} -o json")
            pods = (last_json(out) or {}).get("items", []) if rc == 0 else []
            verdict = rccl_job_verdict(pods, jobs)
            if verdict["state"] == "failed":
                raise SetupError(f"RCCL all-reduce validation failed: {verdict['reason']}", code=2)
            if verdict["state"] == "done":
                break
            if time.monotonic() > deadline:
                raise SetupError(f"RCCL all-reduce did not finish within {max(10.0, self.rccl_timeout or self.timeout):.0f}s: "
                                 f"{verdict['reason']}", code=124)
            time.sleep(poll)
        results = {}
        for node, pod in verdict["pods"].items():
            rc, log = self._master_exec(f"{KUBECTL} -n kube-system logs {shlex.quote(pod)}")
            res = last_json(log)
            if rc != 0 or res is None or not res.get("ok"):
                raise SetupError(f"RCCL all-reduce validation failed on {node}: pod {pod} reported "
                                 f"{json.dumps(res)[:400] if res else repr(log.strip()[-400:])}", code=2)
            results[node] = res
        from .fabric import bandwidth_summary

        # one Job per node: each node's ranks form their own communicator (busbw null for a 1-GPU node)
        bw = bandwidth_summary(list(results.values()), max(gpu_nodes.values()))
        return {"ok": True, "platform": "kubeadm", "run": run_id, "jobs": [f"kube-system/{j}" for j in jobs.values()],
                "pods": len(results), "nranks": sum(gpu_nodes.values()), "gpus_per_pod": max(gpu_nodes.values()),
                **bw,
                "rank_results": [{"pod": verdict["pods"][n], "node": n, "ok": True,
                                  "peak_busbw_gbps": r.get("peak_busbw_gbps"), "comm_init_ms": r.get("comm_init_ms")}
                                 for n, r in sorted(results.items())]}

    def _kubeadm_group_vars(self) -> dict:
        from .utils import yamlio

        p = self.ws.ansible / "group_vars" / "all.yml"
        try:
            return yamlio.load(p.read_text()) or {}
        except OSError:
            return {}

    def _kubeadm_finish(self, ready: dict, rccl, t_ready: float, total: float) -> dict:
        m = self.engine.machines()[self.cfg.RANCHER_MASTER_HOSTNAME]
        kubeconfig = self.ws.ansible / "tmp" / "kubeconfig"
        port = self._kubeadm_group_vars().get("dashboard_node_port", 30443)
        self.summary = {
            "platform": "kubeadm", "ready_seconds": round(t_ready, 4), "total_seconds": round(total, 4),
            "rccl_check_s": round(self.events.phases.get("rccl", 0.0), 4),
            "nodes": int(self.cfg.KUBERNETES_NUMBER_OF_NODES), "kubernetes_nodes": len(self.kube_node_names()),
            "single_node": self.kubeadm_single_node,
            "gpus_allocatable": ready.get("gpus_allocatable", 0),
            "nodes_validated": ready.get("nodes_validated", 0), "rccl": rccl,
            "phases": {k: round(v, 4) for k, v in self.events.phases.items()},
            "api": f"https://{m.primaryip}:6443", "kubectl_config": str(kubeconfig),
            "dashboard": f"https://{m.primaryip}:{port}/",
            "dashboard_token": str(self.ws.ansible / "tmp" / "dashboard-token"),
            "project": self.project_id() if self.ws.env_id_file.exists() else "",
        }
        self.ws.save_state(summary=self.summary, finished=time.time())
        self.events.emit("setup_done", **{k: v for k, v in self.summary.items() if k != "phases"})
        self.out("")
        self.out("Congratulations, your Kubernetes cluster setup has been complete.")
        self.out(f"----> Kubernetes dashboard is at {self.summary['dashboard']} "
                 f"(login token: {self.summary['dashboard_token']})")
        self.out(f"----> Kubernetes CLI config is at {kubeconfig}  (KUBECONFIG={kubeconfig} kubectl get nodes)")
        self.out(f"----> Kubernetes API server is at {self.summary['api']}")
        if self.kubeadm_single_node:
            self.out(f"----> single-node cluster: {self.cfg.RANCHER_MASTER_HOSTNAME} runs the control plane and every "
                     f"GPU; the {self.summary['nodes']} worker(s) are GPU slots of it, "
                     f"{self.summary['gpus_allocatable']} x amd.com/gpu allocatable")
        else:
            self.out(f"----> {self.summary['nodes']} node(s) Ready, {self.summary['gpus_allocatable']} x amd.com/gpu "
                     "allocatable")
        if rccl:
            bw = (f"peak busbw {rccl['peak_busbw_gbps']:.1f} GB/s" if rccl.get("peak_busbw_gbps") is not None
                  else "1 GPU per node: no fabric")
            self.out(f"----> RCCL all-reduce: {rccl['pods']} node(s), {rccl['nranks']} GPU(s), {bw}")
        self.out(f"----> bring-up: {t_ready:.3f}s to all nodes Ready ({total:.3f}s including fabric validation)")
        return self.summary


def rccl_job_verdict(pods: list[dict], jobs: dict[str, str]) -> dict:
    """State of the RCCL-tests Jobs from their pods (``kubectl get pods -o json``): ``done`` when
    every GPU node (jobs: node -> Job name) has exactly one pod that terminated with exit code 0,
    ``failed`` as soon as any of them failed (or a node got more than one pod: the Jobs run with
    backoffLimit 0, so a second pod means a retry nobody asked for), else ``waiting`` with why."""
    by_job: dict[str, list[dict]] = {j: [] for j in jobs.values()}
    for p in pods:
        j = (p.get("metadata", {}).get("labels") or {}).get("job-name") or ""
        if j in by_job:
            by_job[j].append(p)
    done, waiting = {}, []
    for node, job in sorted(jobs.items()):
        ps = by_job[job]
        if not ps:
            waiting.append(f"{node}: no pod yet")
            continue
        if len(ps) > 1:
            return {"state": "failed", "reason": f"{node}: {len(ps)} pods for Job {job} (expected exactly one)"}
        p = ps[0]
        st = p.get("status") or {}
        phase = st.get("phase", "Pending")
        term = ((((st.get("containerStatuses") or [{}])[0]).get("state") or {}).get("terminated")) or {}
        name = p["metadata"]["name"]
        if phase == "Failed" or (term and int(term.get("exitCode", 1)) != 0):
            why = term.get("reason") or st.get("reason") or "Error"
            msg = term.get("message") or st.get("message") or ""
            return {"state": "failed", "reason": f"{node}: pod {name} failed ({why}, exit code {term.get('exitCode', '?')})"
                                                 + (f": {msg}" if msg else "")}
        if phase == "Succeeded":
            done[node] = name
            continue
        cond = next((c for c in st.get("conditions") or [] if c.get("type") == "PodScheduled"
                     and c.get("status") == "False"), None)
        waiting.append(f"{node}: pod {name} {phase}" + (f" ({cond.get('message', '')})" if cond else ""))
    if waiting:
        return {"state": "waiting", "reason": "; ".join(waiting), "pods": done}
    return {"state": "done", "reason": "", "pods": done}


def last_json(text: str) -> dict | None:
    """The JSON object in a command's output: the whole text when it is one (``kubectl -o json``),
    else the last line that parses as one (tk8s-rccl prints RCCL's banner first)."""
    text = text or ""
    i = text.find("{")
    if i >= 0:
        try:
            return json.loads(text[i:])
        except ValueError:
            pass
    for line in reversed(text.splitlines()):
        line = line.strip()
        if line.startswith("{"):
            try:
                return json.loads(line)
            except ValueError:
                continue
    return None


def kubeadm_extra_vars(setup, cfg) -> dict:
    """What the kubeadm roles need beyond the inventory and the role defaults."""
    per_node = 0
    try:
        per_node = int(setup.provider.package_by_id_or_name(cfg.HOST_PACKAGE).gpus or 0)
    except Exception:  # noqa: BLE001
        pass
    return {"tk8s_expected_gpus": per_node * int(cfg.KUBERNETES_NUMBER_OF_NODES), "tk8s_gpus_per_node": per_node,
            "tk8s_ready_timeout": int(setup.timeout), "tk8s_single_node": single_node(setup.provider)}


KUBEADM_RESET = ("kubeadm reset -f --cri-socket unix:///run/containerd/containerd.sock; "
                 'rm -rf "${TK8S_SYSROOT:-}/etc/cni/net.d" "${TK8S_SYSROOT:-}/root/.kube" '
                 '"${TK8S_SYSROOT:-}/etc/kubernetes/tk8s"; systemctl restart containerd || true')


def kubeadm_reset(ws, provider, out) -> None:
    """Undo kubeadm init/join on every host before the machines go, once per host (single-node
    mode puts every machine on one host; best effort: a machine that is gone needs nothing)."""
    if not (ws.tf / "terraform.tfstate").exists():
        return
    from .provision import Engine

    machines = list(Engine(ws.tf, provider).machines().values())
    per_host: dict[str, object] = {}
    for m in sorted(machines, key=lambda m: (m.tags.get("role") != "master", m.name)):
        per_host.setdefault(m.tags.get("tk8s_host") or m.name, m)
    targets = list(per_host.values())
    with Pool(max(1, len(targets)), "kubeadm-reset") as pool:
        for m, (rc, text) in zip(targets, pool.map(lambda m: provider.exec(m, KUBEADM_RESET, timeout=300), targets)):
            out(f"    kubeadm reset on {m.name}: {'ok' if rc == 0 else 'failed: ' + text.strip()[-200:]}")
