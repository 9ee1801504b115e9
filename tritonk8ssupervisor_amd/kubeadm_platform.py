"""The kubeadm platform's side of the orchestrator (``--platform kubeadm``): the roles
(clusterUp-kubeadm.yml) install ROCm, amdgpu-dkms, containerd and kubeadm, init the master, join
the workers and run the RCCL-tests DaemonSet; the orchestrator then reads readiness back from
the real API server through the master, and ``./setup.sh -c`` undoes kubeadm on every machine
before the machines go. ``KubeadmPlatform`` is a mixin of orchestrator.Setup.
"""
from __future__ import annotations

import json
import time

from .executor import MachineExecutor
from .utils.pool import Pool
from .workspace import SetupError


class KubeadmPlatform:
    # -- kubeadm platform -------------------------------------------------------------------
    def _master_exec(self, cmd: str, timeout: float = 120) -> tuple[int, str]:
        ex = MachineExecutor(self.provider, self.engine.machines())
        return ex.exec(self.cfg.RANCHER_MASTER_HOSTNAME, cmd, timeout=timeout)

    def _kubeadm_nodes(self) -> list[dict]:
        hv = getattr(self, "playbook_result", None)
        reg = ((hv.hostvars if hv else {}).get(self.cfg.RANCHER_MASTER_HOSTNAME) or {}).get("tk8s_nodes") or {}
        text = reg.get("stdout") or ""
        if not text:  # --resume past the playbook: ask the API server
            rc, text = self._master_exec("kubectl --kubeconfig /etc/kubernetes/admin.conf get nodes -o json")
            if rc != 0:
                raise SetupError(f"kubectl get nodes failed on the master: {text.strip()[-400:]}")
        return json.loads(text)["items"]

    def _kubeadm_ready(self) -> dict:
        """Readiness on the kubeadm platform: the kubeadmvalidate role already waited (bounded) for
        every node Ready and the expected amd.com/gpu; this reads back what the API server said."""
        items = self._kubeadm_nodes()
        workers = set(self.cfg.node_names())
        ready = [n for n in items if n["metadata"]["name"] in workers and any(
            c.get("type") == "Ready" and c.get("status") == "True" for c in n.get("status", {}).get("conditions", []))]
        gpus = sum(int((n.get("status", {}).get("allocatable") or {}).get("amd.com/gpu", "0") or 0) for n in ready)
        out = {"ready": len(ready) == len(workers) and gpus >= self.expected_gpus(), "nodes_ready": len(ready),
               "gpus_allocatable": gpus, "nodes_validated": len(ready)}
        if not out["ready"]:
            raise SetupError(f"cluster not ready: {len(ready)}/{len(workers)} workers Ready, {gpus} amd.com/gpu "
                             f"(expected {self.expected_gpus()})", code=124)
        return out

    def _kubeadm_finish(self, ready: dict, rccl, t_ready: float, total: float) -> dict:
        m = self.engine.machines()[self.cfg.RANCHER_MASTER_HOSTNAME]
        kubeconfig = self.ws.ansible / "tmp" / "kubeconfig"
        self.summary = {
            "platform": "kubeadm", "ready_seconds": round(t_ready, 4), "total_seconds": round(total, 4),
            "nodes": int(self.cfg.KUBERNETES_NUMBER_OF_NODES), "gpus_allocatable": ready.get("gpus_allocatable", 0),
            "nodes_validated": ready.get("nodes_validated", 0), "rccl": rccl,
            "phases": {k: round(v, 4) for k, v in self.events.phases.items()},
            "api": f"https://{m.primaryip}:6443", "kubectl_config": str(kubeconfig),
            "project": self.project_id() if self.ws.env_id_file.exists() else "",
        }
        self.ws.save_state(summary=self.summary, finished=time.time())
        self.events.emit("setup_done", **{k: v for k, v in self.summary.items() if k != "phases"})
        self.out("")
        self.out("Congratulations, your Kubernetes cluster setup has been complete.")
        self.out(f"----> Kubernetes API server is at {self.summary['api']}")
        self.out(f"----> kubectl: KUBECONFIG={kubeconfig} kubectl get nodes")
        self.out(f"----> {self.summary['nodes']} node(s) Ready, {self.summary['gpus_allocatable']} x amd.com/gpu allocatable")
        self.out(f"----> bring-up: {t_ready:.3f}s to all nodes Ready ({total:.3f}s including fabric validation)")
        return self.summary


def kubeadm_extra_vars(setup, cfg) -> dict:
    """What the kubeadm roles need beyond the inventory and the role defaults."""
    per_node = 0
    try:
        per_node = int(setup.provider.package_by_id_or_name(cfg.HOST_PACKAGE).gpus or 0)
    except Exception:  # noqa: BLE001
        pass
    return {"tk8s_expected_gpus": per_node * int(cfg.KUBERNETES_NUMBER_OF_NODES), "tk8s_gpus_per_node": per_node,
            "tk8s_ready_timeout": int(setup.timeout)}


KUBEADM_RESET = ("kubeadm reset -f --cri-socket unix:///run/containerd/containerd.sock; "
                 'rm -rf "${TK8S_SYSROOT:-}/etc/cni/net.d" "${TK8S_SYSROOT:-}/root/.kube" '
                 '"${TK8S_SYSROOT:-}/etc/kubernetes/tk8s"; systemctl restart containerd || true')


def kubeadm_reset(ws, provider, out) -> None:
    """Undo kubeadm init/join on every machine before the machines go (best effort: a machine
    that is gone already needs nothing)."""
    if not (ws.tf / "terraform.tfstate").exists():
        return
    from .provision import Engine

    machines = list(Engine(ws.tf, provider).machines().values())
    with Pool(max(1, len(machines)), "kubeadm-reset") as pool:
        for m, (rc, text) in zip(machines, pool.map(lambda m: provider.exec(m, KUBEADM_RESET, timeout=300), machines)):
            out(f"    kubeadm reset on {m.name}: {'ok' if rc == 0 else 'failed: ' + text.strip()[-200:]}")
