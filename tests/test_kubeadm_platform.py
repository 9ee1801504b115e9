"""The kubeadm platform (``./setup.sh --platform kubeadm``): a real node runtime (ROCm,
amdgpu-dkms, containerd, kubeadm/kubelet) and a real Kubernetes on machines reached over SSH.

Nothing of it can run in this offline container (it needs root, apt mirrors, container images and
MI355X GPUs), so the tests pin what it WOULD do:

* every task of ansible/clusterUp-kubeadm.yml and its roles uses a core ``ansible.builtin``
  module, so stock ``ansible-playbook`` runs the same files (real Ansible itself is not installed
  here: parity with it is unpinned beyond this static check);
* ``--check`` through the in-repo engine renders every command, file and manifest, and the result
  is compared with a golden file (tests/golden/kubeadm_check.jsonl; regenerate with
  TK8S_REGOLDEN=1 after a deliberate change);
* the orchestrator refuses the platform on colocated sandboxes and reads readiness back from
  ``kubectl get nodes`` output.
"""
import json
import os
import shutil
from pathlib import Path

import pytest
import yaml

from tritonk8ssupervisor_amd.playbook import Playbook

REPO = Path(__file__).resolve().parents[1]
GOLDEN = REPO / "tests" / "golden" / "kubeadm_check.jsonl"
ROLES = ("k8sruntime", "kubeadmmaster", "kubeadmhost", "kubeadmvalidate")
BUILTIN = {"apt", "apt_repository", "get_url", "file", "copy", "command", "shell", "stat", "assert", "replace",
           "systemd_service", "fetch", "lineinfile", "uri", "wait_for", "set_fact", "debug", "slurp"}
TASK_KEYS = {"name", "register", "when", "until", "retries", "delay", "run_once", "delegate_to", "changed_when",
             "failed_when", "args", "local_action", "become", "notify", "ignore_errors", "loop", "with_items"}


def _tasks(role):
    return yaml.safe_load((REPO / "ansible" / "roles" / role / "tasks" / "main.yml").read_text())


def test_every_task_is_a_core_ansible_module():
    plays = yaml.safe_load((REPO / "ansible" / "clusterUp-kubeadm.yml").read_text())
    assert [p["roles"] for p in plays] == [[r] for r in ROLES]
    for role in ROLES:
        for t in _tasks(role):
            mods = [k for k in t if k not in TASK_KEYS]
            if "local_action" in t:
                assert not mods and t["local_action"]["module"] in BUILTIN, t
                continue
            assert len(mods) == 1, t
            mod = mods[0]
            assert mod.startswith("ansible.builtin.") and mod.split(".")[-1] in BUILTIN, (role, t.get("name"), mod)
            assert t.get("name"), t  # every task says what it does


def _inventory(tmp: Path) -> Path:
    inv = tmp / "hosts"
    inv.write_text("[MASTER]\nkubemaster ansible_host=10.20.0.1 tk8s_home=/home/ops/.tk8s/dist/0123456789abcdef\n"
                   "[HOST]\nkubenode1 ansible_host=10.20.0.2 tk8s_home=/home/ops/.tk8s/dist/0123456789abcdef\n"
                   "kubenode2 ansible_host=10.20.0.3 tk8s_home=/home/ops/.tk8s/dist/0123456789abcdef\n")
    return inv


def _check_run(tmp_path: Path) -> Playbook:
    from tritonk8ssupervisor_amd.orchestrator import init_workspace

    ws = init_workspace(tmp_path / "ws")
    ws.vars_file.write_text('master: 10.20.0.1\nkubernetes_name: "k8s dev"\nkubernetes_description: "k8s dev"\n')
    facts = {"ansible_kernel": "6.8.0-45-generic", "ansible_distribution_release": "jammy",
             "ansible_distribution": "Ubuntu", "ansible_architecture": "x86_64"}
    pb = Playbook(ws.ansible / "clusterUp-kubeadm.yml", _inventory(tmp_path), check=True, out=None,
                  extra_vars={**facts, "tk8s_manifests": "MANIFESTS", "tk8s_expected_gpus": 2, "tk8s_gpus_per_node": 1,
                              "tk8s_ready_timeout": 900})
    # the manifests are rendered from the repository's copy, their path is not part of the golden
    pb.extra_vars["tk8s_manifests"] = str(ws.manifests)
    res = pb.run()
    assert res.ok, res.failures
    return pb


def _normal(pb: Playbook, tmp_path: Path) -> list[dict]:
    out = []
    for t in pb.trace:
        if t["module"] in ("setup",):
            continue
        s = json.dumps(t, sort_keys=True).replace(str(tmp_path / "ws"), "WS")
        out.append(json.loads(s))
    return out


def test_check_mode_renders_the_golden_plan(tmp_path):
    pb = _check_run(tmp_path)
    got = _normal(pb, tmp_path)
    if os.environ.get("TK8S_REGOLDEN") == "1":
        GOLDEN.parent.mkdir(parents=True, exist_ok=True)
        GOLDEN.write_text("".join(json.dumps(t, sort_keys=True) + "\n" for t in got))
    want = [json.loads(x) for x in GOLDEN.read_text().splitlines()]
    assert len(got) == len(want)
    for g, w in zip(got, want):
        assert g == w, (g["task"], g["host"])


def test_check_mode_plan_content(tmp_path):
    """What the golden holds, spelled out: driver and runtime on every machine, kubeadm init on the
    master with the inventory's addresses, the AMD device plugin and the RCCL-tests DaemonSet."""
    t = _normal(_check_run(tmp_path), tmp_path)
    by = {}
    for x in t:
        by.setdefault((x["host"], x["task"]), x)
    for h in ("kubenode1", "kubenode2"):
        apt = by[(h, "GPU hosts - amdgpu-dkms, the HIP runtime, RCCL and AMD SMI")]["args"]
        assert apt["name"] == ["amdgpu-dkms", "rocm-hip-runtime", "rccl", "amd-smi-lib", "rocminfo"]
        assert "linux-headers-6.8.0-45-generic" in by[(h, "Base packages and the running kernel's headers "
                                                          "(amdgpu-dkms builds against them)")]["args"]["name"]
    assert ("kubemaster", "GPU hosts - amdgpu-dkms, the HIP runtime, RCCL and AMD SMI") not in by  # no GPU driver
    repo = by[("kubenode1", "ROCm repository")]["args"]["repo"]
    assert repo.endswith("https://repo.radeon.com/rocm/apt/7.0 jammy main")
    init = by[("kubemaster", "kubeadm init (etcd, kube-apiserver, kube-scheduler, kube-controller-manager)")]["args"]
    assert "--apiserver-advertise-address 10.20.0.1" in init["cmd"] and init["creates"] == "/etc/kubernetes/admin.conf"
    dp = by[("kubemaster", "AMD GPU device plugin manifest (amd.com/gpu on every MI355X node)")]["args"]["content"]
    assert "image: docker.io/rocm/k8s-device-plugin:latest" in dp and "/var/lib/kubelet/device-plugins" in dp
    assert by[("kubenode1", "The node's tk8s tools at a fixed path (hostPath of the RCCL-tests DaemonSet)")][
        "args"]["src"] == "/home/ops/.tk8s/dist/0123456789abcdef"


def test_kubeadm_refused_on_colocated_sandboxes(tmp_path, monkeypatch):
    from tritonk8ssupervisor_amd.orchestrator import Setup, SetupError, init_workspace

    monkeypatch.setenv("TK8S_FAKE_GPUS", "2")
    ws = init_workspace(tmp_path)
    s = Setup(ws, answers={"nodes": 1}, assume_yes=True, platform="kubeadm", out=lambda _l: None)
    with pytest.raises(SetupError, match="kubeadm platform"):
        s.configure()


def test_kubeadm_readiness_from_kubectl(tmp_path, monkeypatch):
    from types import SimpleNamespace

    from tritonk8ssupervisor_amd.orchestrator import Setup, SetupError, init_workspace

    ws = init_workspace(tmp_path)
    s = Setup(ws, platform="kubeadm", out=lambda _l: None)
    s.cfg = SimpleNamespace(RANCHER_MASTER_HOSTNAME="kubemaster", node_names=lambda: ["kubenode1", "kubenode2"],
                            KUBERNETES_NUMBER_OF_NODES=2, HOST_PACKAGE="bm-1gpu")
    monkeypatch.setattr(s, "expected_gpus", lambda: 2)

    def node(name, ready, gpus):
        return {"metadata": {"name": name}, "status": {"allocatable": {"amd.com/gpu": str(gpus)},
                                                        "conditions": [{"type": "Ready", "status": ready}]}}

    items = [node("kubemaster", "True", 0), node("kubenode1", "True", 1), node("kubenode2", "True", 1)]
    s.playbook_result = SimpleNamespace(hostvars={"kubemaster": {"tk8s_nodes": {"stdout": json.dumps({"items": items})}}})
    assert s.wait_ready() == {"ready": True, "nodes_ready": 2, "gpus_allocatable": 2, "nodes_validated": 2}
    items[2] = node("kubenode2", "False", 1)
    s.playbook_result.hostvars["kubemaster"]["tk8s_nodes"]["stdout"] = json.dumps({"items": items})
    with pytest.raises(SetupError, match="1/2 workers Ready"):
        s.wait_ready()
