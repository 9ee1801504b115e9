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
GOLDEN_SINGLE = REPO / "tests" / "golden" / "kubeadm_check_single.jsonl"
ROLES = ("k8sruntime", "kubeadmmaster", "kubeadmhost", "kubeadmvalidate")
BUILTIN = {"apt", "apt_repository", "get_url", "file", "copy", "command", "shell", "stat", "assert", "replace",
           "systemd_service", "fetch", "lineinfile", "uri", "wait_for", "set_fact", "debug", "slurp"}
TASK_KEYS = {"name", "register", "when", "until", "retries", "delay", "run_once", "delegate_to", "changed_when",
             "failed_when", "args", "local_action", "become", "notify", "ignore_errors", "loop", "with_items",
             "no_log"}


def _tasks(role):
    return yaml.safe_load((REPO / "ansible" / "roles" / role / "tasks" / "main.yml").read_text())


def test_every_task_is_a_core_ansible_module():
    plays = yaml.safe_load((REPO / "ansible" / "clusterUp-kubeadm.yml").read_text())
    assert [[r if isinstance(r, str) else r["role"] for r in p["roles"]] for p in plays] == [[r] for r in ROLES]
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


def _inventory(tmp: Path, single: bool = False) -> Path:
    inv = tmp / "hosts"
    home = "tk8s_home=/home/ops/.tk8s/dist/0123456789abcdef"
    if single:  # one host: the master machine and the GPU slots share its address
        inv.write_text(f"[MASTER]\nkubemaster ansible_host=10.20.0.1 {home}\n"
                       + "[HOST]\n" + "".join(f"kubenode{i} ansible_host=10.20.0.1 {home}\n" for i in range(1, 9)))
        return inv
    inv.write_text(f"[MASTER]\nkubemaster ansible_host=10.20.0.1 {home}\n"
                   f"[HOST]\nkubenode1 ansible_host=10.20.0.2 {home}\n"
                   f"kubenode2 ansible_host=10.20.0.3 {home}\n")
    return inv


def _check_run(tmp_path: Path, single: bool = False) -> Playbook:
    from tritonk8ssupervisor_amd.orchestrator import init_workspace

    ws = init_workspace(tmp_path / "ws")
    ws.vars_file.write_text('master: 10.20.0.1\nkubernetes_name: "k8s dev"\nkubernetes_description: "k8s dev"\n')
    facts = {"ansible_kernel": "6.8.0-45-generic", "ansible_distribution_release": "jammy",
             "ansible_distribution": "Ubuntu", "ansible_architecture": "x86_64"}
    pb = Playbook(ws.ansible / "clusterUp-kubeadm.yml", _inventory(tmp_path, single), check=True, out=None,
                  extra_vars={**facts, "tk8s_manifests": "MANIFESTS", "tk8s_expected_gpus": 8 if single else 2,
                              "tk8s_gpus_per_node": 1, "tk8s_ready_timeout": 900, "tk8s_single_node": single})
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


@pytest.mark.parametrize("single", [False, True], ids=["multi-host", "single-node"])
def test_check_mode_renders_the_golden_plan(tmp_path, single):
    pb = _check_run(tmp_path, single)
    got = _normal(pb, tmp_path)
    golden = GOLDEN_SINGLE if single else GOLDEN
    if os.environ.get("TK8S_REGOLDEN") == "1":
        golden.parent.mkdir(parents=True, exist_ok=True)
        golden.write_text("".join(json.dumps(t, sort_keys=True) + "\n" for t in got))
    want = [json.loads(x) for x in golden.read_text().splitlines()]
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
    assert repo.endswith("https://repo.radeon.com/rocm/apt/7.2 jammy main")
    init = by[("kubemaster", "kubeadm init (etcd, kube-apiserver, kube-scheduler, kube-controller-manager)")]["args"]
    assert "--apiserver-advertise-address 10.20.0.1" in init["cmd"] and init["creates"] == "/etc/kubernetes/admin.conf"
    dp = by[("kubemaster", "AMD GPU device plugin manifest (amd.com/gpu on every MI355X node)")]["args"]["content"]
    assert "image: docker.io/rocm/k8s-device-plugin:1.31.0.6" in dp and "/var/lib/kubelet/device-plugins" in dp
    # the dashboard is deployed and every image / manifest is pinned
    assert by[("kubemaster", "Kubernetes dashboard")]["args"]["_raw_params"].endswith(
        "kubernetes/dashboard/v2.7.0/aio/deploy/recommended.yaml")
    access = by[("kubemaster", "Dashboard access objects manifest (NodePort service, admin service account)")]
    assert "nodePort: 30443" in access["args"]["content"] and "name: cluster-admin" in access["args"]["content"]
    assert not [x for x in t if ":latest" in json.dumps(x["args"]) or "releases/latest" in json.dumps(x["args"])]
    # Ready stops at the nodes and their GPUs: the RCCL-tests Job runs after ALL NODES READY (fabric.py)
    assert not [x for x in t if "rccl" in json.dumps(x["args"]).lower() and x["play"].startswith("Every node")]
    assert by[("kubenode1", "The node's tk8s tools at a fixed path (hostPath of the RCCL-tests Job)")][
        "args"]["src"] == "/home/ops/.tk8s/dist/0123456789abcdef"


def test_single_node_check_plan(tmp_path):
    """one host carries the control plane and the GPU worker. Only the master machine
    installs the runtime; its taint is removed; no machine joins; the master's node is the GPU node."""
    t = _normal(_check_run(tmp_path, single=True), tmp_path)
    hosts = {x["host"] for x in t}
    assert hosts == {"kubemaster"}, hosts  # the GPU slots run nothing
    names = [x["task"] for x in t]
    assert "GPU hosts - amdgpu-dkms, the HIP runtime, RCCL and AMD SMI" in names
    untaint = next(x for x in t if x["task"].startswith("Single-node cluster"))
    assert untaint["args"]["_raw_params"].endswith("taint nodes kubemaster node-role.kubernetes.io/control-plane:NoSchedule-")
    assert not any(x["task"].startswith("kubeadm join") for x in t)
    assert not any(x["task"].startswith("Join command") for x in t)
    label = next(x for x in t if x["task"].startswith("Label the GPU nodes"))
    assert "label node kubemaster amd.com/gpu.family=gfx950" in label["args"]["_raw_params"]


def test_kubeadm_refused_on_colocated_sandboxes(tmp_path, monkeypatch):
    from tritonk8ssupervisor_amd.orchestrator import Setup, SetupError, init_workspace

    monkeypatch.setattr(os, "geteuid", lambda: 1000)  # not root: no kubeadm on this host itself
    monkeypatch.delenv("TK8S_LOCAL_HOST_ROOT", raising=False)
    monkeypatch.setenv("TK8S_FAKE_GPUS", "2")
    ws = init_workspace(tmp_path)
    s = Setup(ws, answers={"nodes": 1}, assume_yes=True, platform="kubeadm", out=lambda _l: None)
    with pytest.raises(SetupError, match="kubeadm platform"):
        s.configure()


def test_kubeadm_readiness_from_kubectl(tmp_path, monkeypatch):
    from types import SimpleNamespace

    from tritonk8ssupervisor_amd.orchestrator import Setup, SetupError, init_workspace

    monkeypatch.setattr(os, "geteuid", lambda: 1000)  # the multi-host form (as root, kubeadm would use this host)
    monkeypatch.delenv("TK8S_LOCAL_HOST_ROOT", raising=False)
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


# ---- the kubeadm platform for real, against simulated system tools ----------------------------------
SAFE_TOOLS = ("bash", "sh", "tar", "gzip", "mkdir", "cat", "mv", "rm", "ln", "chmod", "install", "grep", "sed", "cut",
              "md5sum", "base64", "stat", "readlink", "head", "tail", "find", "sleep", "date", "setsid", "kill", "env",
              "dirname", "basename", "id", "hostname", "uname", "nproc", "ip", "awk", "touch", "wc", "sort", "xargs",
              "tr", "cp", "ls", "pwd", "test", "true", "false", "printf", "echo")
FAKE_TOOLS = ("apt-get", "apt-mark", "dpkg-query", "modprobe", "sysctl", "swapoff", "systemctl", "containerd", "curl",
              "kubeadm", "kubectl")


def _fake_root_host(root: Path, addr: str, pubkey: str, state: Path, gpus: int = 0) -> Path:
    import sys

    h = root / addr
    (h / ".ssh").mkdir(parents=True)
    (h / ".ssh" / "authorized_keys").write_text(pubkey)
    (h / ".fakeroot").touch()
    (h / ".env").write_text(f"FAKE_K8S_STATE={state}\nFAKE_HOST_GPUS={gpus}\n")
    (h / "sysroot" / "etc").mkdir(parents=True)
    (h / "sysroot" / "etc" / "fstab").write_text("/dev/sda1 / ext4 defaults 0 1\n/swap.img none swap sw 0 0\n")
    b = h / "bin"
    b.mkdir()
    for t in SAFE_TOOLS:
        real = shutil.which(t)
        if real:
            (b / t).symlink_to(real)
    (b / "python3").symlink_to(sys.executable)
    tool = REPO / "tests" / "fakeroot" / "faketool.py"
    for t in FAKE_TOOLS:  # one wrapper per tool name; the stand-in dispatches on FAKETOOL_NAME
        (b / t).write_text(f"#!/bin/sh\nFAKETOOL_NAME={t} exec {sys.executable} {tool} \"$@\"\n")
        (b / t).chmod(0o755)
    return h


def test_kubeadm_platform_end_to_end_against_simulated_tools(tmp_path):
    """./setup.sh --backend baremetal --platform kubeadm for real: every task of the four plays runs
    over ssh on two fake-root hosts whose apt-get/kubeadm/kubectl/systemctl/... are stand-ins
    (tests/fakeroot/faketool.py) and whose system paths live under a staging root -- so the roles'
    control flow (facts, registered results, the join command handed from master to hosts, the
    readiness waits, the RCCL-tests DaemonSet check) is exercised end to end, then torn down with
    kubeadm reset."""
    import subprocess
    import sys

    from tritonk8ssupervisor_amd.orchestrator import init_workspace

    ws = tmp_path / "ws"
    ws.mkdir()
    init_workspace(ws)
    for f in ("setup.sh", "tk8s", "kubectl"):
        shutil.copy2(REPO / f, ws / f)
    # the staging root of each host, from its login HOME (ansible_env, gathered in play 1)
    gv = ws / "ansible" / "group_vars" / "all.yml"
    gv.write_text(gv.read_text().replace('tk8s_sysroot: ""', 'tk8s_sysroot: "{{ ansible_env.HOME }}/sysroot"'))
    keydir = tmp_path / "keys"
    keydir.mkdir()
    subprocess.run(["ssh-keygen", "-q", "-t", "ed25519", "-N", "", "-f", str(keydir / "id_ed25519")], check=True)
    root = tmp_path / "hosts"
    state = tmp_path / "cluster.json"
    hosts = {"mi355x-a": "127.0.7.30", "mi355x-b": "127.0.7.31", "mi355x-c": "127.0.7.32"}
    for h, addr in hosts.items():
        _fake_root_host(root, addr, (keydir / "id_ed25519.pub").read_text(), state, gpus=0 if h == "mi355x-a" else 1)
    inv = {"ssh": {"user": "root", "key": str(keydir / "id_ed25519")}, "python": sys.executable,
           "hosts": [{"name": "mi355x-a", "address": hosts["mi355x-a"], "gpus": 0, "role": "master"},
                     {"name": "mi355x-b", "address": hosts["mi355x-b"], "gpus": 1},
                     {"name": "mi355x-c", "address": hosts["mi355x-c"], "gpus": 1}]}
    (ws / "inventory.yml").write_text(json.dumps(inv))
    env = dict(os.environ, PYTHONPATH=str(REPO), TK8S_PYTHON=sys.executable, TK8S_BACKEND="baremetal",
               TK8S_SSH=f"{sys.executable} {REPO / 'tests' / 'fakessh.py'}", FAKESSH_ROOT=str(root),
               TK8S_SSH_CONNECT_RETRIES="0", TK8S_RCCL_POLL="0.05")
    env.pop("TK8S_FAKE_GPUS", None)
    r = subprocess.run(["./setup.sh", "--platform", "kubeadm", "--yes", "--json", "--nodes", "2", "--timeout", "60"],
                       cwd=ws, env=env, capture_output=True, text=True, timeout=300)
    try:
        assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-3000:]
        s = json.loads(r.stdout.strip().splitlines()[-1])
        assert s["platform"] == "kubeadm" and s["nodes"] == 2 and s["gpus_allocatable"] == 2
        assert s["rccl"]["ok"] and s["rccl"]["pods"] == 2 and s["rccl"]["platform"] == "kubeadm"
        assert s["api"] == f"https://{hosts['mi355x-a']}:6443"
        assert (ws / "ansible" / "tmp" / "kubeconfig").read_text().startswith("apiVersion: v1")
        assert (ws / "ansible" / "tmp" / "kubernetes_environment.id").read_text() == json.loads(state.read_text())["uid"]
        log_a = (root / hosts["mi355x-a"] / "sysroot" / "var" / "log" / "fake-tools.log").read_text()
        log_b = (root / hosts["mi355x-b"] / "sysroot" / "var" / "log" / "fake-tools.log").read_text()
        log_c = (root / hosts["mi355x-c"] / "sysroot" / "var" / "log" / "fake-tools.log").read_text()
        assert "kubeadm init --apiserver-advertise-address 127.0.7.30" in log_a
        assert "amdgpu-dkms" in log_b and "amdgpu-dkms" not in log_a  # the GPU driver on GPU hosts only
        for log in (log_b, log_c):  # every worker on its own host joined with the master's token
            assert log.count("kubeadm join 127.0.7.30:6443 --token abcdef.0123456789abcdef") == 1
        assert (root / hosts["mi355x-b"] / "sysroot" / "dev" / "kfd").exists()
        cfg = (root / hosts["mi355x-b"] / "sysroot" / "etc" / "containerd" / "config.toml").read_text()
        assert "SystemdCgroup = true" in cfg
        assert "# /swap.img none swap" in (root / hosts["mi355x-b"] / "sysroot" / "etc" / "fstab").read_text()
        assert (root / hosts["mi355x-b"] / "sysroot" / "etc" / "apt" / "sources.list.d" / "rocm.list").exists()
        nodes = json.loads(state.read_text())["nodes"]
        assert nodes["kubenode1"]["gpus"] + nodes["kubenode2"]["gpus"] == 2
        assert nodes["kubenode1"]["labels"]["amd.com/gpu.family"] == "gfx950"
        st = json.loads(subprocess.run(["./tk8s", "status", "--json"], cwd=ws, env=env, capture_output=True,
                                       text=True, timeout=60).stdout)
        assert st["cluster"]["nodes_ready"] == 3 and st["cluster"]["gpus_allocatable"] == 2, st
        k = subprocess.run(["./kubectl", "get", "nodes"], cwd=ws, env={**env, "PATH": "/usr/bin:/bin"},
                           capture_output=True, text=True, timeout=60)
        assert k.returncode == 1 and "KUBECONFIG=" in k.stderr and "ansible/tmp/kubeconfig" in k.stderr
        # shrink: kubenode2 is drained and deleted on the master, reset on its host, its machine destroyed
        sc = subprocess.run(["./tk8s", "scale", "1", "--json"], cwd=ws, env=env, capture_output=True, text=True,
                            timeout=300)
        assert sc.returncode == 0, sc.stdout[-3000:] + sc.stderr[-2000:]
        assert json.loads(sc.stdout.strip().splitlines()[-1])["nodes"] == 1
        assert "kubenode2" not in json.loads(state.read_text())["nodes"]
        gone = next(h for h in ("mi355x-b", "mi355x-c")
                    if not list((root / hosts[h]).glob("tk8s/machines/kubenode*")))
        assert "kubeadm reset -f" in (root / hosts[gone] / "sysroot" / "var" / "log" / "fake-tools.log").read_text()
    finally:
        c = subprocess.run(["./setup.sh", "-c", "--yes"], cwd=ws, env=env, capture_output=True, text=True, timeout=120)
    assert c.returncode == 0 and "kubeadm reset on kubenode1: ok" in c.stdout, c.stdout + c.stderr
    for h in ("mi355x-b", "mi355x-c"):
        assert not (root / hosts[h] / "sysroot" / "etc" / "kubernetes" / "kubelet.conf").exists()


def _kubeadm_env(tmp_path: Path, hosts: dict[str, tuple[str, int]], state: Path, scenario: dict | None = None):
    """A workspace, fake-root hosts ({name: (address, gpus)}) and the env to run ./setup.sh
    --backend baremetal --platform kubeadm against them."""
    import subprocess
    import sys

    from tritonk8ssupervisor_amd.orchestrator import init_workspace

    ws = tmp_path / "ws"
    ws.mkdir()
    init_workspace(ws)
    for f in ("setup.sh", "tk8s", "kubectl"):
        shutil.copy2(REPO / f, ws / f)
    gv = ws / "ansible" / "group_vars" / "all.yml"
    gv.write_text(gv.read_text().replace('tk8s_sysroot: ""', 'tk8s_sysroot: "{{ ansible_env.HOME }}/sysroot"'))
    keydir = tmp_path / "keys"
    keydir.mkdir()
    subprocess.run(["ssh-keygen", "-q", "-t", "ed25519", "-N", "", "-f", str(keydir / "id_ed25519")], check=True)
    root = tmp_path / "hosts"
    for addr, gpus in hosts.values():
        _fake_root_host(root, addr, (keydir / "id_ed25519.pub").read_text(), state, gpus=gpus)
    if scenario is not None:
        state.write_text(json.dumps({"nodes": {}, "objects": [], "uid": "", "master": "", "rccl_scenario": scenario}))
    inv = {"ssh": {"user": "root", "key": str(keydir / "id_ed25519")}, "python": sys.executable,
           "hosts": [{"name": n, "address": a, "gpus": g, **({"role": "master"} if i == 0 else {})}
                     for i, (n, (a, g)) in enumerate(hosts.items())]}
    (ws / "inventory.yml").write_text(json.dumps(inv))
    env = dict(os.environ, PYTHONPATH=str(REPO), TK8S_PYTHON=sys.executable, TK8S_BACKEND="baremetal",
               TK8S_SSH=f"{sys.executable} {REPO / 'tests' / 'fakessh.py'}", FAKESSH_ROOT=str(root),
               TK8S_SSH_CONNECT_RETRIES="0", TK8S_RCCL_POLL="0.05")
    env.pop("TK8S_FAKE_GPUS", None)
    return ws, root, env


def _fake_kubectl(host_dir: Path, state: Path, *args) -> "subprocess.CompletedProcess":
    import subprocess
    import sys

    env = dict(os.environ, TK8S_SYSROOT=str(host_dir / "sysroot"), FAKE_K8S_STATE=str(state), FAKETOOL_NAME="kubectl")
    return subprocess.run([sys.executable, str(REPO / "tests" / "fakeroot" / "faketool.py"), *args], env=env,
                          capture_output=True, text=True, timeout=60)


def test_kubeadm_single_node_on_one_8gpu_host(tmp_path):
    """./setup.sh --platform kubeadm with a ONE-host inventory (the 8x MI355X box):
    kubeadm init on that host, its control-plane taint removed, 8 amd.com/gpu on its one node, the
    8 workers are GPU slots of it; the RCCL-tests Job leaves every GPU schedulable; -c resets it."""
    import subprocess

    state = tmp_path / "cluster.json"
    ws, root, env = _kubeadm_env(tmp_path, {"mi355x": ("127.0.7.40", 8)}, state)
    r = subprocess.run(["./setup.sh", "--platform", "kubeadm", "--yes", "--json", "--nodes", "8", "--timeout", "60"],
                       cwd=ws, env=env, capture_output=True, text=True, timeout=300)
    host = root / "127.0.7.40"
    try:
        assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-3000:]
        s = json.loads(r.stdout.strip().splitlines()[-1])
        assert s["single_node"] is True and s["nodes"] == 8 and s["kubernetes_nodes"] == 1
        assert s["gpus_allocatable"] == 8 and s["nodes_validated"] == 1
        assert "ALL NODES READY: 1 node(s) (single-node: kubemaster is control plane and GPU worker, 8 worker slot(s)), " \
               "8 x amd.com/gpu allocatable" in r.stdout
        nodes = json.loads(state.read_text())["nodes"]
        assert list(nodes) == ["kubemaster"] and nodes["kubemaster"]["gpus"] == 8
        assert nodes["kubemaster"]["taints"] == [] and nodes["kubemaster"]["labels"]["amd.com/gpu.family"] == "gfx950"
        # the fabric check ran after Ready: one Job, one pod, all 8 GPUs, then the GPUs are free again
        assert s["rccl"]["ok"] and s["rccl"]["pods"] == 1 and s["rccl"]["nranks"] == 8 and s["rccl"]["gpus_per_pod"] == 8
        assert r.stdout.index("ALL NODES READY") < r.stdout.index("Running RCCL all-reduce on 1 GPU node(s)")
        assert s["rccl_check_s"] > 0 and s["ready_seconds"] < s["total_seconds"]
        pod = tmp_path / "gpu-pod.yaml"
        pod.write_text(yaml.safe_dump({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "hello-gpu"},
                                       "spec": {"containers": [{"name": "c", "image": "rocm/dev-ubuntu-22.04:7.2",
                                                                "resources": {"limits": {"amd.com/gpu": 1}}}]}}))
        assert _fake_kubectl(host, state, "apply", "-f", str(pod)).returncode == 0
        got = json.loads(_fake_kubectl(host, state, "get", "pod", "hello-gpu", "-o", "json").stdout)
        assert got["status"]["phase"] == "Running" and got["spec"]["nodeName"] == "kubemaster"
        # the reference's deliverables: dashboard URL + kubectl config
        assert s["dashboard"] == "https://127.0.7.40:30443/" and "Kubernetes dashboard is at https://127.0.7.40:30443/" in r.stdout
        assert (ws / "ansible" / "tmp" / "dashboard-token").read_text().startswith("eyJ")
        assert f"Kubernetes CLI config is at {ws / 'ansible' / 'tmp' / 'kubeconfig'}" in r.stdout
        log = (host / "sysroot" / "var" / "log" / "fake-tools.log").read_text()
        assert log.count("kubeadm init") == 1 and "kubeadm join" not in log
        # the node runtime went in once (play 1 on the master machine only), not once per GPU slot
        assert sum(ln.startswith("apt-get") and "amdgpu-dkms" in ln for ln in log.splitlines()) == 1, log
        assert "taint nodes kubemaster node-role.kubernetes.io/control-plane:NoSchedule-" in log
        # the GPU slots are machines of the one host, each with one of its GPUs
        alloc = json.loads((ws / ".tk8s" / "baremetal-alloc.json").read_text())["machines"]
        assert sorted(g for m, rec in alloc.items() if m != "kubemaster" for g in rec["gpus"]) == list(range(8))
    finally:
        c = subprocess.run(["./setup.sh", "-c", "--yes"], cwd=ws, env=env, capture_output=True, text=True, timeout=120)
    assert c.returncode == 0, c.stdout + c.stderr
    assert c.stdout.count("kubeadm reset on ") == 1 and "kubeadm reset on kubemaster: ok" in c.stdout
    assert not (host / "sysroot" / "etc" / "kubernetes" / "admin.conf").exists()


def test_rccl_job_verdict_states():
    """the wait needs exactly one successfully terminated pod per GPU node."""
    from tritonk8ssupervisor_amd.kubeadm_platform import rccl_job_verdict

    jobs = {"n1": "j-0", "n2": "j-1"}

    def pod(job, phase, code=None, name=None):
        st = {"phase": phase}
        if code is not None:
            st["containerStatuses"] = [{"state": {"terminated": {"exitCode": code, "reason": "Error" if code else "Completed"}}}]
        return {"metadata": {"name": name or f"{job}-x", "labels": {"job-name": job}}, "status": st}

    assert rccl_job_verdict([], jobs)["state"] == "waiting"  # no pods yet: still waiting
    v = rccl_job_verdict([pod("j-0", "Pending"), pod("j-1", "Pending")], jobs)
    assert v["state"] == "waiting" and "n1: pod j-0-x Pending" in v["reason"]
    assert rccl_job_verdict([pod("j-0", "Succeeded", 0)], jobs)["state"] == "waiting"  # n2 has none
    v = rccl_job_verdict([pod("j-0", "Succeeded", 0), pod("j-1", "Failed", 1)], jobs)
    assert v["state"] == "failed" and "n2: pod j-1-x failed (Error, exit code 1)" in v["reason"]
    v = rccl_job_verdict([pod("j-0", "Succeeded", 0), pod("j-1", "Succeeded", 0)], jobs)
    assert v["state"] == "done" and v["pods"] == {"n1": "j-0-x", "n2": "j-1-x"}
    v = rccl_job_verdict([pod("j-0", "Succeeded", 0), pod("j-0", "Running", name="j-0-y"), pod("j-1", "Succeeded", 0)], jobs)
    assert v["state"] == "failed" and "2 pods" in v["reason"]


def test_kubeadm_rccl_failure_fails_setup(tmp_path):
    """one node's RCCL pod failing fails ./setup.sh (exit != 0, with the reason), after
    the ALL NODES READY line -- and no Congratulations."""
    import subprocess

    state = tmp_path / "cluster.json"
    ws, root, env = _kubeadm_env(tmp_path, {"mi355x-a": ("127.0.7.50", 0), "mi355x-b": ("127.0.7.51", 1),
                                            "mi355x-c": ("127.0.7.52", 1)}, state,
                                 scenario={"pending_polls": 2, "fail": ["kubenode2"]})
    r = subprocess.run(["./setup.sh", "--platform", "kubeadm", "--yes", "--json", "--nodes", "2", "--timeout", "60"],
                       cwd=ws, env=env, capture_output=True, text=True, timeout=300)
    try:
        assert r.returncode == 2, r.stdout[-3000:] + r.stderr[-2000:]
        assert "ALL NODES READY: 2 node(s), 2 x amd.com/gpu allocatable" in r.stdout
        assert "RCCL all-reduce validation failed: kubenode2: pod" in r.stderr and "exit code 1" in r.stderr
        assert "Congratulations" not in r.stdout
    finally:
        subprocess.run(["./setup.sh", "-c", "--yes"], cwd=ws, env=env, capture_output=True, text=True, timeout=120)


def test_both_platforms_report_ready_and_rccl_alike():
    """'Ready' means the same on both platforms -- the summaries carry ready_seconds
    (to the ALL NODES READY line, before the fabric check) and rccl / rccl_check_s (after it)."""
    import inspect

    from tritonk8ssupervisor_amd import kubeadm_platform, orchestrator

    for src in (inspect.getsource(orchestrator.Setup.run), inspect.getsource(kubeadm_platform.KubeadmPlatform._kubeadm_finish)):
        for key in ('"ready_seconds"', '"rccl_check_s"', '"rccl"', '"total_seconds"'):
            assert key in src, key
    run = inspect.getsource(orchestrator.Setup.run)
    assert run.index("self.ready_line(") < run.index("self.run_rccl()") < run.index("_kubeadm_finish")
    # the kubeadm playbook's last play waits for nodes + GPUs only; no RCCL object is created in it
    role = (REPO / "ansible" / "roles" / "kubeadmvalidate" / "tasks" / "main.yml").read_text()
    assert "rccl-tests" not in role.split("\n- name:", 1)[1].lower().replace("rccl-tests select", "")


def test_kubeadm_single_node_as_root_on_this_host(tmp_path, monkeypatch):
    """the natural command on the north-star box -- ``./setup.sh --platform
    kubeadm --nodes 8`` as root with the default (local) backend -- runs the kubeadm roles on THIS
    host through a one-host inventory reached without ssh (``connection: local``): kubeadm init,
    the control-plane taint removed, 8 x amd.com/gpu on the one node; ``-c`` resets it. The host
    here is a fake root (its apt-get/kubeadm/kubectl/systemctl are tests/fakeroot stand-ins, its
    system paths under a staging root), the same simulation the ssh tests use."""
    import subprocess
    import sys

    from tritonk8ssupervisor_amd.orchestrator import init_workspace

    state = tmp_path / "cluster.json"
    ws = tmp_path / "ws"
    ws.mkdir()
    init_workspace(ws)
    for f in ("setup.sh", "tk8s", "kubectl"):
        shutil.copy2(REPO / f, ws / f)
    gv = ws / "ansible" / "group_vars" / "all.yml"
    gv.write_text(gv.read_text().replace('tk8s_sysroot: ""', 'tk8s_sysroot: "{{ ansible_env.HOME }}/sysroot"'))
    host = _fake_root_host(tmp_path / "hosts", "this-host", "", state, gpus=8)
    (host / ".ssh" / "authorized_keys").unlink()  # no ssh involved at all
    env = dict(os.environ, PYTHONPATH=str(REPO), TK8S_PYTHON=sys.executable, TK8S_LOCAL_HOST_ROOT=str(host),
               TK8S_LOCAL_HOST_GPUS="8", TK8S_SSH="false", TK8S_RCCL_POLL="0.05")
    for k in ("TK8S_FAKE_GPUS", "TK8S_BACKEND", "TK8S_INVENTORY"):
        env.pop(k, None)
    r = subprocess.run(["./setup.sh", "--platform", "kubeadm", "--yes", "--json", "--nodes", "8", "--timeout", "60"],
                       cwd=ws, env=env, capture_output=True, text=True, timeout=300)
    try:
        assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-3000:]
        s = json.loads(r.stdout.strip().splitlines()[-1])
        assert s["single_node"] is True and s["nodes"] == 8 and s["kubernetes_nodes"] == 1
        assert s["gpus_allocatable"] == 8 and s["rccl"]["ok"]
        inv = json.loads((ws / ".tk8s" / "local-host-inventory.json").read_text())
        assert inv["hosts"][0]["connection"] == "local" and inv["hosts"][0]["gpus"] == 8
        assert "TK8S_BACKEND=baremetal" in (ws / "config").read_text()
        assert "ansible_connection=local" in (ws / "ansible" / "hosts").read_text()
        log = (host / "sysroot" / "var" / "log" / "fake-tools.log").read_text()
        assert log.count("kubeadm init") == 1 and "kubeadm join" not in log
        assert "taint nodes" in log and "NoSchedule-" in log
        nodes = json.loads(state.read_text())["nodes"]
        assert len(nodes) == 1 and next(iter(nodes.values()))["gpus"] == 8
    finally:
        c = subprocess.run(["./setup.sh", "-c", "--yes"], cwd=ws, env=env, capture_output=True, text=True, timeout=120)
    assert c.returncode == 0, c.stdout + c.stderr
    assert "kubeadm reset on" in c.stdout and ": ok" in c.stdout
    assert not (host / "sysroot" / "etc" / "kubernetes" / "admin.conf").exists()


def test_kubeadm_refused_on_this_host_without_root(tmp_path, monkeypatch):
    from tritonk8ssupervisor_amd.orchestrator import Setup, SetupError, init_workspace

    monkeypatch.setattr(os, "geteuid", lambda: 1000)
    monkeypatch.delenv("TK8S_LOCAL_HOST_ROOT", raising=False)
    monkeypatch.setenv("TK8S_FAKE_GPUS", "2")
    ws = init_workspace(tmp_path)
    s = Setup(ws, answers={"nodes": 1}, assume_yes=True, platform="kubeadm", out=lambda _l: None)
    with pytest.raises(SetupError, match="as root"):
        s.configure()


GOLDEN_LOCAL = REPO / "tests" / "golden" / "kubeadm_check_local_root.txt"


def test_kubeadm_as_root_on_this_host_check_plan(tmp_path):
    """``./setup.sh --platform kubeadm --nodes 8 --dry-run`` as root on this host
    (simulated root): the Terraform plan (1 master machine = the host, 8 GPU slots) and the kubeadm
    playbook in check mode, task by task, pinned by a golden file (TK8S_REGOLDEN=1 rewrites it)."""
    import subprocess
    import sys

    from tritonk8ssupervisor_amd.orchestrator import init_workspace

    ws = tmp_path / "ws"
    ws.mkdir()
    init_workspace(ws)
    for f in ("setup.sh", "tk8s", "kubectl"):
        shutil.copy2(REPO / f, ws / f)
    host = _fake_root_host(tmp_path / "hosts", "this-host", "", tmp_path / "cluster.json", gpus=8)
    env = dict(os.environ, PYTHONPATH=str(REPO), TK8S_PYTHON=sys.executable, TK8S_LOCAL_HOST_ROOT=str(host),
               TK8S_LOCAL_HOST_GPUS="8", TK8S_SSH="false")
    for k in ("TK8S_FAKE_GPUS", "TK8S_BACKEND", "TK8S_INVENTORY"):
        env.pop(k, None)
    r = subprocess.run(["./setup.sh", "--platform", "kubeadm", "--yes", "--json", "--nodes", "8", "--dry-run"],
                       cwd=ws, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-3000:]
    s = json.loads(r.stdout.strip().splitlines()[-1])
    assert s["dry_run"] and s["platform"] == "kubeadm" and s["backend"] == "baremetal" and s["check_ok"]
    assert len(s["plan"]) == 9 and all(p["action"] == "create" for p in s["plan"])
    plan = s["check_plan"]
    if os.environ.get("TK8S_REGOLDEN") == "1":
        GOLDEN_LOCAL.write_text("\n".join(plan) + "\n")
    assert plan == GOLDEN_LOCAL.read_text().splitlines()
    assert {ln.split(":", 1)[0] for ln in plan} == {"kubemaster"}  # the GPU slots run nothing
    assert "kubemaster: kubeadm init (etcd, kube-apiserver, kube-scheduler, kube-controller-manager)" in plan
    assert not (ws / "config").exists() and not (ws / "terraform" / "rancher.tf").exists()  # nothing written
