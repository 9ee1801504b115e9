"""End-to-end bring-up on the CPU box: ``./setup.sh`` -> all nodes Ready -> ``./setup.sh -c``.

The local provider runs every machine as a sandbox + process group on this host; the GPU
inventory is faked (TK8S_FAKE_GPUS=8 virtual gfx950 devices) so the allocation, validation
and RCCL-job paths run without a GPU (BASELINE.json configs 1-2).
"""
import json
import os
import shutil
import subprocess
import sys
import time
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
pytestmark = pytest.mark.slow


@pytest.fixture
def ws(tmp_path):
    from tritonk8ssupervisor_amd.orchestrator import init_workspace

    init_workspace(tmp_path)
    for f in ("setup.sh", "tk8s", "kubectl"):
        shutil.copy2(REPO / f, tmp_path / f)
    yield tmp_path
    # never leave processes behind, whatever the test did
    subprocess.run(["./setup.sh", "-c", "--yes"], cwd=tmp_path, env=_env(), capture_output=True, timeout=120)


def _env(**kw):
    env = dict(os.environ)
    env["PYTHONPATH"] = str(REPO)
    env["TK8S_PYTHON"] = sys.executable
    env["TK8S_FAKE_GPUS"] = "8"
    env.pop("TK8S_FAULTS", None)
    env.update({k: str(v) for k, v in kw.items()})
    return env


def _setup(ws, *args, env=None, timeout=180):
    return subprocess.run(["./setup.sh", "--yes", "--json", "--port", "0", *args], cwd=ws, env=env or _env(),
                          capture_output=True, text=True, timeout=timeout)


def _summary(r):
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def _pids(ws):
    out = []
    for pf in [*(ws / ".tk8s" / "machines").glob("*/run/agent.pid"), *(ws / ".tk8s" / "machines").glob("*/run/controlplane.pid")]:
        try:
            out.append(int(json.loads(pf.read_text())["pid"]))
        except (ValueError, KeyError, OSError):
            pass
    return out


def _alive(pid):
    try:
        os.kill(pid, 0)
    except OSError:
        return False
    try:  # zombies count as gone
        with open(f"/proc/{pid}/stat") as f:
            return f.read().split(") ", 1)[1][0] != "Z"
    except OSError:
        return False


@pytest.mark.parametrize("n", [1, 2, 4, 8])
def test_setup_ready_and_clean_teardown(ws, n):
    t = time.monotonic()
    s = _summary(_setup(ws, "--nodes", str(n)))
    wall = time.monotonic() - t
    assert s["nodes"] == n and s["gpus_allocatable"] == n and s["nodes_validated"] == n
    if n >= 2:  # the RCCL fabric check ran across all GPUs, one rank per GPU
        rc = s["rccl"]
        assert rc["ok"] and rc["nranks"] == n
        # every worker is a one-GPU slice of this one host: ONE pod, ONE process driving all n GPUs
        # as ranks 0..n-1, its GPUs claimed on every node of the host meanwhile
        assert rc["pods"] == 1 and rc["gpus_per_pod"] == n and rc["scope"] == "host", rc
        r = subprocess.run(["./kubectl", "get", "pods", "-n", "kube-system", "-l", f"job-name={rc['job']}", "-o",
                            "json"], cwd=ws, env=_env(), capture_output=True, text=True)
        (pod,) = json.loads(r.stdout)["items"]
        res = pod["status"]["result"]
        assert (res["first_rank"], res["local_ranks"], res["nranks"]) == (0, n, n), res
        claims = json.loads(pod["metadata"]["annotations"]["tk8s.amd.com/host-claims"])
        assert claims == {f"kubenode{i}": 1 for i in range(1, n + 1)}
    assert wall < 60  # the reference's fixed sleeps alone are 51 s
    # reference artefacts exist, with reference names
    for rel in ("config", "terraform/rancher.tf", "terraform/masters.ip", "terraform/hosts.ip", "ansible/hosts",
                "ansible/roles/ranchermaster/vars/vars.yml", "ansible/tmp/kubernetes_environment.id"):
        assert (ws / rel).exists(), rel
    assert len((ws / "terraform" / "hosts.ip").read_text().split()) == n
    cfg = (ws / "config").read_text()
    assert f"KUBERNETES_NUMBER_OF_NODES={n}" in cfg and "ANSIBLE_HOST_KEY_CHECKING=False" in cfg
    # kubectl sees every node Ready with its GPU
    r = subprocess.run(["./kubectl", "get", "nodes", "-o", "json"], cwd=ws, env=_env(), capture_output=True, text=True)
    items = json.loads(r.stdout)["items"]
    assert sorted(i["metadata"]["name"] for i in items) == [f"kubenode{i}" for i in range(1, n + 1)]
    assert all(i["status"]["allocatable"]["amd.com/gpu"] == "1" for i in items)
    # the validation pods' results (shared from the host burn-in for n >= 2) reach the nodes
    assert all(i["metadata"]["annotations"].get("tk8s.amd.com/hbm-write-gbps") == "6200.0" for i in items)
    # distinct GPUs per worker
    ids = [i["status"]["devices"][0]["id"] for i in items]
    assert len(set(ids)) == n
    pids = _pids(ws)
    assert len(pids) == n + 1 and all(_alive(p) for p in pids)
    # the early GPU burn-in ran on every worker and the validation pods reused its result
    for i in range(1, n + 1):
        burn = json.loads((ws / ".tk8s" / "machines" / f"kubenode{i}" / "run" / "gpu-burnin.json.consumed").read_text())
        assert burn["ok"] and burn["probed"] == 1
        # one host-level burn-in (the runtime starts once, before the machines exist), split per machine
        assert burn["host_burnin"] and burn["devices"][0]["host_index"] == int(items[i - 1]["status"]["devices"][0]["id"][3:])
    # teardown: machines gone, every artefact removed -- including the env-id file the
    # reference never cleans (setup.sh:513 removes ./tmp/* instead of ansible/tmp/*)
    (ws / "ansible" / "tmp" / ".keep").touch()  # the repository's tracked placeholder
    r = subprocess.run(["./setup.sh", "-c", "--yes"], cwd=ws, env=_env(), capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "All clear!" in r.stdout
    for rel in ("config", "terraform/rancher.tf", "terraform/masters.ip", "terraform/hosts.ip", "terraform/terraform.tfstate",
                "ansible/hosts", "ansible/roles/ranchermaster/vars/vars.yml", "ansible/tmp/kubernetes_environment.id",
                "terraform/.terraform"):
        assert not (ws / rel).exists(), rel
    assert (ws / "ansible" / "ansible.cfg").read_text().count("private_key_file = \n") == 1
    assert (ws / "ansible" / "tmp" / ".keep").exists()  # tracked placeholder survives the teardown
    deadline = time.monotonic() + 10
    while any(_alive(p) for p in pids) and time.monotonic() < deadline:
        time.sleep(0.05)
    assert not any(_alive(p) for p in pids)


def test_refuses_to_run_over_a_previous_configuration(ws):
    _summary(_setup(ws, "--nodes", "1"))
    r = _setup(ws, "--nodes", "1")
    assert r.returncode != 0 and "./setup.sh -c" in (r.stdout + r.stderr)


def test_clean_without_confirmation_keeps_everything(ws):
    _summary(_setup(ws, "--nodes", "1"))
    r = subprocess.run(["./setup.sh", "-c"], cwd=ws, env=_env(), input="no\n", capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "WARNING: You are about to destroy" in r.stdout
    assert (ws / "config").exists() and (ws / "terraform" / "rancher.tf").exists()


def test_interactive_prompts_via_stdin(ws):
    # 8 prompts (all defaults except 2 nodes) + yes
    answers = "\n".join(["", "", "", "", "2", "", "", "", "yes"]) + "\n"
    r = subprocess.run(["./setup.sh", "--json", "--port", "0"], cwd=ws, env=_env(), input=answers,
                       capture_output=True, text=True, timeout=180)
    s = _summary(r)
    assert s["nodes"] == 2
    assert "Verify that the following configuration is correct" in r.stdout


def test_no_at_confirmation_exits_zero_and_creates_nothing(ws):
    answers = "\n" * 8 + "no\n"
    r = subprocess.run(["./setup.sh"], cwd=ws, env=_env(), input=answers, capture_output=True, text=True, timeout=60)
    assert r.returncode == 0
    assert not (ws / "terraform" / "rancher.tf").exists()


def test_agent_crash_mid_join_is_restarted(ws):
    # fault injection: kubenode1's agent dies right after registering, once; the supervisor
    # (tk8s-supervise, restart unless-stopped) brings it back and the cluster still converges
    s = _summary(_setup(ws, "--nodes", "2", "--rccl", "off", env=_env(TK8S_FAULTS="agent.crash@kubenode1:1")))
    assert s["nodes_validated"] == 2
    assert (ws / ".tk8s" / "machines" / "kubenode1" / "run" / "crash.count").read_text() == "1"


def test_validation_failure_fails_setup_fast(ws):
    t = time.monotonic()
    r = _setup(ws, "--nodes", "2", env=_env(TK8S_FAKE_PROBE_FAIL="kubenode2"))
    assert r.returncode == 2 and "GPU validation failed" in r.stderr
    assert time.monotonic() - t < 60


def test_crashed_burnin_falls_back_to_probing_in_the_pod(ws):
    t = time.monotonic()
    s = _summary(_setup(ws, "--nodes", "2", "--rccl", "off", env=_env(TK8S_FAKE_BURNIN_CRASH="kubenode2")))
    assert s["nodes_validated"] == 2 and time.monotonic() - t < 30  # no 120 s --reuse wait
    assert not (ws / ".tk8s" / "machines" / "kubenode2" / "run" / "gpu-burnin.json.consumed").exists()
    assert (ws / ".tk8s" / "machines" / "kubenode1" / "run" / "gpu-burnin.json.consumed").exists()


def test_stalled_node_hits_the_bounded_timeout(ws):
    # the reference's readiness loop has no timeout (setup.sh:59-85); ours exits 124
    t = time.monotonic()
    r = _setup(ws, "--nodes", "1", "--timeout", "3", env=_env(TK8S_FAKE_PROBE_HANG="kubenode1"))
    assert r.returncode == 124 and "not ready after" in r.stderr
    assert time.monotonic() - t < 60


def test_lost_heartbeats_mark_node_not_ready(ws):
    _summary(_setup(ws, "--nodes", "2", "--rccl", "off", "--node-grace", "0.5"))
    # stop kubenode2's agent (and its supervisor): the lease expires and the node goes NotReady
    from tritonk8ssupervisor_amd.utils.procs import kill_pidfile

    assert kill_pidfile(ws / ".tk8s" / "machines" / "kubenode2" / "run" / "agent.pid")
    deadline = time.monotonic() + 10
    while time.monotonic() < deadline:
        r = subprocess.run(["./kubectl", "get", "nodes"], cwd=ws, env=_env(), capture_output=True, text=True)
        if "NotReady" in r.stdout:
            break
        time.sleep(0.1)
    line = next(l for l in r.stdout.splitlines() if l.startswith("kubenode2"))
    assert "NotReady" in line


def test_provision_failure_then_resume(ws):
    r = _setup(ws, "--nodes", "2", env=_env(TK8S_FAKE_GPUS=1))
    assert r.returncode != 0 and "provisioning limit" in r.stdout
    st = json.loads((ws / ".tk8s" / "state.json").read_text())
    assert "provision" not in st["completed"]
    s = _summary(_setup(ws, "--resume", "--rccl", "off"))
    assert s["nodes"] == 2 and s["gpus_allocatable"] == 2
    st = json.loads((ws / ".tk8s" / "state.json").read_text())
    assert set(st["completed"]) >= {"configure", "provision", "ansible-config", "ansible", "ready"}


def test_status_and_events_log(ws):
    _summary(_setup(ws, "--nodes", "2", "--rccl", "off"))
    dv = subprocess.run(["./tk8s", "debug-vars"], cwd=ws, env=_env(), capture_output=True, text=True).stdout
    assert "KUBERNETES_NUMBER_OF_NODES=2" in dv and dv.splitlines()[0].startswith("KUBERNETES_NAME=")
    r = subprocess.run(["./tk8s", "status", "--json"], cwd=ws, env=_env(), capture_output=True, text=True)
    st = json.loads(r.stdout)
    assert st["cluster"]["nodes_ready"] == 2 and st["cluster"]["gpus_allocatable"] == 2
    assert set(st["timings"]) >= {"provision", "ansible", "ready"}
    from tritonk8ssupervisor_amd.utils.events import read_events

    evs = read_events(ws / ".tk8s" / "events.jsonl")
    names = [e["event"] for e in evs]
    assert "setup_start" in names and "setup_done" in names and names.count("machine_created") == 3


def test_kubectl_workload_on_the_cluster(ws, tmp_path_factory):
    _summary(_setup(ws, "--nodes", "2", "--rccl", "off"))
    d = tmp_path_factory.mktemp("m")
    (d / "job.yaml").write_text(
        "apiVersion: batch/v1\nkind: Job\nmetadata:\n  name: hello\nspec:\n  completions: 2\n  parallelism: 2\n"
        "  completionMode: Indexed\n  template:\n    spec:\n      restartPolicy: Never\n      containers:\n"
        "        - name: c\n          command: [\"sh\", \"-c\", \"echo rank=$JOB_COMPLETION_INDEX gpus=$ROCR_VISIBLE_DEVICES\"]\n"
        "          resources:\n            limits:\n              amd.com/gpu: 1\n")
    kc = lambda *a: subprocess.run(["./kubectl", *a], cwd=ws, env=_env(), capture_output=True, text=True, timeout=60)
    r = kc("apply", "-f", str(d / "job.yaml"))
    assert r.returncode == 0, r.stderr
    r = kc("wait", "job/hello", "--timeout", "30")
    assert r.returncode == 0, r.stdout + r.stderr
    pods = json.loads(kc("get", "pods", "-l", "job-name=hello", "-o", "json").stdout)["items"]
    assert len(pods) == 2 and all(p["status"]["phase"] == "Succeeded" for p in pods)
    logs = [kc("logs", p["metadata"]["name"]).stdout.strip() for p in pods]
    assert sorted(l.split()[0] for l in logs) == ["rank=0", "rank=1"]
    vis = {l.split("gpus=")[1] for l in logs}
    assert len(vis) == 2  # each rank saw exactly its own GPU
    r = kc("describe", "node", "kubenode1")
    assert "amd.com/gpu" in r.stdout


def test_manual_flow(ws):
    """docs/manual-setup.md, command for command: tk8s env/networks/packages, a hand-written
    rancher.tf, tk8s terraform get/plan/apply, hand-written inventory + vars, tk8s
    ansible-playbook (--check, then for real), kubectl with the served kubeconfig."""
    import urllib.error
    import urllib.request

    env = _env()
    sh = lambda *a, **kw: subprocess.run(list(a), cwd=ws, env=env, capture_output=True, text=True, timeout=120, **kw)
    exports = sh("./tk8s", "env").stdout
    assert "SDC_KEY_ID" in exports
    pub = next(l.split()[1] for l in sh("./tk8s", "networks").stdout.splitlines() if l.startswith("local-public"))
    pkg = next(l.split()[1] for l in sh("./tk8s", "packages").stdout.splitlines() if l.startswith("mi355x-1gpu"))
    key = ws / ".tk8s" / "keys" / "tk8s_cluster_key"
    mods = "".join(f'\nmodule "{n}" {{\n    source = "{src}"\n    hostname = "{n}"\n    networks = ["{pub}"]\n'
                   f'    root_authorized_keys = "${{file("{key}.pub")}}"\n    package = "{pkg}"\n}}\n'
                   for n, src in (("kubemaster", "master"), ("kubenode1", "host")))
    (ws / "terraform" / "rancher.tf").write_text(
        f'provider "local" {{\n    account = "root"\n    key_material = "${{file("{key}")}}"\n    key_id = "x"\n'
        f'    url = "local://h"\n}}\n' + mods)
    assert sh("./tk8s", "terraform", "get").returncode == 0
    assert "Plan: 2 to add" in sh("./tk8s", "terraform", "plan").stdout
    assert sh("./tk8s", "terraform", "apply").returncode == 0
    m_ip = (ws / "terraform" / "masters.ip").read_text().split()[0]
    h_ip = (ws / "terraform" / "hosts.ip").read_text().split()[0]
    (ws / "ansible" / "hosts").write_text(f"[MASTER]\nkubemaster ansible_host={m_ip}\n[HOST]\nkubenode1 ansible_host={h_ip}\n")
    (ws / "ansible" / "roles" / "ranchermaster" / "vars" / "vars.yml").write_text(
        f"master: {m_ip}\nkubernetes_name: manual\nkubernetes_description: manual\n")
    port = __import__("tritonk8ssupervisor_amd.orchestrator", fromlist=["_free_port"])._free_port()
    (ws / "config").write_text(f'RANCHER_MASTER_HOSTNAME="kubemaster"\nTK8S_MASTER_PORT={port}\n')
    r = sh("./tk8s", "ansible-playbook", "--check", "-i", "hosts", "clusterUp.yml")
    assert r.returncode == 0, r.stdout[-2000:]
    assert not (ws / "ansible" / "tmp" / "kubernetes_environment.id").exists()
    r = sh("./tk8s", "ansible-playbook", "-i", "hosts", "clusterUp.yml")
    assert r.returncode == 0, r.stdout[-2000:]
    env_id = (ws / "ansible" / "tmp" / "kubernetes_environment.id").read_text().strip()
    base = f"http://{m_ip}:{port}"
    # the control plane's admin token, as ranchermaster kept it (controlplane/authn.py)
    auth = {"Authorization": "Bearer " + (ws / ".tk8s" / "admin-token").read_text().strip()}
    with pytest.raises(urllib.error.HTTPError) as ei:  # nothing but health and discovery without it
        urllib.request.urlopen(f"{base}/env/{env_id}/kubernetes/kubectl?format=json")
    assert ei.value.code == 401
    w = json.loads(urllib.request.urlopen(urllib.request.Request(
        f"{base}/v1/cluster/wait?project={env_id}&nodes=1&gpus=1&timeout=30", headers=auth), timeout=40).read())
    assert w["ready"], w
    (ws / "kc.json").write_bytes(urllib.request.urlopen(urllib.request.Request(
        f"{base}/env/{env_id}/kubernetes/kubectl?format=json", headers=auth)).read())
    out = sh("./kubectl", "--kubeconfig", "kc.json", "get", "nodes").stdout
    assert "kubenode1" in out and "Ready" in out


def test_rerunning_the_playbook_is_idempotent(ws):
    """Re-running clusterUp.yml on a live cluster changes nothing: the control plane and the
    agents keep running, no second environment and no second node registration appear."""
    s = _summary(_setup(ws, "--nodes", "2", "--rccl", "off"))
    pids = sorted(_pids(ws))
    r = subprocess.run(["./tk8s", "ansible-playbook", "-i", "hosts", "clusterUp.yml"], cwd=ws, env=_env(),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-2000:]
    assert sorted(_pids(ws)) == pids
    assert (ws / "ansible" / "tmp" / "kubernetes_environment.id").read_text().strip() == s["project"]
    out = subprocess.run(["./kubectl", "get", "nodes", "-o", "json"], cwd=ws, env=_env(), capture_output=True, text=True)
    assert len(json.loads(out.stdout)["items"]) == 2


def test_guestbook_loadbalancer_service(ws):
    """docs/detailed.md acceptance demo: a Deployment behind a LoadBalancer Service, reached
    through the external IP and through the ClusterIP, round-robin over both replicas."""
    import urllib.request

    _summary(_setup(ws, "--nodes", "2", "--rccl", "off"))
    kc = lambda *a: subprocess.run(["./kubectl", *a], cwd=ws, env=_env(), capture_output=True, text=True, timeout=60)
    r = kc("apply", "-f", str(REPO / "manifests" / "examples" / "guestbook.yaml"))
    assert r.returncode == 0, r.stderr
    svc = json.loads(kc("get", "svc", "frontend", "-o", "json").stdout)
    ext = svc["status"]["loadBalancer"]["ingress"][0]["ip"]
    cip = svc["spec"]["clusterIP"]
    assert cip.startswith("127.96.") and svc["spec"]["ports"][0]["nodePort"] >= 30000
    assert "LoadBalancer" in kc("get", "svc").stdout
    deadline = time.monotonic() + 30
    seen = set()
    while time.monotonic() < deadline and len(seen) < 2:
        try:
            body = urllib.request.urlopen(f"http://{ext}:8000/", timeout=5).read().decode()
            seen.add(body.split()[2])
        except OSError:
            time.sleep(0.1)
    assert len(seen) == 2, seen  # both replicas answered
    assert urllib.request.urlopen(f"http://{cip}:8000/", timeout=5).read().decode().startswith("guestbook frontend")
    pods = json.loads(kc("get", "pods", "-l", "app=guestbook", "-o", "json").stdout)["items"]
    ips = {p["status"]["podIP"] for p in pods}
    assert len(ips) == 2 and all(ip.startswith("127.1") for ip in ips)
    assert kc("delete", "-f", str(REPO / "manifests" / "examples" / "guestbook.yaml")).returncode == 0
    time.sleep(0.3)
    with pytest.raises(OSError):
        urllib.request.urlopen(f"http://{ext}:8000/", timeout=2).read()


def test_ecc_errors_take_a_gpu_out_of_allocatable(ws, tmp_path_factory):
    """AMD SMI health (tk8s-smi; here its fake twin): a GPU reporting uncorrectable ECC errors
    goes Unhealthy and leaves allocatable; it comes back when the errors clear."""
    faults = tmp_path_factory.mktemp("smi") / "ue"
    faults.write_text("")
    env = _env(TK8S_SMI_DELAY="0.05", TK8S_SMI_INTERVAL="0.1", TK8S_FAKE_SMI_FILE=faults)
    s = _summary(_setup(ws, "--nodes", "2", "--rccl", "off", env=env))
    assert s["gpus_allocatable"] == 2
    kc = lambda *a: subprocess.run(["./kubectl", *a], cwd=ws, env=env, capture_output=True, text=True, timeout=60)

    def node(name):
        return json.loads(kc("get", "node", name, "-o", "json").stdout)

    def wait_for(pred, what):
        deadline = time.monotonic() + 15
        while time.monotonic() < deadline:
            n = node("kubenode2")
            if pred(n):
                return n
            time.sleep(0.05)
        raise AssertionError(f"timed out waiting for {what}: {json.dumps(n)[:2000]}")

    n = wait_for(lambda n: n["metadata"].get("annotations", {}).get("amd.com/gpu-health-source") == "amdsmi",
                 "first AMD SMI sample")
    gpu = n["status"]["devices"][0]
    host_ordinal = gpu["ordinal"]
    assert gpu["health"] == "Healthy" and "telemetry" in gpu and gpu["pciBusId"]
    faults.write_text(f"{host_ordinal}:2")
    n = wait_for(lambda n: n["status"]["allocatable"].get("amd.com/gpu") == "0", "ECC -> Unhealthy")
    assert n["status"]["devices"][0]["health"] == "Unhealthy"
    assert n["status"]["devices"][0]["reason"].startswith("ECC: 2 uncorrectable")
    assert node("kubenode1")["status"]["allocatable"]["amd.com/gpu"] == "1"  # the other GPU is untouched
    assert "ECC: 2 uncorrectable" in kc("describe", "node", "kubenode2").stdout
    faults.write_text("")
    wait_for(lambda n: n["status"]["allocatable"].get("amd.com/gpu") == "1", "errors cleared -> Healthy")


def test_setup_with_the_kubelet_grpc_device_plugin(ws):
    """TK8S_DEVICE_PLUGIN=grpc: every agent serves the amd.com/gpu plugin on the kubelet
    device-plugin API (v1beta1, Unix sockets) and allocates through it; the RCCL Job's ranks get
    their GPUs from gRPC Allocate and see the node (tk8s.amd.com/gpu-visibility: node)."""
    s = _summary(_setup(ws, "--nodes", "2", env=_env(TK8S_DEVICE_PLUGIN="grpc")))
    assert s["gpus_allocatable"] == 2 and s["nodes_validated"] == 2 and s["rccl"]["ok"]
    for i in (1, 2):
        log = (ws / ".tk8s" / "machines" / f"kubenode{i}" / "logs" / "agent.log").read_text()
        assert "via gRPC v1beta1" in log and "registered with the kubelet" in log


def test_pod_gpu_env_visibility_modes():
    from tritonk8ssupervisor_amd.agent.agent import pod_gpu_env

    alloc = {"ROCR_VISIBLE_DEVICES": "5", "HIP_VISIBLE_DEVICES": "0", "CUDA_VISIBLE_DEVICES": "0"}
    assert pod_gpu_env(alloc, [5]) == alloc
    node = pod_gpu_env(alloc, [5, 6], "node")
    assert node == {"TK8S_GPU_DEVICES": "5,6", "TK8S_GPU_DEVICE": "5"}


def test_host_burnin_split_per_machine():
    from tritonk8ssupervisor_amd.burnin import split_host_result

    res = {"ok": False, "md5_expected": "x", "timings_ms": {"hip_init": 50.0},
           "devices": [{"device": i, "ok": i != 2, "hbm": {"gbps": 6000.0 + i}} for i in range(3)],
           "gpuinfo": {"ok": True, "devices": [{"index": i, "pci_bus_id": f"0000:{i:02x}:00.0"} for i in range(3)],
                       "links": [[{"type": "self" if a == b else "xgmi", "ab": (a, b)} for b in range(3)] for a in range(3)]}}
    gpus = [1, 4, 6]  # host indices the burn-in process saw as its devices 0, 1, 2
    one = split_host_result(res, gpus, [4])
    assert one["ok"] and one["probed"] == 1 and one["devices"][0]["host_index"] == 4 and one["devices"][0]["device"] == 0
    assert one["hbm"]["gbps"] == 6001.0 and one["gpuinfo"]["devices"][0]["pci_bus_id"] == "0000:01:00.0"
    assert one["gpuinfo"]["links"] == [[{"type": "self", "ab": (1, 1)}]] and one["host_burnin"]
    two = split_host_result(res, gpus, [6, 1])
    assert not two["ok"] and [d["host_index"] for d in two["devices"]] == [6, 1]
    assert two["gpuinfo"]["links"][0][1]["ab"] == (2, 0)
    assert split_host_result(res, gpus, [5]) is None and split_host_result({}, gpus, [1]) is None
    # a failed pull from another machine's GPU does not fail this machine; one inside it does
    res["devices"][0].update(ok=False, peers=[{"src_device": 1, "dst_device": 0, "ok": False}])
    assert split_host_result(res, gpus, [1])["ok"]
    assert split_host_result(res, gpus, [1])["devices"][0]["host_peers"][0]["ok"] is False
    assert not split_host_result(res, gpus, [1, 4])["ok"]


def test_failed_host_burnin_falls_back_to_per_machine_probes(ws):
    """The shared (host-level) burn-in fails as a whole: no machine gets a share, every
    validation pod probes its own GPU, and the bring-up still completes validated."""
    s = _summary(_setup(ws, "--nodes", "2", "--rccl", "off", env=_env(TK8S_FAKE_PROBE_FAIL="host")))
    assert s["nodes_validated"] == 2 and s["gpus_allocatable"] == 2
    for i in (1, 2):  # no shared result; at most the machine's own burn-in (rocmsetup) ran
        f = ws / ".tk8s" / "machines" / f"kubenode{i}" / "run" / "gpu-burnin.json.consumed"
        assert not f.exists() or not json.loads(f.read_text()).get("host_burnin")
    events = (ws / ".tk8s" / "events.jsonl").read_text()
    assert "gpu_burnin_share_failed" in events and "gpu_burnin_host_done" in events


def test_two_gpu_workers_share_one_host_burnin(ws):
    """mi355x-2gpu workers: one burn-in over all 4 GPUs, each machine gets exactly its two
    (renumbered as it sees them), and every node advertises 2 validated amd.com/gpu."""
    s = _summary(_setup(ws, "--nodes", "2", "--package", "mi355x-2gpu", "--rccl", "off"))
    assert s["gpus_allocatable"] == 4 and s["nodes_validated"] == 2
    seen = []
    for i in (1, 2):
        m = json.loads((ws / ".tk8s" / "machines" / f"kubenode{i}" / "machine.json").read_text())
        burn = json.loads((ws / ".tk8s" / "machines" / f"kubenode{i}" / "run" / "gpu-burnin.json.consumed").read_text())
        assert burn["host_burnin"] and burn["probed"] == 2
        assert [d["host_index"] for d in burn["devices"]] == m["gpus"] and [d["device"] for d in burn["devices"]] == [0, 1]
        seen += m["gpus"]
    assert sorted(seen) == [0, 1, 2, 3]


def test_answers_file_bring_up_starts_the_burnin_before_the_cli_imports(ws):
    """``./setup.sh --answers FILE``: the burn-in is spawned first thing (earlyburn.py) and the
    orchestrator adopts it; the workers get its GPUs and reuse its result."""
    (ws / "answers.json").write_text(json.dumps({"nodes": 2, "package": "mi355x-1gpu", "confirm": "yes"}))
    s = _summary(_setup(ws, "--answers", "answers.json", "--rccl", "off"))
    assert s["nodes_validated"] == 2 and s["gpus_allocatable"] == 2
    events = [json.loads(line) for line in (ws / ".tk8s" / "events.jsonl").read_text().splitlines()]
    started = [e for e in events if e["event"] == "gpu_burnin_host_started"]
    assert len(started) == 1 and started[0].get("early") and started[0]["gpus"] == [0, 1]
    assert not any(e["event"] == "gpu_burnin_early_discarded" for e in events)
    # the control plane's interpreter started with the CLI and got its arguments at master boot
    boot = [e for e in events if e["event"] == "controlplane_boot_started"]
    assert len(boot) == 1 and boot[0].get("zygote")
    assert json.loads((ws / ".tk8s" / "machines" / "kubemaster" / "run" / "controlplane.args").read_text())[0] == "--host"
    # the agents' interpreters started with the CLI too (one zygote per planned worker) and got
    # their argv and machine environment at worker boot; rocmsetup's standby task found them running
    agents = [e for e in events if e["event"] == "agent_boot_started"]
    assert sorted(e["name"] for e in agents) == ["kubenode1", "kubenode2"] and all(e.get("zygote") for e in agents)
    for i in (1, 2):
        spec = json.loads((ws / ".tk8s" / "machines" / f"kubenode{i}" / "run" / "agent.args").read_text())
        assert spec["argv"][:2] == ["--await-url", "run/registration-url"] and spec["env"]["TK8S_MACHINE"] == f"kubenode{i}"
        assert spec["cwd"].endswith(f"kubenode{i}")
    standby = [e for e in events if e.get("task", "").endswith("Start the node agent in standby on every host")]
    assert standby and all(v in ("ok", "skipped") for v in standby[0]["results"].values()), standby
    for i in (1, 2):
        burn = json.loads((ws / ".tk8s" / "machines" / f"kubenode{i}" / "run" / "gpu-burnin.json.consumed").read_text())
        assert burn["host_burnin"] and burn["ok"]
    # teardown stops the adopted processes too (the zygote's supervisor holds the master's pidfile)
    sup = json.loads((ws / ".tk8s" / "machines" / "kubemaster" / "run" / "controlplane.pid").read_text())["pid"]
    pids = _pids(ws) + [sup]
    assert all(_alive(p) for p in pids)
    r = subprocess.run(["./setup.sh", "-c", "--yes"], cwd=ws, env=_env(), capture_output=True, text=True, timeout=120)
    assert r.returncode == 0
    deadline = time.monotonic() + 10
    while any(_alive(p) for p in pids) and time.monotonic() < deadline:
        time.sleep(0.05)
    assert not any(_alive(p) for p in pids)


def test_agent_boot_hook_uses_the_roles_standby_argv():
    """The worker boot hook pre-starts the agent the rocmsetup role would start: same argv, so
    the role's task finds it running instead of starting a second one."""
    import yaml

    from tritonk8ssupervisor_amd.orchestrator import agent_standby_argv

    tasks = yaml.safe_load((REPO / "ansible" / "roles" / "rocmsetup" / "tasks" / "main.yml").read_text())
    t = next(t for t in tasks if t.get("name") == "Start the node agent in standby on every host")
    subst = {"{{ tk8s_python }}": sys.executable, "{{ inventory_hostname }}": "kubenode1", "{{ ansible_host }}": "127.0.1.2"}
    assert [subst.get(a, a) for a in t["tk8s_daemon"]["argv"]] == agent_standby_argv("kubenode1", "127.0.1.2")


def test_scale_workers_up_and_down(ws):
    """Elastic node count: 2 -> 3 joins a new validated worker; 3 -> 1 drains (the Deployment's
    pods move), deletes the removed nodes and destroys their machines."""
    _summary(_setup(ws, "--nodes", "2", "--rccl", "off"))
    tk = lambda *a: subprocess.run(["./tk8s", *a], cwd=ws, env=_env(), capture_output=True, text=True, timeout=180)
    kc = lambda *a: subprocess.run(["./kubectl", *a], cwd=ws, env=_env(), capture_output=True, text=True, timeout=60)
    r = tk("scale", "3", "--json")
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert r.returncode == 0 and out["nodes"] == 3 and out["nodes_validated"] == 3 and out["gpus_allocatable"] == 3
    nodes = json.loads(kc("get", "nodes", "-o", "json").stdout)["items"]
    assert sorted(n["metadata"]["name"] for n in nodes) == ["kubenode1", "kubenode2", "kubenode3"]
    assert len((ws / "terraform" / "hosts.ip").read_text().split()) == 3
    assert "KUBERNETES_NUMBER_OF_NODES=3" in (ws / "config").read_text()
    # a workload on the node that goes away moves
    kc("create", "deployment", "web", "--image", "nginx", "--replicas", "2")
    kc("rollout", "status", "deploy/web", "--timeout", "60s")
    gone = [ws / ".tk8s" / "machines" / f"kubenode{i}" for i in (2, 3)]
    agent_pids = [json.loads((d / "run" / "agent.pid").read_text())["pid"] for d in gone]
    r = tk("scale", "1", "--json")
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert r.returncode == 0 and out["removed"] == ["kubenode2", "kubenode3"] and out["nodes_validated"] == 1, r.stdout[-2000:]
    nodes = json.loads(kc("get", "nodes", "-o", "json").stdout)["items"]
    assert [n["metadata"]["name"] for n in nodes] == ["kubenode1"]
    kc("rollout", "status", "deploy/web", "--timeout", "60s")
    pods = json.loads(kc("get", "pods", "-l", "app=web", "-o", "json").stdout)["items"]
    assert pods and all(p["spec"]["nodeName"] == "kubenode1" for p in pods if p["status"].get("phase") == "Running")
    assert not any(d.exists() for d in gone)
    deadline = time.monotonic() + 10
    while any(_alive(p) for p in agent_pids) and time.monotonic() < deadline:
        time.sleep(0.05)
    assert not any(_alive(p) for p in agent_pids)
    assert len((ws / "terraform" / "hosts.ip").read_text().split()) == 1
    assert tk("scale", "0").returncode != 0


def test_xgmi_link_report_judges_the_pull_matrix(monkeypatch):
    from tritonk8ssupervisor_amd import xgmi
    from tritonk8ssupervisor_amd.burnin import split_host_result

    def pull(s, d, g, ok=True):
        return {"ok": ok, "src_device": s, "dst_device": d, "kernel_gbps": g}

    n = 4
    res = {"ok": True, "devices": [{"device": d, "ok": True, "peers": [pull(s, d, 60.0) for s in range(n) if s != d]}
                                   for d in range(n)]}
    res["devices"][2]["peers"][0] = pull(0, 2, 12.0)           # 0 -> 2 runs at a fifth of the rest
    res["devices"][3]["peers"][1] = pull(1, 3, None, ok=False)  # 1 -> 3 failed outright
    gpus = [2, 3, 5, 7]  # host ordinals of the probe's devices 0..3
    rep = xgmi.link_report(res, gpus, fraction=0.5)
    assert rep["pulls"] == 12 and rep["median_gbps"] == 60.0 and rep["floor_gbps"] == 30.0
    assert {(e["src"], e["dst"]) for e in rep["degraded"]} == {(2, 5), (3, 7)}
    v = xgmi.node_view(rep, [7])
    assert not v["healthy"] and v["pulls"] == 6 and [(e["src"], e["dst"]) for e in v["degraded"]] == [(3, 7)]
    ann = xgmi.annotations(v)
    assert ann["tk8s.amd.com/xgmi-healthy"] == "false" and "3->7:failed" in ann["tk8s.amd.com/xgmi-links"]
    share = split_host_result(res, gpus, [3])
    assert share["ok"] and not share["xgmi"]["healthy"]  # its own GPU is fine; a link is not
    # the fault point scales one directed link (host ordinals)
    monkeypatch.setenv("TK8S_FAULTS", "xgmi.degrade@5-7:0.25")
    rep = xgmi.link_report(res, gpus, fraction=0.5)
    assert {(e["src"], e["dst"]) for e in rep["degraded"]} == {(2, 5), (3, 7), (5, 7)}


def test_host_burnin_pulls_every_link_only_with_two_or_more_gpus():
    from tritonk8ssupervisor_amd.earlyburn import default_validation_command, host_burnin_command

    base = default_validation_command(peers=False)
    assert "--peers" not in host_burnin_command(base, [0])       # N=1: a no-op by construction
    assert host_burnin_command(base, [0, 1]).count("--peers") == 1
    assert host_burnin_command(host_burnin_command(base, [0, 1]), [0, 1]).count("--peers") == 1


def test_setup_checks_xgmi_links_before_ready(ws):
    s = _summary(_setup(ws, "--nodes", "3", "--rccl", "off"))
    assert s["xgmi"]["pulls"] == 6 and not s["xgmi"]["degraded"]
    for i in (1, 2, 3):
        ann = s["validation"][f"kubenode{i}"]
        assert ann["xgmi-healthy"] == "true" and len(ann["xgmi-links"].split(",")) == 4  # 2 in + 2 out
    r = subprocess.run(["./kubectl", "get", "node", "kubenode1", "-o", "json"], cwd=ws, env=_env(),
                       capture_output=True, text=True)
    conds = {c["type"]: c for c in json.loads(r.stdout)["status"]["conditions"]}
    assert conds["XGMILinksHealthy"]["status"] == "True" and conds["Ready"]["status"] == "True"


def test_degraded_xgmi_link_marks_its_nodes_not_ready(ws):
    t = time.monotonic()
    r = _setup(ws, "--nodes", "3", "--rccl", "off", env=_env(TK8S_FAULTS="xgmi.degrade@0-1:0.1"))
    assert r.returncode == 2 and "XGMILinkDegraded" in r.stderr, r.stdout[-2000:] + r.stderr[-2000:]
    assert time.monotonic() - t < 60
    out = subprocess.run(["./kubectl", "get", "nodes"], cwd=ws, env=_env(), capture_output=True, text=True).stdout
    state = {l.split()[0]: l.split()[1] for l in out.splitlines()[1:] if l.strip()}
    # the machines are created concurrently: which node got host GPU 0 / 1 is not fixed
    alloc = json.loads((ws / ".tk8s" / "alloc.json").read_text())["gpus"]
    on_link = {alloc["0"], alloc["1"]}
    assert {n for n, st in state.items() if st == "NotReady"} == on_link, (out, alloc)
    d = subprocess.run(["./kubectl", "describe", "node", sorted(on_link)[0]], cwd=ws, env=_env(), capture_output=True,
                       text=True).stdout
    assert "XGMILinkDegraded" in d and "0->1" in d


def _kube(ws):
    from tritonk8ssupervisor_amd.controlplane.client import client_from_kubeconfig

    return client_from_kubeconfig(json.loads((ws / ".tk8s" / "kubeconfig.json").read_text()))


def _wait_pod(k, ns, name, timeout=30):
    deadline = time.monotonic() + timeout
    while time.monotonic() < deadline:
        p = k.get(k.k8s(f"/api/v1/namespaces/{ns}/pods/{name}"))
        if p.get("status", {}).get("phase") in ("Succeeded", "Failed"):
            return p
        time.sleep(0.05)
    raise AssertionError(f"pod {ns}/{name} did not finish: {p.get('status')}")


def test_pods_are_isolated_from_the_agent(ws):
    """P4: a pod's env is its spec + downward API + the device plugin's, not the agent's; node-wide
    GPU visibility is refused outside the cluster's own kube-system Jobs; CPU pods get their own
    PID namespace when the kernel allows it (and say so either way)."""
    from tritonk8ssupervisor_amd.controlplane.client import ApiError

    _summary(_setup(ws, "--nodes", "1", "--rccl", "off", env=_env(TK8S_FAULTS="agent.never@nowhere")))
    k = _kube(ws)
    script = "env; echo PIDNS_PID=$$"
    pod = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "envdump", "namespace": "default"},
           "spec": {"restartPolicy": "Never", "containers": [{"name": "c", "command": ["sh", "-c", script],
                                                              "env": [{"name": "MINE", "value": "x-$(POD_NAME)"}]}]}}
    k.post(k.k8s("/api/v1/namespaces/default/pods"), pod)
    p = _wait_pod(k, "default", "envdump")
    assert p["status"]["phase"] == "Succeeded"
    log = Path(p["metadata"]["annotations"]["tk8s.amd.com/log-path"]).read_text()
    env = dict(line.split("=", 1) for line in log.splitlines() if "=" in line)
    assert env["MINE"] == "x-envdump" and env["POD_NAME"] == "envdump" and env["NODE_NAME"] == "kubenode1"
    for leaked in ("PYTHONPATH", "TK8S_FAULTS", "TK8S_MACHINE", "TK8S_MACHINE_GPUS", "TK8S_PYTHON_PATH"):
        assert leaked not in env, leaked
    assert "TK8S_FAKE_GPUS" in env  # the fake-GPU switch of the test tier passes (POD_ENV_KEEP_PREFIXES)
    how = p["metadata"]["annotations"]["tk8s.amd.com/isolation"]
    assert how == "user,pid,mount" or how.startswith("none: ")
    if how == "user,pid,mount":
        assert env["PIDNS_PID"] in ("1", "2")  # init of its own PID namespace (or its first child)
    # node-wide GPU visibility: refused at admission for a user pod / a user Job ...
    vis = {"tk8s.amd.com/gpu-visibility": "node"}
    bad = json.loads(json.dumps(pod))
    bad["metadata"].update(name="peek", annotations=vis)
    with pytest.raises(ApiError) as e:
        k.post(k.k8s("/api/v1/namespaces/default/pods"), bad)
    assert e.value.status == 403
    job = {"apiVersion": "batch/v1", "kind": "Job", "metadata": {"name": "peekjob", "namespace": "default"},
           "spec": {"template": {"metadata": {"annotations": vis}, "spec": pod["spec"]}}}
    with pytest.raises(ApiError) as e:
        k.post(k.k8s("/apis/batch/v1/namespaces/default/jobs"), job)
    assert e.value.status == 403
    # ... and by the agent for a kube-system pod that no Job owns
    from tritonk8ssupervisor_amd.agent.agent import node_visibility_allowed

    assert not node_visibility_allowed({"metadata": {"namespace": "kube-system"}})
    assert node_visibility_allowed({"metadata": {"namespace": "kube-system", "ownerReferences": [{"kind": "Job"}]}})
    assert not node_visibility_allowed({"metadata": {"namespace": "default", "ownerReferences": [{"kind": "Job"}]}})


def test_shared_burnin_result_is_single_use(ws):
    """a re-created validation pod (agent restart, --resume, re-join) must probe the GPU
    again, never re-report a burn-in result an earlier pod already consumed."""
    _summary(_setup(ws, "--nodes", "1", "--rccl", "off"))
    run = ws / ".tk8s" / "machines" / "kubenode1" / "run"
    assert (run / "gpu-burnin.json.consumed").exists() and not (run / "gpu-burnin.json").exists()
    k = _kube(ws)
    k.delete(k.k8s("/api/v1/namespaces/kube-system/pods/amd-gpu-validation-kubenode1"))
    deadline = time.monotonic() + 30
    while True:  # the DaemonSet re-creates the pod; it finds no result and probes by itself
        try:
            p = k.get(k.k8s("/api/v1/namespaces/kube-system/pods/amd-gpu-validation-kubenode1"))
            if p.get("status", {}).get("phase") == "Succeeded":
                break
        except Exception:  # noqa: BLE001 - not re-created yet
            p = None
        if time.monotonic() >= deadline:
            log = ws / ".tk8s" / "machines" / "kubenode1" / "pods" / "kube-system_amd-gpu-validation-kubenode1" / "log"
            raise AssertionError(json.dumps({"status": (p or {}).get("status"), "run": sorted(x.name for x in run.iterdir()),
                                             "log": log.read_text()[-1500:] if log.exists() else None})[:4000])
        time.sleep(0.05)
    res = p["status"]["result"]
    assert res["ok"] and not res.get("host_burnin")  # its own probe, not the shared burn-in


def test_bringup_with_the_stock_terraform_modules(ws):
    """TK8S_TERRAFORM_FORM=compat: rancher.tf points at terraform/compat (terraform_data modules a
    stock `terraform plan` loads); the engine brings the same cluster up from them."""
    s = _summary(_setup(ws, "--nodes", "2", "--rccl", "off", env=_env(TK8S_TERRAFORM_FORM="compat")))
    assert s["nodes"] == 2 and s["nodes_validated"] == 2
    assert 'source = "compat/host"' in (ws / "terraform" / "rancher.tf").read_text()
    st = json.loads((ws / "terraform" / "terraform.tfstate").read_text())
    assert all(".terraform_data." in a for a in st["resources"])


def test_dry_run_plans_and_checks_without_changing_anything(ws):
    """BASELINE.json config 1 in one command: `terraform plan` + `ansible-playbook --check`."""
    r = _setup(ws, "--dry-run", "--nodes", "2")
    s = _summary(r)
    assert s["dry_run"] and s["check_ok"] and [p["action"] for p in s["plan"]] == ["create"] * 3
    assert "Plan: 3 to add, 0 to change, 0 to destroy." in r.stdout and "PLAY RECAP" in r.stdout
    for rel in ("config", "terraform/rancher.tf", "terraform/terraform.tfstate", "ansible/hosts",
                "ansible/tmp/kubernetes_environment.id"):
        assert not (ws / rel).exists(), rel
    assert not (ws / ".tk8s" / "machines").exists() and not _pids(ws)
    _summary(_setup(ws, "--nodes", "1", "--rccl", "off"))  # and a real run after it is unaffected


def test_dry_run_of_the_kubeadm_platform_on_an_inventory(ws):
    inv = {"ssh": {"user": "root", "key": str(ws / "nokey")}, "hosts": [
        {"name": "a", "address": "10.1.0.1", "gpus": 0, "role": "master"}, {"name": "b", "address": "10.1.0.2", "gpus": 8}]}
    subprocess.run(["ssh-keygen", "-q", "-t", "ed25519", "-N", "", "-f", str(ws / "nokey")], check=True)
    (ws / "inventory.yml").write_text(json.dumps(inv))
    r = _setup(ws, "--dry-run", "--nodes", "1", "--backend", "baremetal", "--platform", "kubeadm", "--package", "bm-8gpu")
    s = _summary(r)
    assert s["platform"] == "kubeadm" and s["check_ok"], r.stdout[-3000:]
    assert "kubeadm init" in r.stdout or "TASK [kubeadmmaster : kubeadm init" in r.stdout
    assert not (ws / "config").exists()


def test_dry_run_exits_nonzero_when_the_check_fails(ws):
    tasks = ws / "ansible" / "roles" / "rocmsetup" / "tasks" / "main.yml"
    tasks.write_text(tasks.read_text() + "\n- name: refuse this machine\n  fail:\n    msg: not today\n")
    r = _setup(ws, "--dry-run", "--nodes", "1")
    assert r.returncode == 2, r.stdout[-2000:] + r.stderr[-2000:]
    s = json.loads(r.stdout.strip().splitlines()[-1])
    assert not s["check_ok"] and s["check_failures"] and "--check playbook failed" in r.stderr
    assert not (ws / "config").exists() and not (ws / "terraform" / "rancher.tf").exists()


def test_rccl_job_runs_one_pod_per_host(ws):
    """mi355x-2gpu workers on two (simulated) hosts: the fabric Job is one pod per host holding
    both of its GPUs, one process driving them as consecutive ranks (not one process per GPU),
    the two pods joined by one communicator (ncclCommInitRank groups)."""
    s = _summary(_setup(ws, "--nodes", "2", "--package", "mi355x-2gpu", "--rccl", "on", env=_env(TK8S_FAKE_HOSTS="2")))
    rc = s["rccl"]
    assert rc["ok"] and rc["nranks"] == 4 and rc["pods"] == 2 and rc["gpus_per_pod"] == 2, rc
    assert rc["scope"] == "node"  # one node per host: no claims on other nodes needed
    assert sorted(r["node"] for r in rc["rank_results"]) == ["kubenode1", "kubenode2"]
    r = subprocess.run(["./kubectl", "get", "pods", "-n", "kube-system", "-l", f"job-name={rc['job']}", "-o", "json"],
                       cwd=ws, env=_env(), capture_output=True, text=True)
    res = sorted((p["status"]["result"] for p in json.loads(r.stdout)["items"]), key=lambda x: x["first_rank"])
    assert [(x["first_rank"], x["local_ranks"], x["mode"]) for x in res] == [(0, 2, "rank_group"), (2, 2, "rank_group")]
    assert all(x["nranks"] == 4 for x in res)


def _fake_gpu_tree(root: Path, n: int) -> tuple[Path, Path]:
    """A KFD topology + /dev/dri twin of TK8S_FAKE_GPUS=n (models/hostinfo.fake_inventory: KFD node
    i+1, render minor 128+i; node 0 the CPU) for the GPU jail to act on."""
    kfd, dri = root / "kfd" / "nodes", root / "dri"
    (kfd / "0").mkdir(parents=True)
    (kfd / "0" / "properties").write_text("cpu_cores_count 64\nsimd_count 0\n")
    dri.mkdir(parents=True)
    for i in range(n):
        (kfd / str(i + 1)).mkdir()
        (kfd / str(i + 1) / "properties").write_text(f"simd_count 1024\ndrm_render_minor {128 + i}\n")
        (dri / f"renderD{128 + i}").write_text(f"gpu{i}\n")
        (dri / f"card{i}").write_text(f"card{i}\n")
    return kfd, dri


def test_pods_can_open_only_their_gpus(ws, tmp_path_factory):
    """GPU isolation that does not depend on the pod's env. Every pod runs in the GPU
    jail (Landlock, native/tools/tk8s_gpujail.cpp): a pod holding one GPU can read that GPU's KFD node
    and render node and nothing of the other GPU -- even after clearing HIP_VISIBLE_DEVICES -- and a pod
    with no amd.com/gpu request can open none; `kubectl describe pod` names the isolation."""
    from tritonk8ssupervisor_amd.agent.runtime import gpu_jail

    if not gpu_jail()[0]:
        pytest.skip(f"GPU jail unavailable here: {gpu_jail()[1]}")
    d = tmp_path_factory.mktemp("jail")
    kfd, dri = _fake_gpu_tree(d, 2)
    env = _env(TK8S_FAKE_GPUS="2", TK8S_GPU_JAIL_KFD_ROOT=str(kfd), TK8S_GPU_JAIL_DRI_ROOT=str(dri))
    _summary(_setup(ws, "--nodes", "2", "--rccl", "off", env=env))
    probe = (f"unset HIP_VISIBLE_DEVICES ROCR_VISIBLE_DEVICES CUDA_VISIBLE_DEVICES; "
             f"for i in 1 2; do cat {kfd}/$i/properties >/dev/null 2>&1 && echo node$i=open || echo node$i=denied; done; "
             f"for m in 128 129; do cat {dri}/renderD$m >/dev/null 2>&1 && echo render$m=open || echo render$m=denied; done; "
             f"cat {kfd}/0/properties >/dev/null && echo cpu=open; echo iso=$TK8S_GPU_ISOLATION")
    for name, gpus in (("with-gpu", 1), ("no-gpu", 0)):
        res = {"limits": {"amd.com/gpu": gpus}} if gpus else {}
        (d / f"{name}.yaml").write_text(json.dumps({
            "apiVersion": "v1", "kind": "Pod", "metadata": {"name": name},
            "spec": {"restartPolicy": "Never", "containers": [{"name": "c", "command": ["sh", "-c", probe],
                                                               "resources": res}]}}))
    kc = lambda *a: subprocess.run(["./kubectl", *a], cwd=ws, env=env, capture_output=True, text=True, timeout=60)
    for name in ("with-gpu", "no-gpu"):
        assert kc("apply", "-f", str(d / f"{name}.yaml")).returncode == 0
    deadline = time.monotonic() + 30
    pods = {}
    while time.monotonic() < deadline:
        pods = {p["metadata"]["name"]: p for p in json.loads(kc("get", "pods", "-o", "json").stdout)["items"]}
        if all(pods.get(n, {}).get("status", {}).get("phase") == "Succeeded" for n in ("with-gpu", "no-gpu")):
            break
        time.sleep(0.2)
    logs = {n: dict(x.split("=", 1) for x in kc("logs", n).stdout.split() if "=" in x) for n in ("with-gpu", "no-gpu")}
    mine = pods["with-gpu"]["metadata"]["annotations"]["amd.com/gpu-ids"]  # gpu0 or gpu1
    i = int(mine[-1])
    other = 1 - i
    # the render nodes are the boundary (no render node: no GPU VM, no memory, no queues); the KFD
    # topology stays readable, as in a container (ROCm 7.2's thunk fails its whole start otherwise)
    assert logs["with-gpu"][f"render{128 + i}"] == "open", logs
    assert logs["with-gpu"][f"render{128 + other}"] == "denied", logs
    assert logs["no-gpu"] == {"node1": "open", "node2": "open", "render128": "denied", "render129": "denied",
                              "cpu": "open", "iso": logs["no-gpu"]["iso"]}, logs
    assert logs["no-gpu"]["iso"].startswith("landlock:abi")
    r = kc("describe", "pod", "no-gpu")
    assert "Isolation:" in r.stdout and "may open no GPU" in r.stdout, r.stdout
    assert f"may open gpu{i}" in kc("describe", "pod", "with-gpu").stdout


def test_rccl_job_one_process_for_multi_gpu_nodes_on_one_host(ws):
    """Two 2-GPU workers on ONE host: one host-scoped pod, one process, 4 ranks."""
    s = _summary(_setup(ws, "--nodes", "2", "--package", "mi355x-2gpu", "--rccl", "on"))
    rc = s["rccl"]
    assert rc["ok"] and rc["nranks"] == 4 and rc["pods"] == 1 and rc["gpus_per_pod"] == 4 and rc["scope"] == "host", rc


def _ws_exec(host: str, port: int, path: str, token: str, proto: str = "v5.channel.k8s.io", stdin: bytes | None = None):
    """A stock kubectl's exec, at the wire level: GET upgraded to a WebSocket, channel-prefixed
    frames back (kubectl >= 1.29 talks exactly this; no kubectl binary is installed here)."""
    import base64
    import socket as _s

    sock = _s.create_connection((host, port), timeout=30)
    key = base64.b64encode(os.urandom(16)).decode()
    sock.sendall((f"GET {path} HTTP/1.1\r\nHost: {host}:{port}\r\nUpgrade: websocket\r\nConnection: Upgrade\r\n"
                  f"Sec-WebSocket-Key: {key}\r\nSec-WebSocket-Version: 13\r\nSec-WebSocket-Protocol: {proto}\r\n"
                  f"Authorization: Bearer {token}\r\n\r\n").encode())
    f = sock.makefile("rb")
    status = f.readline().decode()
    headers = {}
    while True:
        line = f.readline().decode().strip()
        if not line:
            break
        k, _, v = line.partition(":")
        headers[k.strip().lower()] = v.strip()

    def send(payload: bytes, opcode=0x2):
        mask = os.urandom(4)
        n = len(payload)
        head = bytes([0x80 | opcode, 0x80 | n]) if n < 126 else bytes([0x80 | opcode, 0x80 | 126]) + n.to_bytes(2, "big")
        sock.sendall(head + mask + bytes(b ^ mask[i & 3] for i, b in enumerate(payload)))

    if stdin is not None and status.startswith("HTTP/1.1 101"):
        send(b"\x00" + stdin)
        send(b"\xff\x00")  # v5: close stdin
    frames = []
    while status.startswith("HTTP/1.1 101"):
        h = f.read(2)
        if len(h) < 2:
            break
        n = h[1] & 0x7F
        if n == 126:
            n = int.from_bytes(f.read(2), "big")
        elif n == 127:
            n = int.from_bytes(f.read(8), "big")
        data = f.read(n)
        if h[0] & 0x0F == 0x8:
            break
        frames.append((data[0], data[1:]))
    sock.close()
    return status, headers, frames


def test_stock_kubectl_exec_over_websocket(ws, tmp_path_factory):
    """`kubectl exec` of a stock client (v5.channel.k8s.io WebSocket; v4 without
    stdin) runs the command in the pod and returns stdout / stderr / the exit Status."""
    from urllib.parse import urlsplit

    _summary(_setup(ws, "--nodes", "1", "--rccl", "off"))
    d = tmp_path_factory.mktemp("wsx")
    (d / "pod.json").write_text(json.dumps({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "box"},
                                            "spec": {"containers": [{"name": "c", "command": ["sleep", "60"]}]}}))
    kc = lambda *a: subprocess.run(["./kubectl", *a], cwd=ws, env=_env(), capture_output=True, text=True, timeout=60)
    assert kc("apply", "-f", str(d / "pod.json")).returncode == 0
    deadline = time.monotonic() + 30
    while time.monotonic() < deadline and json.loads(kc("get", "pod", "box", "-o", "json").stdout)["status"].get("phase") != "Running":
        time.sleep(0.1)
    cfg = json.loads((ws / ".tk8s" / "kubeconfig.json").read_text())
    server = urlsplit(cfg["clusters"][0]["cluster"]["server"])
    token = cfg["users"][0]["user"]["token"]
    base = f"{server.path}/api/v1/namespaces/default/pods/box/exec"
    q = "?command=sh&command=-c&command=echo+out%3B+echo+err+%3E%262%3B+exit+3&stdout=true&stderr=true"
    status, headers, frames = _ws_exec(server.hostname, server.port, base + q, token)
    assert status.startswith("HTTP/1.1 101") and headers["sec-websocket-protocol"] == "v5.channel.k8s.io", status
    by = {}
    for ch, data in frames:
        by[ch] = by.get(ch, b"") + data
    assert by[1] == b"out\n" and by[2] == b"err\n", frames
    st = json.loads(by[3])
    assert st["status"] == "Failure" and st["details"]["causes"][0]["message"] == "3", st
    # stdin (v5 closes it with [255, 0])
    q = "?command=cat&stdin=true&stdout=true"
    status, _, frames = _ws_exec(server.hostname, server.port, base + q, token, stdin=b"hello from stdin")
    assert (1, b"hello from stdin") in frames and json.loads(dict(frames)[3])["status"] == "Success", frames
    # binary both ways, as `kubectl cp` streams tar archives: every byte value survives
    blob = bytes(range(256)) * 4
    status, _, frames = _ws_exec(server.hostname, server.port, base + q, token, stdin=blob)
    assert b"".join(d for ch, d in frames if ch == 1) == blob, frames[:3]
    q2 = "?command=sh&command=-c&command=mkdir+-p+t%3B+printf+%27%5C000%5C377%27+%3E+t%2Fb%3B+tar+cf+-+t&stdout=true"
    status, _, frames = _ws_exec(server.hostname, server.port, base + q2, token)
    import io
    import tarfile

    tar = tarfile.open(fileobj=io.BytesIO(b"".join(d for ch, d in frames if ch == 1)))
    assert tar.extractfile("t/b").read() == b"\x00\xff"
    # no token, no exec
    status, _, _ = _ws_exec(server.hostname, server.port, base + q, "wrong")
    assert status.startswith("HTTP/1.1 401"), status


def test_stock_kubectl_exec_with_a_tty_is_interactive(ws, tmp_path_factory):
    """VERDICT r5 missing-3: `kubectl exec -it` (tty=true): the command runs on a pseudo-terminal
    in the pod and the bytes stream both ways WHILE it runs -- a resize (channel 4) reaches the
    terminal, stdin typed after the start is read, and the exit status comes back last."""
    from urllib.parse import urlsplit

    from tritonk8ssupervisor_amd.controlplane.wsclient import WSClient

    _summary(_setup(ws, "--nodes", "1", "--rccl", "off"))
    d = tmp_path_factory.mktemp("wsxt")
    (d / "pod.json").write_text(json.dumps({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "tty"},
                                            "spec": {"containers": [{"name": "c", "command": ["sleep", "120"]}]}}))
    kc = lambda *a: subprocess.run(["./kubectl", *a], cwd=ws, env=_env(), capture_output=True, text=True, timeout=60)
    assert kc("apply", "-f", str(d / "pod.json")).returncode == 0
    deadline = time.monotonic() + 30
    while time.monotonic() < deadline and json.loads(kc("get", "pod", "tty", "-o", "json").stdout)["status"].get("phase") != "Running":
        time.sleep(0.1)
    cfg = json.loads((ws / ".tk8s" / "kubeconfig.json").read_text())
    server = urlsplit(cfg["clusters"][0]["cluster"]["server"])
    token = cfg["users"][0]["user"]["token"]
    w = WSClient.connect(server.hostname, server.port, f"{server.path}/api/v1/namespaces/default/pods/tty/exec",
                         query=[("command", "sh"), ("stdin", "true"), ("stdout", "true"), ("tty", "true")],
                         token=token, protocols=("v5.channel.k8s.io",), timeout=30)
    assert w.protocol == "v5.channel.k8s.io"
    w.send(b"\x04" + json.dumps({"Width": 101, "Height": 37}).encode())
    time.sleep(0.3)  # typed after the command started: read from the terminal as it runs
    w.send(b"\x00" + b"stty size; echo answer=$((6*7)); exit 5\n")
    out, status = b"", None
    deadline = time.monotonic() + 30
    while time.monotonic() < deadline:
        m = w.recv()
        if m is None:
            break
        if m[:1] == b"\x01":
            out += m[1:]
        elif m[:1] == b"\x03":
            status = json.loads(m[1:])
            break
    w.close()
    text = out.decode(errors="replace")
    assert "37 101" in text and "answer=42" in text, text
    assert status and status["status"] == "Failure" and status["details"]["causes"][0]["message"] == "5", status
    # the bundled kubectl's `exec -it` speaks the same (stdin a pipe here, not a terminal)
    r = subprocess.run(["./kubectl", "exec", "-it", "tty", "--", "sh"], cwd=ws, env=_env(), capture_output=True,
                       input="echo hi-$((2+3)); exit 3\n", text=True, timeout=60)
    assert r.returncode == 3 and "hi-5" in r.stdout, (r.returncode, r.stdout, r.stderr)


def test_attach_to_a_pods_stdin_and_tty_and_kubectl_run_it(ws, tmp_path_factory):
    """`kubectl attach -it` and `kubectl run -it --rm`: a container started with `stdin: true` /
    `tty: true` keeps its input open (a pipe, or a pty whose output the agent pumps to the log
    and to attached sessions). A session sees the resize and the typed input while the container
    runs; a client that detaches leaves it running; its exit status ends the last session."""
    from urllib.parse import urlsplit

    from tritonk8ssupervisor_amd.controlplane.wsclient import WSClient, WSClosed

    _summary(_setup(ws, "--nodes", "1", "--rccl", "off"))
    d = tmp_path_factory.mktemp("wsat")
    kc = lambda *a, **kw: subprocess.run(["./kubectl", *a], cwd=ws, env=_env(), capture_output=True, text=True,
                                         timeout=60, **kw)

    def pod(name, c):
        (d / f"{name}.json").write_text(json.dumps({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name},
                                                    "spec": {"restartPolicy": "Never",
                                                             "containers": [{"name": "c", **c}]}}))
        assert kc("apply", "-f", str(d / f"{name}.json")).returncode == 0
        deadline = time.monotonic() + 30
        while time.monotonic() < deadline and json.loads(kc("get", "pod", name, "-o", "json").stdout)["status"].get("phase") != "Running":
            time.sleep(0.1)

    cfg = json.loads((ws / ".tk8s" / "kubeconfig.json").read_text())
    server = urlsplit(cfg["clusters"][0]["cluster"]["server"])
    token = cfg["users"][0]["user"]["token"]

    def attach(name, query):
        return WSClient.connect(server.hostname, server.port, f"{server.path}/api/v1/namespaces/default/pods/{name}/attach",
                                query=query, token=token, protocols=("v5.channel.k8s.io",), timeout=30)

    def read_until(w, needle):
        out, status, deadline = b"", None, time.monotonic() + 30
        while time.monotonic() < deadline and needle not in out and status is None:
            m = w.recv()
            if m is None:
                break
            if m[:1] == b"\x01":
                out += m[1:]
            elif m[:1] == b"\x03":
                status = json.loads(m[1:])
        return out.decode(errors="replace"), status

    # a container without stdin: true refuses -i
    pod("plain", {"command": ["sleep", "120"]})
    with pytest.raises(WSClosed, match="stdin"):
        attach("plain", [("stdin", "true"), ("stdout", "true")])
    # a tty container: resize, input, detach (it runs on), a second session sees its exit status
    pod("term", {"command": ["sh"], "stdin": True, "tty": True})
    w = attach("term", [("stdin", "true"), ("stdout", "true"), ("tty", "true")])
    w.send(b"\x04" + json.dumps({"Width": 99, "Height": 33}).encode())
    time.sleep(0.2)
    w.send(b"\x00" + b"stty size; echo v=$((6*7))\n")
    text, status = read_until(w, b"v=42")
    assert "33 99" in text and "v=42" in text and status is None, (text, status)
    w.close()  # detach
    time.sleep(0.5)
    assert json.loads(kc("get", "pod", "term", "-o", "json").stdout)["status"]["phase"] == "Running"
    w = attach("term", [("stdin", "true"), ("stdout", "true"), ("tty", "true")])
    w.send(b"\x00" + b"echo again-$((1+1)); exit 4\n")
    text, status = read_until(w, b"never")
    w.close()
    assert "again-2" in text and status and status["details"]["causes"][0]["message"] == "4", (text, status)
    # stdin without a tty: the bundled kubectl's `attach -i`, the output from the container's log
    pod("pipe", {"command": ["sh", "-c", "read x; echo got-$x; exit 0"], "stdin": True, "stdinOnce": True})
    r = kc("attach", "-i", "pipe", input="hello\n")
    assert r.returncode == 0 and "got-hello" in r.stdout, (r.returncode, r.stdout, r.stderr)
    # kubectl run -it --rm: created, attached, the container's exit code, deleted
    r = kc("run", "-i", "-t", "--rm", "--restart=Never", "oneoff", "--image=busybox", "--command", "--",
           "sh", "-c", "read a; echo run-$a; exit 6", input="yes\n")
    assert r.returncode == 6 and "run-yes" in r.stdout and 'pod "oneoff" deleted' in r.stderr, (r.returncode, r.stdout, r.stderr)
    assert kc("get", "pod", "oneoff").returncode != 0


def test_exec_it_on_a_node_without_pseudo_terminals_runs_on_pipes(ws):
    """The MI355X GPU boxes mount no devpts: `kubectl exec -it` there runs the command on pipes
    (keystrokes in, output back as it comes, its exit code last) and says so, and a `tty: true`
    pod runs as `tty: false` with its stdin pipe (node.no_pty injects the missing devpts)."""
    _summary(_setup(ws, "--nodes", "1", "--rccl", "off", env=_env(TK8S_FAULTS="node.no_pty")))
    kc = lambda *a, **kw: subprocess.run(["./kubectl", *a], cwd=ws, env=_env(), capture_output=True, text=True,
                                         timeout=60, **kw)
    (ws / "p.json").write_text(json.dumps({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "np"},
                                           "spec": {"containers": [{"name": "c", "command": ["sleep", "120"]}]}}))
    assert kc("apply", "-f", str(ws / "p.json")).returncode == 0
    deadline = time.monotonic() + 30
    while time.monotonic() < deadline and json.loads(kc("get", "pod", "np", "-o", "json").stdout)["status"].get("phase") != "Running":
        time.sleep(0.1)
    r = kc("exec", "-it", "np", "--", "sh", input="echo piped-$((4+5)); [ -t 0 ] || echo notty; exit 4\n")
    assert r.returncode == 4 and "piped-9" in r.stdout and "notty" in r.stdout, (r.returncode, r.stdout, r.stderr)
    assert "no pseudo-terminal on node" in r.stdout, r.stdout
    # a tty pod: no pty to give it, so its stdin is a pipe (the bundled kubectl run -it still works)
    r = kc("run", "-i", "-t", "--rm", "--restart=Never", "tt", "--image=busybox", "--command", "--",
           "sh", "-c", "read a; echo run-$a; [ -t 0 ] || echo nopty", input="ok\n")
    assert r.returncode == 0 and "run-ok" in r.stdout and "nopty" in r.stdout, (r.returncode, r.stdout, r.stderr)
