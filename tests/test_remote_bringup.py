"""Bring-up over SSH: ``./setup.sh --backend baremetal`` against an inventory of two "hosts".

Every host is a directory driven by a fake ``ssh`` (tests/fakessh.py): commands run there with
the host's own login environment (its ``.env``), never the controller's. The test proves the
remote path end to end (VERDICT r1 "Next round" #1):

* the tk8s distribution is installed on each host over ssh and every daemon (control plane,
  agents, GPU burn-ins) runs from THAT install, started through an ssh session -- the
  controller spawns none of them;
* machines are placed as GPU slices of the hosts (inventory order, one host filled first);
* all nodes reach Ready with their GPUs validated, and ``./setup.sh -c`` stops every process
  and removes every machine directory on the hosts.
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
HOSTS = {"mi355x-a": "127.0.7.10", "mi355x-b": "127.0.7.11"}


def _alive(pid: int) -> bool:
    try:
        os.kill(pid, 0)
        with open(f"/proc/{pid}/stat") as f:
            return f.read().rsplit(")", 1)[1].split()[0] != "Z"
    except OSError:
        return False


def _environ(pid: int) -> dict:
    try:
        raw = Path(f"/proc/{pid}/environ").read_bytes()
    except OSError:
        return {}
    return dict(x.split("=", 1) for x in raw.decode(errors="replace").split("\0") if "=" in x)


@pytest.fixture
def bm(tmp_path):
    from tritonk8ssupervisor_amd.orchestrator import init_workspace

    ws = tmp_path / "ws"
    ws.mkdir()
    init_workspace(ws)
    for f in ("setup.sh", "tk8s", "kubectl"):
        shutil.copy2(REPO / f, ws / f)
    keydir = tmp_path / "keys"
    keydir.mkdir()
    subprocess.run(["ssh-keygen", "-q", "-t", "ed25519", "-N", "", "-f", str(keydir / "id_ed25519")], check=True)
    root = tmp_path / "hosts"
    for name, addr in HOSTS.items():
        h = root / addr
        (h / ".ssh").mkdir(parents=True)
        (h / ".ssh" / "authorized_keys").write_text((keydir / "id_ed25519.pub").read_text())
        # the host's login environment: 4 (fake) MI355X GPUs
        (h / ".env").write_text("TK8S_FAKE_GPUS=4\nTK8S_HOST_LABEL=" + name + "\n")
    inv = {"ssh": {"user": "root", "key": str(keydir / "id_ed25519")}, "python": sys.executable,
           "hosts": [{"name": n, "address": a, "gpus": 4} for n, a in HOSTS.items()]}
    (ws / "inventory.yml").write_text(json.dumps(inv))  # JSON is YAML
    env = dict(os.environ)
    env.update(PYTHONPATH=str(REPO), TK8S_PYTHON=sys.executable, TK8S_BACKEND="baremetal",
               TK8S_SSH=f"{sys.executable} {REPO / 'tests' / 'fakessh.py'}", FAKESSH_ROOT=str(root),
               TK8S_FAKE_GPUS="4", TK8S_CONTROLLER_ONLY="leak-check", TK8S_SSH_CONNECT_RETRIES="0", TK8S_PLATFORM="tk8s")
    env.pop("TK8S_FAULTS", None)
    yield ws, root, env
    subprocess.run(["./setup.sh", "-c", "--yes"], cwd=ws, env=env, capture_output=True, timeout=120)


def _daemon_pids(root: Path) -> list[int]:
    out = []
    for pf in [*root.glob("*/tk8s/machines/*/run/agent.pid"), *root.glob("*/tk8s/machines/*/run/controlplane.pid")]:
        try:
            out.append(int(json.loads(pf.read_text())["pid"]))
        except (ValueError, KeyError, OSError):
            pass
    return out


def test_baremetal_bringup_over_ssh(bm):
    ws, root, env = bm
    t = time.monotonic()
    r = subprocess.run(["./setup.sh", "--yes", "--json", "--port", "0", "--nodes", "5"],
                       cwd=ws, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    s = json.loads(r.stdout.strip().splitlines()[-1])
    assert s["nodes"] == 5 and s["gpus_allocatable"] == 5 and s["nodes_validated"] == 5
    # the fabric check ran across both hosts: one rank per GPU, on the machines' own installs
    assert s["rccl"]["ok"] and s["rccl"]["nranks"] == 5
    assert len({r["node"] for r in s["rccl"]["rank_results"]}) == 5
    assert time.monotonic() - t < 180
    cfg = (ws / "config").read_text()
    assert "TK8S_BACKEND=baremetal" in cfg and "HOST_PACKAGE=" in cfg

    # placement: the master and 4 workers fill host a (4 GPUs), the 5th worker spills to host b
    # (creates run concurrently, so which worker spills is not fixed)
    alloc = json.loads((ws / ".tk8s" / "baremetal-alloc.json").read_text())["machines"]
    assert alloc["kubemaster"]["host"] == "mi355x-a" and alloc["kubemaster"]["gpus"] == []
    workers = [alloc[f"kubenode{i}"] for i in range(1, 6)]
    assert sorted(w["host"] for w in workers) == ["mi355x-a"] * 4 + ["mi355x-b"]
    assert sorted(g for w in workers if w["host"] == "mi355x-a" for g in w["gpus"]) == [0, 1, 2, 3]
    assert [w["gpus"] for w in workers if w["host"] == "mi355x-b"] == [[0]]
    hosts_ip = (ws / "terraform" / "hosts.ip").read_text().split()  # module order
    assert hosts_ip == [HOSTS[w["host"]] for w in workers]

    # the tk8s distribution was installed on both hosts; machines live under the hosts' homes
    for addr in HOSTS.values():
        dists = list((root / addr / ".tk8s" / "dist").glob("*/.tk8s-dist-ok"))
        assert len(dists) == 1
    machines = {m.name: m for m in
                __import__("tritonk8ssupervisor_amd.provider.baremetal", fromlist=["x"]).BareMetalProvider(
                    ws / ".tk8s").list_machines()}
    spilled = next(f"kubenode{i}" for i, w in enumerate(workers, 1) if w["host"] == "mi355x-b")
    assert machines[spilled].sandbox.startswith(str(root / HOSTS["mi355x-b"]))

    # every daemon runs from the host's install, started through an ssh login session: its
    # environment is the host's (FAKESSH_HOST, the host's .env), never the controller's
    pids = _daemon_pids(root)
    assert len(pids) == 6
    names = sorted(p.name for p in root.glob("*/tk8s/machines/*/run/*.pid"))
    assert names.count("agent.pid") == 5 and names.count("controlplane.pid") == 1
    for pid in pids:
        assert _alive(pid)
        e = _environ(pid)
        assert e.get("FAKESSH_HOST") in HOSTS.values(), e
        assert "TK8S_CONTROLLER_ONLY" not in e
        assert e.get("TK8S_HOST_LABEL") in HOSTS
        assert str(REPO) not in e.get("PYTHONPATH", ""), e.get("PYTHONPATH")
        assert "/.tk8s/dist/" in e.get("PYTHONPATH", "")
    # every remote command went through ssh with the inventory key and host-key checking on
    calls = [json.loads(x) for x in (root / "calls.jsonl").read_text().splitlines()]
    assert calls and all(c["key"] and c["opts"].get("StrictHostKeyChecking") == "accept-new" for c in calls)
    assert {c["host"] for c in calls} == set(HOSTS.values())
    kh = (ws / ".tk8s" / "known_hosts").read_text()
    assert all(a in kh for a in HOSTS.values())

    # the GPU burn-in ran ON the host (its result file is in the machine's dir there)
    for i in range(1, 6):
        m = machines[f"kubenode{i}"]
        burn = json.loads(Path(m.sandbox, "run", "gpu-burnin.json.consumed").read_text())
        assert burn["ok"]

    # kubectl sees 5 Ready nodes with one GPU each
    k = subprocess.run(["./kubectl", "get", "nodes", "-o", "json"], cwd=ws, env=env, capture_output=True, text=True)
    items = json.loads(k.stdout)["items"]
    assert len(items) == 5 and all(i["status"]["allocatable"]["amd.com/gpu"] == "1" for i in items)

    # teardown over ssh: every daemon stopped, every machine dir removed on the hosts
    c = subprocess.run(["./setup.sh", "-c", "--yes"], cwd=ws, env=env, capture_output=True, text=True, timeout=120)
    assert c.returncode == 0 and "All clear!" in c.stdout, c.stdout + c.stderr
    deadline = time.monotonic() + 10
    while any(_alive(p) for p in pids) and time.monotonic() < deadline:
        time.sleep(0.05)
    assert not any(_alive(p) for p in pids)
    assert not list(root.glob("*/tk8s/machines/*"))
    assert not json.loads((ws / ".tk8s" / "baremetal-alloc.json").read_text()).get("machines")


def test_baremetal_unreachable_host_fails_provisioning(bm):
    ws, root, env = bm
    shutil.rmtree(root / HOSTS["mi355x-a"])  # the host is down
    r = subprocess.run(["./setup.sh", "--yes", "--json", "--port", "0", "--nodes", "1", "--rccl", "off"],
                       cwd=ws, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "No route to host" in (r.stdout + r.stderr) or "provisioning limit" in (r.stdout + r.stderr)


def test_baremetal_wrong_key_is_refused(bm, tmp_path):
    ws, root, env = bm
    for addr in HOSTS.values():  # the hosts authorise a different key
        (root / addr / ".ssh" / "authorized_keys").write_text("ssh-ed25519 AAAAnotthekey other\n")
    r = subprocess.run(["./setup.sh", "--yes", "--json", "--port", "0", "--nodes", "1", "--rccl", "off"],
                       cwd=ws, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "Permission denied" in (r.stdout + r.stderr)


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_baremetal_bringup_over_ssh_on_a_real_gpu(tmp_path):
    """The remote path with the real validation payload: one inventory host (this GPU box behind
    the fake ssh) with its real MI355X(s); the tk8s distribution is pushed, the burn-in
    (tk8s-hsaprobe) and the agent run through ssh sessions, the validation pod reuses the
    burn-in's result with tk8s-reuse, and the node is Ready with its GPU validated."""
    from tritonk8ssupervisor_amd.models.hostinfo import discover
    from tritonk8ssupervisor_amd.orchestrator import init_workspace

    n = discover().count
    if n < 1:
        pytest.skip("no GPU")
    ws = tmp_path / "ws"
    ws.mkdir()
    init_workspace(ws)
    for f in ("setup.sh", "tk8s", "kubectl"):
        shutil.copy2(REPO / f, ws / f)
    keydir = tmp_path / "keys"
    keydir.mkdir()
    subprocess.run(["ssh-keygen", "-q", "-t", "ed25519", "-N", "", "-f", str(keydir / "id_ed25519")], check=True)
    root = tmp_path / "hosts"
    h = root / "127.0.7.20"
    (h / ".ssh").mkdir(parents=True)
    (h / ".ssh" / "authorized_keys").write_text((keydir / "id_ed25519.pub").read_text())
    keep = {k: v for k, v in os.environ.items() if k.startswith(("HSA_", "ROCM", "HIP_", "LD_LIBRARY_PATH"))}
    (h / ".env").write_text("".join(f"{k}={v}\n" for k, v in keep.items()))
    inv = {"ssh": {"user": "root", "key": str(keydir / "id_ed25519")}, "python": sys.executable,
           "hosts": [{"name": "box", "address": "127.0.7.20", "gpus": n}]}
    (ws / "inventory.yml").write_text(json.dumps(inv))
    env = {k: v for k, v in os.environ.items() if k != "TK8S_FAKE_GPUS"}
    env.update(PYTHONPATH=str(REPO), TK8S_PYTHON=sys.executable, TK8S_BACKEND="baremetal", TK8S_PLATFORM="tk8s",
               TK8S_SSH=f"{sys.executable} {REPO / 'tests' / 'fakessh.py'}", FAKESSH_ROOT=str(root),
               TK8S_SSH_CONNECT_RETRIES="0")
    try:
        r = subprocess.run(["./setup.sh", "--yes", "--json", "--port", "0", "--nodes", "1", "--timeout", "120"],
                           cwd=ws, env=env, capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
        s = json.loads(r.stdout.strip().splitlines()[-1])
        assert s["gpus_allocatable"] == 1 and s["nodes_validated"] == 1
        v = s["validation"]["kubenode1"]
        assert float(v["hbm-write-gbps"]) > 1000.0
        burn = next(root.glob("*/tk8s/machines/kubenode1/run/gpu-burnin.json.consumed"))
        res = json.loads(burn.read_text())
        assert res["ok"] and res["md5"]["digest"] == res["md5_expected"]
    finally:
        subprocess.run(["./setup.sh", "-c", "--yes"], cwd=ws, env=env, capture_output=True, timeout=120)
    assert not list(root.glob("*/tk8s/machines/*"))
