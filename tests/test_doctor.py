"""./tk8s doctor: preflight checks per backend/platform (tritonk8ssupervisor_amd/doctor.py)."""
import json
import os
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]


def _doctor(*args, env=None, cwd=REPO):
    e = dict(os.environ, PYTHONPATH=str(REPO))
    e.update(env or {})
    r = subprocess.run([str(REPO / "tk8s"), "doctor", "--json", *args], cwd=cwd, env=e, capture_output=True,
                       text=True, timeout=120)
    assert r.stdout.strip(), r.stderr[-2000:]
    return r.returncode, {c["check"]: c for c in json.loads(r.stdout)}


def test_local_backend_with_fake_gpus_passes_with_warnings():
    rc, checks = _doctor(env={"TK8S_FAKE_GPUS": "2"})
    assert rc == 0, checks
    assert checks["python"]["status"] == "OK" and checks["native build"]["status"] in ("OK", "WARN")
    assert checks["gpus"]["status"] == "WARN" and "fake" in checks["gpus"]["detail"]
    assert {"loopback addresses", "pod isolation", "disk", "/dev/kfd"} <= set(checks)


def test_local_backend_without_a_gpu_fails():
    if os.path.exists("/dev/kfd"):
        import pytest

        pytest.skip("this host has a KFD")
    env = {k: v for k, v in os.environ.items() if k != "TK8S_FAKE_GPUS"}
    e = dict(env, PYTHONPATH=str(REPO))
    r = subprocess.run([str(REPO / "tk8s"), "doctor"], cwd=REPO, env=e, capture_output=True, text=True, timeout=120)
    assert r.returncode == 1 and "FAIL" in r.stdout and "/dev/kfd" in r.stdout


def test_kubeadm_platform_on_the_local_backend_needs_root():
    rc, checks = _doctor("--platform", "kubeadm", env={"TK8S_FAKE_GPUS": "2"})
    if os.geteuid() == 0:  # one-command single-node kubeadm on this host
        assert checks["kubeadm platform"]["status"] == "OK" and "single-node" in checks["kubeadm platform"]["detail"]
    else:
        assert rc == 1 and checks["kubeadm platform"]["status"] == "FAIL" and "root" in checks["kubeadm platform"]["detail"]


def test_doctor_reports_pod_signals_and_resource_limits():
    _rc, checks = _doctor(env={"TK8S_FAKE_GPUS": "2"})
    assert checks["resource limits"]["status"] in ("OK", "WARN") and checks["resource limits"]["detail"]
    assert checks["pod signals"]["status"] in ("OK", "WARN")
    _rc, checks = _doctor(env={"TK8S_FAKE_GPUS": "2", "TK8S_POD_RESOURCES": "watchdog"})
    assert checks["resource limits"]["status"] == "WARN" and "watchdog" in checks["resource limits"]["detail"]


def test_baremetal_hosts_are_checked_over_ssh(tmp_path):
    """Two reachable fake hosts (tests/fakessh.py) and one that is not in the fake-ssh root."""
    keydir = tmp_path / "keys"
    keydir.mkdir()
    subprocess.run(["ssh-keygen", "-q", "-t", "ed25519", "-N", "", "-f", str(keydir / "id")], check=True)
    root = tmp_path / "hosts"
    hosts = {"a": "127.0.8.10", "b": "127.0.8.11"}
    for name, addr in hosts.items():
        h = root / addr
        (h / ".ssh").mkdir(parents=True)
        (h / ".ssh" / "authorized_keys").write_text((keydir / "id.pub").read_text())
        (h / ".env").write_text("TK8S_FAKE_GPUS=4\n")
    inv = {"ssh": {"user": "root", "key": str(keydir / "id")}, "hosts": [
        {"name": n, "address": a, "gpus": 4} for n, a in hosts.items()] + [{"name": "gone", "address": "127.0.8.99", "gpus": 4}]}
    ws = tmp_path / "ws"
    ws.mkdir()
    (ws / "inventory.yml").write_text(json.dumps(inv))
    env = {"TK8S_SSH": f"{sys.executable} {REPO / 'tests' / 'fakessh.py'}", "FAKESSH_ROOT": str(root),
           "TK8S_SSH_CONNECT_RETRIES": "0", "TK8S_FAKE_GPUS": "4"}
    rc, checks = _doctor("--backend", "baremetal", env={**env, "TK8S_WORKDIR": str(ws)}, cwd=ws)
    assert checks["inventory"]["status"] == "OK" and "3 host(s)" in checks["inventory"]["detail"]
    assert checks["ssh a"]["status"] == "WARN" and "fake GPUs" in checks["ssh a"]["detail"], checks["ssh a"]
    assert checks["ssh b"]["status"] == "WARN"
    assert checks["ssh gone"]["status"] == "FAIL" and rc == 1
    # the kubeadm platform also needs root and apt on every host
    rc, checks = _doctor("--backend", "baremetal", "--platform", "kubeadm", env={**env, "TK8S_WORKDIR": str(ws)}, cwd=ws)
    assert "apt" in checks["ssh a"]["detail"] and checks["kubeadm platform"]["status"] == "OK"
