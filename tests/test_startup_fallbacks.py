"""Failure injection for every start-up shortcut of the bring-up: each one must
fall back to a correct, slower bring-up when it breaks.

* control-plane / node-agent zygotes (earlyburn.controlplane_zygote / agent_zygotes): an
  interpreter started early that waits for its arguments -- here never handed them;
* the CPU-cache-walk skip of the GPU tools (native/tools/cachewalk.h) -- here switched off with
  ``TK8S_HSA_CPU_CACHES=1`` (GPU test: tests/test_kernels_gpu.py).

docs/architecture.md ("Start-up shortcuts") lists each with its off-switch.
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


def _env(**kw):
    env = dict(os.environ)
    env.update(PYTHONPATH=str(REPO), TK8S_PYTHON=sys.executable, TK8S_FAKE_GPUS="8")
    env.pop("TK8S_FAULTS", None)
    env.update({k: str(v) for k, v in kw.items()})
    return env


@pytest.fixture
def ws(tmp_path, native_build):
    from tritonk8ssupervisor_amd.orchestrator import init_workspace

    init_workspace(tmp_path)
    for f in ("setup.sh", "tk8s", "kubectl"):
        shutil.copy2(REPO / f, tmp_path / f)
    (tmp_path / "answers.json").write_text(json.dumps({"nodes": 2, "package": "mi355x-1gpu", "confirm": "yes"}))
    yield tmp_path
    subprocess.run(["./setup.sh", "-c", "--yes"], cwd=tmp_path, env=_env(), capture_output=True, timeout=120)


def _cmdline(pid: int) -> str:
    try:
        return Path(f"/proc/{pid}/cmdline").read_bytes().replace(b"\0", b" ").decode()
    except OSError:
        return ""


def test_zygotes_never_handed_their_arguments_are_replaced(ws):
    """The boot hooks skip handing the control plane's and one agent's zygote their arguments
    (fault zygote.no_args): the playbook's daemon tasks find a zygote that would wait forever,
    stop it and start the daemon the plain way -- the cluster still comes up Ready."""
    faults = "zygote.no_args@kubemaster,zygote.no_args@kubenode1"
    r = subprocess.run(["./setup.sh", "--answers", "answers.json", "--yes", "--json", "--port", "0", "--rccl", "off"],
                       cwd=ws, env=_env(TK8S_FAULTS=faults), capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    s = json.loads(r.stdout.strip().splitlines()[-1])
    assert s["nodes"] == 2 and s["nodes_validated"] == 2 and s["gpus_allocatable"] == 2
    machines = ws / ".tk8s" / "machines"
    for m, daemon in (("kubemaster", "controlplane"), ("kubenode1", "agent")):
        run = machines / m / "run"
        assert (run / f"{daemon}.zygote").exists()          # a zygote was started for it ...
        assert not (run / f"{daemon}.args").exists()        # ... and never handed its arguments
        child = json.loads((run / f"{daemon}.pid").read_text())["child"]
        assert "--await-args" not in _cmdline(child), _cmdline(child)  # the running one is a plain start
    # the other agent's zygote was handed its arguments as usual
    assert (machines / "kubenode2" / "run" / "agent.args").exists()
