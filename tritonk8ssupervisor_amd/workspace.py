"""The bring-up's workspace and the daemon/pod command lines every phase shares.

A workspace is the directory ``./setup.sh`` runs in: the reference's layout (``config``,
``terraform/``, ``ansible/`` with the roles, ``manifests/``) plus ``.tk8s/`` for the state the
reference kept nowhere (phases done, events, machines). ``init_workspace`` copies the templates
into a fresh one; orchestrator.Setup, the fabric check and the kubeadm platform work in it.
"""
from __future__ import annotations

import os
import sys
from pathlib import Path

from .utils.fsutil import atomic_write_json, read_json
from .utils.record import record as dataclass

REPO = Path(__file__).resolve().parents[1]
TEMPLATE_DIRS = ["terraform/master", "terraform/host", "terraform/compat", "ansible/roles", "ansible/group_vars",
                 "manifests"]
TEMPLATE_FILES = ["ansible/ansible.cfg", "ansible/clusterUp.yml", "ansible/clusterUp-kubeadm.yml"]
PHASES = ["configure", "provision", "ansible-config", "ansible", "ready", "rccl"]
PLATFORMS = ("tk8s", "kubeadm")
PLAYBOOKS = {"tk8s": "clusterUp.yml", "kubeadm": "clusterUp-kubeadm.yml"}


class SetupError(RuntimeError):
    def __init__(self, msg: str, code: int = 1):
        super().__init__(msg)
        self.code = code


@dataclass
class Workspace:
    root: Path

    @property
    def config(self) -> Path: return self.root / "config"
    @property
    def tf(self) -> Path: return self.root / "terraform"
    @property
    def ansible(self) -> Path: return self.root / "ansible"
    @property
    def manifests(self) -> Path: return self.root / "manifests"
    @property
    def state_dir(self) -> Path: return self.root / ".tk8s"
    @property
    def state_file(self) -> Path: return self.state_dir / "state.json"
    @property
    def events(self) -> Path: return self.state_dir / "events.jsonl"
    @property
    def env_id_file(self) -> Path: return self.ansible / "tmp" / "kubernetes_environment.id"
    @property
    def vars_file(self) -> Path: return self.ansible / "roles" / "ranchermaster" / "vars" / "vars.yml"
    @property
    def admin_token_file(self) -> Path: return self.state_dir / "admin-token"

    def admin_token(self) -> str | None:
        """The control plane's admin token, as ranchermaster keeps it (controlplane/authn.py)."""
        try:
            return self.admin_token_file.read_text().strip() or None
        except OSError:
            return None

    def state(self) -> dict:
        return read_json(self.state_file, {}) or {}

    def save_state(self, **kw) -> dict:
        st = self.state()
        st.update(kw)
        atomic_write_json(self.state_file, st)
        return st


def init_workspace(dst: str | os.PathLike, src: Path = REPO) -> Workspace:
    """Copy the module/role/manifest templates into a fresh workspace directory."""
    import shutil

    d = Path(dst)
    for rel in TEMPLATE_DIRS:
        if (d / rel).exists():
            shutil.rmtree(d / rel)
        shutil.copytree(src / rel, d / rel, ignore=shutil.ignore_patterns("vars.yml", "__pycache__"))
    for rel in TEMPLATE_FILES:
        (d / rel).parent.mkdir(parents=True, exist_ok=True)
        shutil.copy2(src / rel, d / rel)
    (d / "ansible" / "tmp").mkdir(parents=True, exist_ok=True)
    (d / "ansible" / "roles" / "ranchermaster" / "vars").mkdir(parents=True, exist_ok=True)
    return Workspace(d)


# The daemons start with ``-c 'import <pkg>.__main__'`` rather than ``-m <pkg>``: the same module
# code and sys.argv positions, without runpy/importlib.util (~4 ms per daemon start on the MI355X
# host, on the bring-up's critical path).
CP_ENTRY = "import tritonk8ssupervisor_amd.controlplane.__main__"
AGENT_ENTRY = "import tritonk8ssupervisor_amd.agent.__main__"


def controlplane_argv(bind: str, port: int, advertise: str, state_dir: str, node_grace: float) -> list[str]:
    """The control plane daemon (the ranchermaster role's rancher/server), one definition for the
    role and the master's boot hook."""
    return [sys.executable, "-S", "-c", CP_ENTRY, "--host", bind, "--port", str(port),
            "--advertise", advertise, "--state-dir", state_dir, "--node-grace", str(node_grace)]


def agent_standby_argv(name: str, ip: str) -> list[str]:
    """The node agent in standby (rocmsetup's "Start the node agent in standby" task spells out
    the same argv), waiting for play 3's registration URL."""
    return [sys.executable, "-S", "-c", AGENT_ENTRY, "--await-url", "run/registration-url",
            "--name", name, "--ip", ip]


def validation_pod_command(command: list[str], result: str = "$(TK8S_MACHINE_DIR)/run/gpu-burnin.json") -> list[str]:
    """The validation DaemonSet pod: reuse the node's burn-in result, probe only without one.
    With the real probe the reuse runs in tk8s-reuse, which loads no ROCm library."""
    from .ops import BIN

    reuse = BIN / "tk8s-reuse"
    if not os.environ.get("TK8S_FAKE_GPUS") and reuse.exists():
        return pod_portable([str(reuse), result, "--", *command])
    return pod_portable([*command, "--reuse", result])


def pod_portable(argv: list[str]) -> list[str]:
    """A pod command in terms of the NODE's tk8s install: the agent expands $(TK8S_HOME) and
    $(TK8S_PYTHON) (Kubernetes $(VAR) syntax) to its own install root and interpreter, so one
    DaemonSet/Job spec runs on colocated sandboxes and on remote machines alike."""
    out = []
    for a in argv:
        a = str(a)
        if a == sys.executable:
            out.append("$(TK8S_PYTHON)")
        else:
            out.append(a.replace(str(REPO), "$(TK8S_HOME)"))
    return out
