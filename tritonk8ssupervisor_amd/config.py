"""Cluster configuration: defaults, ``./config`` KEY=value persistence and environment export.

Reference behaviour (setup.sh):
  * setVarDefaults    setup.sh:240-254  — defaults; ANSIBLE_HOST_KEY_CHECKING=False
  * setConfigToFile   setup.sh:199-208  — appends 8 KEY=value lines
  * exportVars        setup.sh:543-549  — exports every non-blank line
The key names are kept so an existing ``config`` file reads the same; values are quoted the
reference's way (strings in double quotes). Writes are atomic instead of ``>>`` appends.
"""
from __future__ import annotations

import os
import shlex
from pathlib import Path

from .utils.fsutil import atomic_write
from .utils.record import asdict, field, fields, record as dataclass

# Reference defaults (setup.sh:245-252); package/network defaults are provider-resolved.
DEFAULT_NAME = "k8s dev"
DEFAULT_MASTER = "kubemaster"
DEFAULT_NODE_PREFIX = "kubenode"
DEFAULT_NODES = 1
MAX_NODES = 9  # setup.sh:297 "HARD LIMIT: 1-9 nodes allowed only since this setup has no HA"

# Order in which keys are written (reference order: setup.sh:253, 211-213, 218, 200-207).
KEY_ORDER = [
    "ANSIBLE_HOST_KEY_CHECKING",
    "SDC_URL",
    "SDC_ACCOUNT",
    "SDC_KEY_ID",
    "SDC_KEY",
    "RANCHER_MASTER_NETWORKS",
    "KUBERNETES_NODE_NETWORKS",
    "KUBERNETES_NUMBER_OF_NODES",
    "KUBERNETES_NAME",
    "KUBERNETES_DESCRIPTION",
    "RANCHER_MASTER_HOSTNAME",
    "KUBERNETES_NODE_HOSTNAME_BEGINSWITH",
    "HOST_PACKAGE",
    "TK8S_BACKEND",
    "TK8S_MASTER_PORT",
    "TK8S_PLATFORM",
]
QUOTED = {
    "SDC_URL", "SDC_ACCOUNT", "SDC_KEY_ID", "SDC_KEY", "KUBERNETES_NAME", "KUBERNETES_DESCRIPTION",
    "RANCHER_MASTER_HOSTNAME", "KUBERNETES_NODE_HOSTNAME_BEGINSWITH", "HOST_PACKAGE",
}


@dataclass
class ClusterConfig:
    ANSIBLE_HOST_KEY_CHECKING: str = "False"
    SDC_URL: str = ""
    SDC_ACCOUNT: str = ""
    SDC_KEY_ID: str = ""
    SDC_KEY: str = ""
    RANCHER_MASTER_NETWORKS: str = ""
    KUBERNETES_NODE_NETWORKS: str = ""
    KUBERNETES_NUMBER_OF_NODES: int = DEFAULT_NODES
    KUBERNETES_NAME: str = DEFAULT_NAME
    KUBERNETES_DESCRIPTION: str = DEFAULT_NAME
    RANCHER_MASTER_HOSTNAME: str = DEFAULT_MASTER
    KUBERNETES_NODE_HOSTNAME_BEGINSWITH: str = DEFAULT_NODE_PREFIX
    HOST_PACKAGE: str = ""
    TK8S_BACKEND: str = "local"
    TK8S_MASTER_PORT: int = 8080
    TK8S_PLATFORM: str = "tk8s"   # tk8s (in-repo control plane + node agents) | kubeadm (real Kubernetes)
    extra: dict = field(default_factory=dict)

    # ---- derived ---------------------------------------------------------------------
    def node_names(self) -> list[str]:
        """Worker hostnames <prefix><i>, i = 1..N (setup.sh:148-152)."""
        return [f"{self.KUBERNETES_NODE_HOSTNAME_BEGINSWITH}{i}" for i in range(1, int(self.KUBERNETES_NUMBER_OF_NODES) + 1)]

    def master_networks(self) -> list[str]:
        return [n for n in self.RANCHER_MASTER_NETWORKS.split(",") if n]

    def node_networks(self) -> list[str]:
        return [n for n in self.KUBERNETES_NODE_NETWORKS.split(",") if n]

    def as_env(self) -> dict[str, str]:
        """What exportVars (setup.sh:543-549) would put in the environment."""
        d = {k: str(v) for k, v in asdict(self).items() if k != "extra"}
        d.update({k: str(v) for k, v in self.extra.items()})
        return d


def _fmt(key: str, value) -> str:
    v = str(value)
    if key in QUOTED:
        return f'{key}="{v.replace(chr(34), "")}"'
    return f"{key}={v}"


def render_config(cfg: ClusterConfig) -> str:
    lines = [_fmt(k, getattr(cfg, k)) for k in KEY_ORDER]
    lines += [_fmt(k, v) for k, v in sorted(cfg.extra.items())]
    return "\n".join(lines) + "\n"


def write_config(path: str | os.PathLike, cfg: ClusterConfig) -> None:
    atomic_write(path, render_config(cfg))


def parse_config_text(text: str) -> dict[str, str]:
    """Parse KEY=value lines (blank lines dropped, quotes stripped like `export "$line"`)."""
    out: dict[str, str] = {}
    for raw in text.splitlines():
        line = raw.strip()
        if not line or line.startswith("#") or "=" not in line:
            continue
        k, v = line.split("=", 1)
        k = k.strip()
        v = v.strip()
        if len(v) >= 2 and v[0] == v[-1] and v[0] in "\"'":
            v = v[1:-1]
        out[k] = v
    return out


def read_config(path: str | os.PathLike) -> ClusterConfig:
    kv = parse_config_text(Path(path).read_text())
    return config_from_dict(kv)


def config_from_dict(kv: dict) -> ClusterConfig:
    cfg = ClusterConfig()
    names = {f.name for f in fields(ClusterConfig)} - {"extra"}
    for k, v in kv.items():
        if k in names:
            cur = getattr(cfg, k)
            setattr(cfg, k, int(v) if isinstance(cur, int) and not isinstance(cur, bool) else str(v))
        else:
            cfg.extra[k] = str(v)
    return cfg


def export_vars(cfg: ClusterConfig, environ: dict | None = None) -> dict:
    env = os.environ if environ is None else environ
    env.update(cfg.as_env())
    return env


def shell_exports(cfg: ClusterConfig) -> str:
    """`export K=V` lines for shells (the tk8s env command)."""
    return "".join(f"export {k}={shlex.quote(v)}\n" for k, v in cfg.as_env().items())
