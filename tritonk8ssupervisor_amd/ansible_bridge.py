"""The tk8s playbook modules as real Ansible modules (``ansible/library/tk8s_*.py``).

``ansible-playbook`` executes a module ON the target machine. The files in ansible/library/ are
thin AnsibleModule front ends: they find the machine's tk8s install (the ``tk8s_home`` argument,
``$TK8S_HOME``, or the newest ``~/.tk8s/dist/<digest>`` the providers push), then call the very
implementation the in-repo engine runs (playbook_modules.MODULES) with a LocalExecutor over the
one machine they are on -- so both runners share one semantics by construction, not by a second
copy of the logic.

Argument specs live here (ARG_SPECS) and are pinned by tests/test_ansible_library.py against
every argument the shipped roles pass.
"""
from __future__ import annotations

import os
import socket
import sys
from pathlib import Path
from types import SimpleNamespace

_COMMON = {
    "machine_dir": {"type": "path"},   # the machine's work dir (host var tk8s_machine_dir)
    "gpus": {"type": "str", "default": ""},  # its GPU ordinals, comma separated (host var tk8s_gpus)
    "tk8s_home": {"type": "path"},     # the tk8s install on the machine (host var tk8s_home)
    "machine": {"type": "str"},        # the machine's name (default: the inventory hostname env)
}

ARG_SPECS: dict[str, dict] = {
    "tk8s_daemon": {
        "name": {"type": "str", "required": True},
        "state": {"type": "str", "default": "started", "choices": ["started", "stopped", "query"]},
        "argv": {"type": "list", "elements": "str"},
        "cmd": {"type": "str"},
        "env": {"type": "dict", "default": {}},
        "restart_policy": {"type": "str", "default": "unless-stopped",
                           "choices": ["no", "on-failure", "always", "unless-stopped"]},
        "wait_for_log": {"type": "str"},
        "timeout": {"type": "float", "default": 300.0},
        **_COMMON,
    },
    "tk8s_burnin": {
        "command": {"type": "list", "elements": "str", "required": True},
        "out": {"type": "str", "default": "run/gpu-burnin.json"},
        "name": {"type": "str", "default": "gpu-burnin"},
        **_COMMON,
    },
    "tk8s_gpu_facts": dict(_COMMON),
    "tk8s_build": {"tk8s_home": {"type": "path"}},
    "tk8s_kube": {
        "api": {"type": "str", "required": True},
        "project": {"type": "str", "required": True},
        "token": {"type": "str", "no_log": True},
        "state": {"type": "str", "default": "present", "choices": ["present", "absent", "wait"]},
        "definition": {"type": "raw"},
        "src": {"type": "path"},
        "vars": {"type": "dict", "default": {}},
        "timeout": {"type": "float", "default": 300.0},
        "tk8s_home": {"type": "path"},
    },
}


def find_home(explicit: str | None = None) -> str | None:
    for cand in (explicit, os.environ.get("TK8S_HOME")):
        if cand and (Path(cand) / "tritonk8ssupervisor_amd").is_dir():
            return str(cand)
    dists = sorted((Path.home() / ".tk8s" / "dist").glob("*/tritonk8ssupervisor_amd"), key=lambda p: p.stat().st_mtime)
    return str(dists[-1].parent) if dists else None


class _OneMachine:
    """A provider for exactly the machine the module runs on (colocated: spawn directly)."""

    colocated = True

    def __init__(self, m):
        self.m = m

    def machine_env(self, m) -> dict:
        return {"TK8S_MACHINE": m.name, "TK8S_MACHINE_DIR": m.sandbox, "TK8S_MACHINE_IP": m.primaryip,
                "TK8S_MACHINE_GPUS": ",".join(map(str, m.gpus)), "TK8S_MACHINE_PACKAGE": m.package}

    def exec(self, m, command, timeout=300, env=None, stdin=None):
        import subprocess

        r = subprocess.run(["bash", "-c", command], cwd=m.sandbox, env={**os.environ, **self.machine_env(m), **(env or {})},
                           input=stdin or b"", capture_output=True, timeout=timeout)
        return r.returncode, (r.stdout or b"").decode(errors="replace") + (r.stderr or b"").decode(errors="replace")


def run(module_name: str, params: dict, check_mode: bool) -> dict:
    """Run one tk8s module on this machine; returns the Ansible result dict."""
    from .executor import LocalExecutor
    from .playbook_modules import run_module
    from .provider.base import Machine

    p = dict(params)
    name = p.pop("machine", None) or os.environ.get("TK8S_MACHINE") or socket.gethostname()
    mdir = p.pop("machine_dir", None) or os.environ.get("TK8S_MACHINE_DIR") or os.getcwd()
    gpus = [int(g) for g in str(p.pop("gpus", "") or os.environ.get("TK8S_MACHINE_GPUS", "")).split(",") if g.strip()]
    p.pop("tk8s_home", None)
    p = {k: v for k, v in p.items() if v is not None}
    Path(mdir).mkdir(parents=True, exist_ok=True)
    m = Machine(name=name, id=name, package="", networks=[], primaryip=os.environ.get("TK8S_MACHINE_IP", "127.0.0.1"),
                gpus=gpus, sandbox=str(mdir))
    ex = LocalExecutor(_OneMachine(m), {name: m})
    ctx = SimpleNamespace(executor=ex, dir=Path(mdir))
    target = SimpleNamespace(name=name, address=m.primaryip)
    return run_module(module_name, p, ctx=ctx, host=target, target=target, local=False, env={}, check=check_mode,
                      variables={})


# ---- ansible/library/<module>.py, generated -------------------------------------------------
# Ansible needs one file per module; every one is the same front end, rendered from LIBRARY_TEMPLATE
# (``python -m tritonk8ssupervisor_amd.ansible_bridge --write-library``; tests/test_ansible_library.py
# checks the shipped files are exactly this output).
SHORT_DESCRIPTIONS = {
    "tk8s_build": "Build the tk8s native validation stack for gfx950 in place (replaces the docker-engine install)",
    "tk8s_burnin": "Start the early GPU burn-in on this machine's MI355X GPUs (one-shot daemon, result shared with the validation pod)",
    "tk8s_daemon": "Start, stop or query a supervised long-running process on this machine (the reference's docker_container rancher/server and docker run rancher/agent)",
    "tk8s_gpu_facts": "ROCm / KFD / GPU facts of this machine, read from sysfs without initialising the GPU (replaces the docker --version probe)",
    "tk8s_kube": "Create, delete or wait for Kubernetes objects through the tk8s control plane",
}

LIBRARY_TEMPLATE = '''#!/usr/bin/python
# -*- coding: utf-8 -*-
# GENERATED by tritonk8ssupervisor_amd/ansible_bridge.py (--write-library): edit the template there.
"""Ansible module {name}: {short}.

Real-Ansible front end of the in-repo playbook engine's module of the same name: it runs on the
target machine, finds that machine's tk8s install ($TK8S_HOME, or the newest ~/.tk8s/dist/<digest>
the baremetal/triton providers push) and calls the shared implementation
(tritonk8ssupervisor_amd/ansible_bridge.py -> playbook_modules.py). Arguments: ansible_bridge.ARG_SPECS.
"""
import glob
import os
import sys

DOCUMENTATION = r"""
module: {name}
short_description: {short}
description: see tritonk8ssupervisor_amd/ansible_bridge.py (ARG_SPECS) and playbook_modules.py
"""


def _home():
    cands = [os.environ.get("TK8S_HOME", "")]
    cands += sorted(glob.glob(os.path.expanduser("~/.tk8s/dist/*")), key=os.path.getmtime, reverse=True)
    for c in cands:
        if c and os.path.isdir(os.path.join(c, "tritonk8ssupervisor_amd")):
            return c
    return None


if __name__ == "__main__":
    home = _home()
    if home and home not in sys.path:
        sys.path.insert(0, home)
    from tritonk8ssupervisor_amd.ansible_bridge import main

    main("{name}")
'''


def library_sources() -> dict[str, str]:
    """{module name: the text of ansible/library/<name>.py}, one per ARG_SPECS entry."""
    return {n: LIBRARY_TEMPLATE.format(name=n, short=SHORT_DESCRIPTIONS[n]) for n in sorted(ARG_SPECS)}


def write_library(directory: str | os.PathLike) -> list[str]:
    out = []
    for name, text in library_sources().items():
        p = Path(directory) / f"{name}.py"
        p.write_text(text)
        p.chmod(0o755)
        out.append(str(p))
    return out


def main(module_name: str) -> None:
    """Entry point of ansible/library/<module_name>.py (after it put the tk8s install on sys.path)."""
    from ansible.module_utils.basic import AnsibleModule  # provided by Ansible on the target

    module = AnsibleModule(argument_spec=ARG_SPECS[module_name], supports_check_mode=True)
    try:
        res = run(module_name, module.params, module.check_mode)
    except Exception as e:  # noqa: BLE001 - a module failure is a task failure
        module.fail_json(msg=f"{module_name}: {type(e).__name__}: {e}")
        return
    if res.get("failed"):
        module.fail_json(**{k: v for k, v in res.items() if k != "failed"})
    else:
        module.exit_json(**res)


def bootstrap(module_name: str, argv_home: str | None = None) -> None:
    """Shared prologue of the library files: locate the install, import, run."""
    home = find_home(argv_home)
    if home and home not in sys.path:
        sys.path.insert(0, home)
    main(module_name)


if __name__ == "__main__" and "--write-library" in sys.argv:
    for f in write_library(Path(__file__).resolve().parents[1] / "ansible" / "library"):
        print(f)
