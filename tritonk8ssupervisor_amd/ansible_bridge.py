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

# What ansible-doc shows for each option (the generated DOCUMENTATION's ``options``; the types,
# defaults, choices and required flags come from ARG_SPECS itself).
OPTION_DOCS = {
    "machine_dir": "The machine's work directory (its sandbox; host var C(tk8s_machine_dir)).",
    "gpus": "The machine's GPU ordinals on the host, comma separated (host var C(tk8s_gpus)); empty for a CPU-only machine.",
    "tk8s_home": "The tk8s install on the machine (default C($TK8S_HOME), else the newest C(~/.tk8s/dist/<digest>) a provider pushed).",
    "machine": "The machine's name (default C($TK8S_MACHINE), else the host name).",
    "name": "The daemon's name on this machine: its pidfile is C(run/<name>.pid), its log C(logs/<name>.log).",
    "state": "What to do: start it (idempotent), stop it, or only report whether it runs.",
    "argv": "The daemon's command as a list (no shell).",
    "cmd": "The daemon's command as one shell string (when I(argv) is not given).",
    "env": "Extra environment of the daemon, on top of the machine's C(TK8S_MACHINE*) variables.",
    "restart_policy": "Restarts by C(tk8s-supervise), as Docker's restart policies (C(no): run it unsupervised).",
    "wait_for_log": "Return only once the daemon's log has this text (the reference waited for rancher/server's C(Listening on)).",
    "timeout": "Seconds to wait (for I(wait_for_log), or for the objects' readiness with C(state=wait)).",
    "command": "The burn-in probe's command (C(tk8s-hsaprobe) / C(tk8s-probe) and its arguments; the machine's GPUs are appended).",
    "out": "Where the burn-in writes its JSON result, relative to the machine directory; the validation pod reads it once.",
    "api": "The control plane's base URL (C(http://<master>:<port>)).",
    "project": "The environment (Rancher project) id whose Kubernetes API receives the objects.",
    "token": "The control plane's admin token (or the environment's API token).",
    "definition": "The objects, inline: one mapping or a list of them.",
    "src": "A manifest file (YAML, several documents allowed; Jinja2 variables from I(vars)).",
    "vars": "Variables for the manifest template in I(src).",
    # per module, where an option means something else there
    ("tk8s_kube", "state"): "C(present): create the objects or update them; C(absent): delete them; C(wait): until "
                            "they are ready.",
    ("tk8s_kube", "timeout"): "Seconds to wait for the objects' readiness with C(state=wait).",
    ("tk8s_burnin", "name"): "The burn-in's name on this machine: its pidfile is C(run/<name>.pid).",
    ("tk8s_daemon", "timeout"): "Seconds to wait for I(wait_for_log).",
}
# (module, state) -> what ansible-doc shows: examples from the shipped roles, and the results
MODULE_EXAMPLES = {
    "tk8s_build": """- name: Build the native validation stack once (hipcc, gfx950)
  tk8s_build:
  run_once: true
  delegate_to: localhost
  when: not tk8s_native_built""",
    "tk8s_burnin": """- name: Start the GPU burn-in on this machine's MI355X GPUs (background)
  tk8s_burnin:
    command: "{{ tk8s_validation_command }}"
    out: run/gpu-burnin.json
    machine_dir: "{{ tk8s_machine_dir }}"
    gpus: "{{ tk8s_gpus }}"
""",
    "tk8s_daemon": """- name: Start the control plane (restart policy unless-stopped)
  tk8s_daemon:
    name: controlplane
    argv: ["{{ tk8s_python }}", "-S", "-c", "import tritonk8ssupervisor_amd.controlplane.__main__",
           "--host", "{{ tk8s_bind }}", "--port", "{{ tk8s_master_port }}"]
    restart_policy: unless-stopped
    wait_for_log: Listening on
    machine_dir: "{{ tk8s_machine_dir }}"
""",
    "tk8s_gpu_facts": """- name: Gather ROCm / GPU facts for this machine
  tk8s_gpu_facts:
    machine_dir: "{{ tk8s_machine_dir }}"
    gpus: "{{ tk8s_gpus }}"
- assert:
    that: [tk8s_rocm_version != '', tk8s_kfd]""",
    "tk8s_kube": """- name: Deploy the GPU validation DaemonSet (tk8s-probe on every MI355X worker)
  tk8s_kube:
    api: "http://{{ master }}:{{ tk8s_master_port }}"
    project: "{{ kubernetes_environment_id }}"
    token: "{{ tk8s_admin_token }}"
    src: "{{ tk8s_manifests }}/gpu-validation-daemonset.yaml"
""",
}
MODULE_RETURNS = {
    "tk8s_build": {"changed": "whether any artefact was rebuilt", "seconds": "how long the build took"},
    "tk8s_burnin": {"gpus": "the GPU ordinals the burn-in validates", "out": "the result file, relative to the machine directory",
                    "pid": "the burn-in process"},
    "tk8s_daemon": {"running": "whether the daemon runs after the task", "pid": "its process id",
                    "log": "its log file", "wait_seconds": "how long I(wait_for_log) waited"},
    "tk8s_gpu_facts": {"ansible_facts": "tk8s_rocm_version, tk8s_kfd, tk8s_host_gpus, tk8s_inventory_source, "
                                        "tk8s_native_built, tk8s_node_python, tk8s_node_kernel, tk8s_machine_gpus"},
    "tk8s_kube": {"objects": "per object: kind, name, namespace and whether it was created",
                  "deleted": "how many objects C(state=absent) deleted"},
}


def documentation(name: str) -> str:
    """The module's DOCUMENTATION block (YAML, what ansible-doc reads), from ARG_SPECS + OPTION_DOCS."""
    import json

    lines = [f"module: {name}", f"short_description: {SHORT_DESCRIPTIONS[name]}",
             "description:", "  - Runs the same implementation as the tk8s playbook engine "
             "(tritonk8ssupervisor_amd/playbook_modules.py) on the target machine.", "options:"]
    for opt, spec in sorted(ARG_SPECS[name].items()):
        lines.append(f"  {opt}:")
        lines.append(f"    description: {json.dumps(OPTION_DOCS.get((name, opt), OPTION_DOCS.get(opt, opt)))}")
        lines.append(f"    type: {spec['type']}")
        if spec.get("elements"):
            lines.append(f"    elements: {spec['elements']}")
        if spec.get("required"):
            lines.append("    required: true")
        if "default" in spec:
            lines.append(f"    default: {json.dumps(spec['default'])}")
        if spec.get("choices"):
            lines.append(f"    choices: {json.dumps(spec['choices'])}")
    lines.append("author: tk8s")
    return "\n".join(lines)


def returns(name: str) -> str:
    import json

    return "\n".join(f"{k}:\n  description: {json.dumps(v)}\n  returned: success" for k, v in MODULE_RETURNS[name].items())


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
{documentation}
"""

EXAMPLES = r"""
{examples}
"""

RETURN = r"""
{returns}
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
    return {n: LIBRARY_TEMPLATE.format(name=n, short=SHORT_DESCRIPTIONS[n], documentation=documentation(n),
                                       examples=MODULE_EXAMPLES[n].rstrip(), returns=returns(n)) for n in sorted(ARG_SPECS)}


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
