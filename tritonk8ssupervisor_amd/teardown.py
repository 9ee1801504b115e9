"""``./setup.sh -c``: cleanRunner (reference setup.sh:484-521) -- confirm, destroy the
machines, reset the configuration. Also removes what the reference left behind (the env-id file,
W13 bug), stops a host burn-in or control-plane zygote an interrupted bring-up left running, and
on the kubeadm platform undoes kubeadm on every machine first.
"""
from __future__ import annotations

import os
import sys

from .config import read_config
from .provider import get_provider
from .provision import Engine
from .utils.fsutil import remove_paths
from .utils.procs import kill_pidfile
from .workspace import Workspace


def clean(ws: Workspace, *, assume_yes: bool = False, inp=None, out=print,
          backend: str | None = None) -> int:
    """cleanRunner (setup.sh:484-521), non-destructive unless confirmed."""
    inp = inp or sys.stdin
    out("Clearing settings....")
    masters, hosts_ = ws.tf / "masters.ip", ws.tf / "hosts.ip"
    while True:
        if masters.exists():
            out("WARNING: You are about to destroy the following machines associated with the cluster:")
            for f in (masters, hosts_):
                if f.exists():
                    out(f.read_text().rstrip())
            q = "Do you wish to destroy the machines and reset configuration (yes | no)? "
        else:
            q = "Do you wish to reset configuration (yes | no)? "
        if assume_yes:
            yn = "yes"
        else:
            sys.stdout.write(q)
            sys.stdout.flush()
            yn = (inp.readline() or "no").strip()
        if yn == "no":
            return 0
        if yn == "yes":
            break
        out("Please answer yes or no.")
    backend = backend or (read_config(ws.config).TK8S_BACKEND if ws.config.exists() else os.environ.get("TK8S_BACKEND", "local"))
    provider = get_provider(backend, ws.state_dir)
    from .burnin import stop_host_burnin

    stop_host_burnin(ws.state_dir)
    if ws.config.exists() and read_config(ws.config).TK8S_PLATFORM == "kubeadm":
        from .kubeadm_platform import kubeadm_reset

        kubeadm_reset(ws, provider, out)
    if (ws.tf / "rancher.tf").exists() or (ws.tf / "terraform.tfstate").exists():
        out("    destroying machines...")
        try:
            Engine(ws.tf, provider).destroy()
        except Exception as e:  # noqa: BLE001 - keep cleaning
            out(f"    warning: destroy: {e}")
    if hasattr(provider, "list_machines"):  # leftovers of an interrupted apply
        for m in provider.list_machines():
            provider.delete_machine(m)
    # A machine sandbox no allocation lists any more can still hold a live process: the control
    # plane zygote started with the CLI of a bring-up that failed before its master existed.
    for pidfile in sorted((ws.state_dir / "machines").glob("*/run/*.pid")):
        kill_pidfile(pidfile, grace=1.0)
    remove_paths([ws.tf / n for n in ("hosts.ip", "masters.ip", "rancher.tf", "terraform.tfstate", ".tfstate.lock",
                                      "hosts.ip.lock", "masters.ip.lock", ".terraform")]
                 + list(ws.tf.glob("terraform.tfstate*")))
    if (ws.ansible / "ansible.cfg").exists():
        from .orchestrator import _set_ini_value

        _set_ini_value(ws.ansible / "ansible.cfg", "private_key_file", "")
    remove_paths([ws.ansible / "hosts", ws.vars_file, *ws.ansible.glob("*.retry"), *(p for p in (ws.ansible / "tmp").glob("*") if not p.name.startswith(".")),
                  ws.config, ws.state_dir / "machines", ws.state_dir / "alloc.json", ws.state_dir / "alloc.lock",
                  ws.state_dir / "state.json", ws.state_dir / "kubeconfig.json", ws.state_dir / "ansible.log",
                  ws.admin_token_file])
    out("    All clear!")
    return 0
