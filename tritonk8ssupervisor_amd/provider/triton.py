"""Joyent Triton provider — parity path with the reference (needs the `triton` CLI + network).

Mirrors setup.sh exactly where the reference talks to Triton:
  * env()       : `eval "$(triton env)"` (setup.sh:210)
  * networks()  : `triton networks -oname,id | sort` (setup.sh:257, 536)
  * packages()  : `triton packages -oname,id | grep -- -kvm- | sort` (setup.sh:259, 541)
  * find_key()  : MD5 fingerprint scan of ~/.ssh (setup.sh:215-230)
  * machines    : `triton instance create/delete` (docs/manual-setup.md:10-23)
  * exec        : ssh as root with the discovered key (SDC_KEY) and a per-cluster known-hosts
                  file -- the reference's `ssh -o StrictHostKeyChecking=no root@ip` (setup.sh:72)
                  used no key and trusted any host key (utils/ssh.py); machines are configured
                  remotely by executor.RemoteExecutor, exactly like the baremetal backend.
The CLI half is not exercised offline (no CLI, no network); the SSH half is shared with the
baremetal provider, which the fake-ssh bring-up test covers.
"""
from __future__ import annotations

import json
import os
import shutil
import subprocess
from pathlib import Path

from ..utils import ssh

from .base import Machine, Network, Package, Provider, ProvisionError


def _run(argv: list[str], timeout: float = 600) -> str:
    if not shutil.which(argv[0]):
        raise ProvisionError(f"`{argv[0]}` CLI not found; the triton backend needs it (README prerequisites)")
    r = subprocess.run(argv, capture_output=True, text=True, timeout=timeout)
    if r.returncode != 0:
        raise ProvisionError(f"{' '.join(argv)} failed: {r.stderr.strip()}")
    return r.stdout


def _table(text: str) -> list[tuple[str, str]]:
    rows = []
    for line in text.splitlines():
        parts = line.split()
        if len(parts) >= 2 and not (parts[0] == "NAME" and parts[-1] == "ID"):
            rows.append((parts[0], parts[-1]))
    return sorted(rows)


class TritonProvider(Provider):
    name = "triton"
    default_network = "Joyent-SDC-Public"
    default_package = "k4-highcpu-kvm-7.75G"

    colocated = False

    def __init__(self, state_dir, **_):
        self.state_dir = Path(state_dir)

    def target(self, ip: str) -> ssh.SSHTarget:
        ctl = ssh.control_dir_for(self.state_dir)
        return ssh.SSHTarget(host=ip, user="root", key=os.environ.get("SDC_KEY", ""),
                             known_hosts=str(self.state_dir / "known_hosts"), control_dir=str(ctl))

    def env(self) -> dict[str, str]:
        out = {}
        for line in _run(["triton", "env"]).splitlines():
            line = line.strip()
            if line.startswith("export ") and "=" in line:
                k, v = line[len("export "):].split("=", 1)
                out[k] = v.strip('"')
        return {k: out.get(k, "") for k in ("SDC_URL", "SDC_ACCOUNT", "SDC_KEY_ID")}

    def find_key(self, key_id: str) -> str | None:
        ssh = Path("~/.ssh").expanduser()
        for f in sorted(ssh.glob("*")):
            base = f.with_suffix("") if f.suffix == ".pub" else f
            for args in (["ssh-keygen", "-E", "md5", "-lf", str(base)], ["ssh-keygen", "-l", "-f", str(base)]):
                try:
                    r = subprocess.run(args, capture_output=True, text=True, timeout=10)
                except (OSError, subprocess.TimeoutExpired):
                    continue
                parts = r.stdout.split()
                if len(parts) > 1 and parts[1].removeprefix("MD5:") == key_id:
                    return str(base)
        return None

    def networks(self) -> list[Network]:
        return [Network(n, i, public=(n == self.default_network)) for n, i in _table(_run(["triton", "networks", "-oname,id"]))]

    def packages(self) -> list[Package]:
        rows = [(n, i) for n, i in _table(_run(["triton", "packages", "-oname,id"])) if "-kvm-" in n]
        return [Package(n, i) for n, i in rows]

    def create_machine(self, name, package, networks, image="", root_authorized_keys="", tags=None) -> Machine:
        argv = ["triton", "instance", "create", "--wait", "--json", f"--name={name}"]
        for n in networks:
            argv += ["-N", n]
        for k, v in (tags or {}).items():
            argv += ["-t", f"{k}={v}"]
        argv += [image or "ubuntu-certified-16.04", package]
        d = json.loads(_run(argv, timeout=1800).splitlines()[-1])
        ip = d.get("primaryIp", "")
        # The VM's node runtime: the tk8s distribution (tar over ssh, once) and the machine's work
        # dir, like the baremetal backend. ssh retries while the VM is still booting.
        t = self.target(ip)
        rc, home, out = ssh.push_dist(t, Path(__file__).resolve().parents[2])
        if rc != 0:
            raise ProvisionError(f"{name}: installing tk8s over ssh failed (rc={rc}): {out.strip()[-400:]}")
        rc, out = ssh.run(t, "mkdir -p tk8s/machine && cd tk8s/machine && mkdir -p run logs pods etc && pwd "
                             "&& command -v python3")
        if rc != 0:
            raise ProvisionError(f"{name}: preparing the machine failed: {out.strip()[-400:]}")
        sandbox, py = out.strip().splitlines()[-2:]
        return Machine(name=name, id=d.get("id", ""), package=package, networks=list(networks), primaryip=ip,
                       ips=d.get("ips", []), image=image, tags=dict(tags or {}), sandbox=sandbox, home=home, python=py)

    def machine_env(self, m: Machine) -> dict[str, str]:
        return {"TK8S_MACHINE": m.name, "TK8S_MACHINE_DIR": m.sandbox, "TK8S_MACHINE_IP": m.primaryip,
                "TK8S_MACHINE_GPUS": ",".join(map(str, m.gpus)), "TK8S_MACHINE_PACKAGE": m.package,
                "TK8S_HOME": m.home}

    def ansible_host_vars(self, m: Machine) -> dict:
        """Inventory variables that let a stock ansible-playbook reach and use this machine the way
        the in-repo engine does (ssh user/port/key, known-hosts policy, the node's tk8s install)."""
        t = self.target(m.primaryip)
        hv = {"ansible_user": t.user, "ansible_port": t.port, "tk8s_home": m.home, "tk8s_machine_dir": m.sandbox,
              "tk8s_gpus": ",".join(map(str, m.gpus)),
              "ansible_python_interpreter": m.python or "python3"}
        if t.key:
            hv["ansible_ssh_private_key_file"] = os.path.expanduser(t.key)
        if t.known_hosts:
            hv["ansible_ssh_common_args"] = f"-o UserKnownHostsFile={t.known_hosts} -o StrictHostKeyChecking=accept-new"
        return hv

    def exec(self, machine, command, timeout=300, env=None, stdin=None):
        script = ssh.remote_script(command, cwd=machine.sandbox or None, env={**self.machine_env(machine), **(env or {})})
        return ssh.run(self.target(machine.primaryip), script, timeout=timeout, stdin=stdin, retries_on_connect=5)

    def delete_machine(self, machine) -> None:
        _run(["triton", "instance", "delete", "--wait", machine.id or machine.name], timeout=1800)
        subprocess.run(["ssh-keygen", "-R", machine.primaryip, "-f", str(self.state_dir / "known_hosts")],
                       capture_output=True, timeout=30)  # the reference's `ssh-keygen -R` (setup.sh:504-508)
