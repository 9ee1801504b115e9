"""Joyent Triton provider — parity path with the reference (needs the `triton` CLI + network).

Mirrors setup.sh exactly where the reference talks to Triton:
  * env()       : `eval "$(triton env)"` (setup.sh:210)
  * networks()  : `triton networks -oname,id | sort` (setup.sh:257, 536)
  * packages()  : `triton packages -oname,id | grep -- -kvm- | sort` (setup.sh:259, 541)
  * find_key()  : MD5 fingerprint scan of ~/.ssh (setup.sh:215-230)
  * machines    : `triton instance create/delete` (docs/manual-setup.md:10-23)
Not exercised offline (no CLI, no network); the local provider is the tested backend.
"""
from __future__ import annotations

import json
import os
import shutil
import subprocess
from pathlib import Path

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

    def __init__(self, state_dir, **_):
        self.state_dir = Path(state_dir)

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
        return Machine(name=name, id=d.get("id", ""), package=package, networks=list(networks),
                       primaryip=d.get("primaryIp", ""), ips=d.get("ips", []), image=image, tags=dict(tags or {}))

    def exec(self, machine, command, timeout=300, env=None):
        argv = ["ssh", "-o", "StrictHostKeyChecking=no", f"root@{machine.primaryip}", command]
        try:
            r = subprocess.run(argv, capture_output=True, text=True, timeout=timeout, env={**os.environ, **(env or {})})
        except subprocess.TimeoutExpired:
            return 124, "timeout"
        return r.returncode, r.stdout + r.stderr

    def delete_machine(self, machine) -> None:
        _run(["triton", "instance", "delete", "--wait", machine.id or machine.name], timeout=1800)
