"""Bare-metal provider: machines on real hosts reached over SSH (BASELINE.json: "Joyent -> local
bare-metal").

The reference's substrate is Triton CloudAPI: ``triton_machine`` resources created by Terraform
(terraform/master/main.tf:1-11), bootstrapped over SSH (:13-27) and configured by Ansible as
root over SSH (ansible/clusterUp.yml). On bare metal nothing is created: the hosts exist and are
listed in an inventory; a "machine" is a claimed slice of one host -- a work directory under the
SSH user's home plus an exclusive set of that host's GPUs (the package shape) -- so one 8x MI355X
host can carry 1 master + 8 one-GPU workers, and a rack of hosts works the same way.

Inventory (YAML or JSON; ``TK8S_INVENTORY`` or ``<workdir>/inventory.yml``; a copy is kept in the
state dir so teardown works after the file moved)::

    ssh: {user: root, key: ~/.ssh/id_ed25519, port: 22}   # defaults for every host
    workdir: tk8s                  # per-host root of the machines, relative to the login home
    python: python3                # interpreter on the hosts
    networks: [{name: fabric}]     # extra networks (each host's ``addresses`` map names -> IPs)
    hosts:
      - name: mi355x-a
        address: 10.0.0.5          # ssh address and default IP of its machines
        gpus: 8                    # count (ordinals 0..7) or an explicit list
        role: master               # optional: where the master machine goes (default: first host)
        ssh: {port: 2222}          # per-host overrides

Machine lifecycle over SSH (utils/ssh.py: per-cluster known-hosts, the inventory key, one
multiplexed connection per host):

* create: claim host + GPUs (flock'd ``baremetal-alloc.json``); install the tk8s distribution on
  the host once (tar over ssh into ``~/.tk8s/dist/<digest>``, the image a VM would boot); make the
  machine's work dir; record the absolute paths (``Machine.sandbox/home/python``);
* exec: ``cd <work dir>; export TK8S_MACHINE*...; bash -c CMD`` on the host;
* delete: stop every process group a pidfile under the work dir names, remove it, free the claim.
"""
from __future__ import annotations

import json
import os
import shlex
import threading
from pathlib import Path

from ..utils import ssh
from ..utils.fsutil import atomic_write_json, file_lock, read_json
from . import keys
from .base import Machine, Network, Package, Provider, ProvisionError

_NS = "7b0e2c4a-1f3d-4e5b-8a6c-9d0e1f2a3b4c"
DEFAULT_NETWORK = "baremetal-default"
SHAPES = [1, 2, 4, 8]
REPO = Path(__file__).resolve().parents[2]
_install_locks: dict[str, threading.Lock] = {}
_install_guard = threading.Lock()


def _uid(kind: str, name: str) -> str:
    from ..utils.ids import uuid5

    return uuid5(_NS, f"tk8s/baremetal/{kind}/{name}")


def load_inventory(path: str | os.PathLike) -> dict:
    text = Path(path).read_text()
    if str(path).endswith(".json"):
        inv = json.loads(text)
    else:
        import yaml

        inv = yaml.safe_load(text)
    return normalize_inventory(inv or {})


def normalize_inventory(inv: dict) -> dict:
    hosts = []
    seen = set()
    for i, h in enumerate(inv.get("hosts") or []):
        if isinstance(h, str):
            h = {"address": h}
        addr = str(h.get("address") or h.get("host") or "")
        if not addr:
            raise ProvisionError(f"inventory host #{i + 1} has no address")
        name = str(h.get("name") or addr)
        if name in seen:
            raise ProvisionError(f"inventory host {name!r} listed twice")
        seen.add(name)
        g = h.get("gpus", 0)
        gpus = list(range(int(g))) if isinstance(g, (int, str)) else [int(x) for x in g]
        conn = str(h.get("connection", "ssh"))
        if conn not in ("ssh", "local"):
            raise ProvisionError(f"inventory host {name!r}: connection {conn!r} is not ssh or local")
        hosts.append({"name": name, "address": addr, "gpus": gpus, "role": str(h.get("role", "")),
                      "addresses": {str(k): str(v) for k, v in (h.get("addresses") or {}).items()},
                      "ssh": dict(h.get("ssh") or {}), "connection": conn})
    if not hosts:
        raise ProvisionError("bare-metal inventory lists no hosts")
    nets = [{"name": DEFAULT_NETWORK, "public": True}]
    for n in inv.get("networks") or []:
        n = {"name": n} if isinstance(n, str) else dict(n)
        if n["name"] != DEFAULT_NETWORK:
            nets.append({"name": str(n["name"]), "public": bool(n.get("public", False))})
    return {"ssh": dict(inv.get("ssh") or {}), "workdir": str(inv.get("workdir", "tk8s")),
            "python": str(inv.get("python", "python3")), "dist_root": str(inv.get("dist_root", ".tk8s/dist")),
            "networks": nets, "hosts": hosts}


def primary_ipv4() -> str:
    """This host's primary IPv4 address -- the one its default route leaves from (a UDP
    "connect" sends nothing) -- which kubeadm advertises: 127.0.0.1 would be every pod's own
    loopback. 127.0.0.1 only when the host has no route at all."""
    import socket

    for probe in ("10.255.255.255", "192.0.2.1"):
        s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        try:
            s.connect((probe, 9))
            ip = s.getsockname()[0]
            if ip and not ip.startswith("127."):
                return ip
        except OSError:
            pass
        finally:
            s.close()
    return "127.0.0.1"


def local_host_inventory(state_dir: str | os.PathLike, gpus: int | None = None) -> Path:
    """A one-host inventory naming THIS host, reached without ssh (``connection: local``): the
    kubeadm platform's single-node bring-up run as root on the 8x MI355X box itself -- the
    reference's one command on one machine (/root/reference/setup.sh:8-92) -- with no
    SSH-to-self. Written to ``<state_dir>/local-host-inventory.json``."""
    import socket
    import sys

    if gpus is None:
        env = os.environ.get("TK8S_LOCAL_HOST_GPUS")
        if env:
            gpus = int(env)
        else:
            from ..models.hostinfo import discover

            gpus = discover().count
    name = (socket.gethostname() or "localhost").split(".")[0]
    priv, _pub, _fp = keys.ensure_cluster_key(Path(state_dir) / "keys")  # the wizard's SDC_KEY (no ssh uses it)
    inv = {"hosts": [{"name": name, "address": primary_ipv4(), "gpus": int(gpus), "role": "master",
                      "connection": "local"}], "ssh": {"key": str(priv)},
           "python": sys.executable, "workdir": str(Path(state_dir).resolve() / "host")}
    p = Path(state_dir) / "local-host-inventory.json"
    atomic_write_json(p, inv)
    return p


class BareMetalProvider(Provider):
    name = "baremetal"
    default_network = DEFAULT_NETWORK
    colocated = False

    def __init__(self, state_dir: str | os.PathLike, inventory: str | os.PathLike | None = None, **_):
        self.state_dir = Path(state_dir).resolve()
        self.alloc_file = self.state_dir / "baremetal-alloc.json"
        self.lock_file = self.state_dir / "baremetal-alloc.lock"
        self.cache = self.state_dir / "baremetal-inventory.json"
        self._inventory_path = inventory
        self._inv: dict | None = None

    # ---- inventory -----------------------------------------------------------------------
    def inventory(self) -> dict:
        if self._inv is not None:
            return self._inv
        src = self._inventory_path or os.environ.get("TK8S_INVENTORY")
        if not src:
            for cand in ("inventory.yml", "inventory.yaml", "inventory.json"):
                if (self.state_dir.parent / cand).exists():
                    src = self.state_dir.parent / cand
                    break
        if src:
            inv = load_inventory(Path(src).expanduser())
            inv["source"] = str(Path(src).expanduser().resolve())
            self.state_dir.mkdir(parents=True, exist_ok=True)
            atomic_write_json(self.cache, inv)
        elif self.cache.exists():
            inv = read_json(self.cache)
        else:
            raise ProvisionError("the baremetal backend needs an inventory: set TK8S_INVENTORY or create "
                                 f"{self.state_dir.parent / 'inventory.yml'} (see provider/baremetal.py)")
        self._inv = inv
        return inv

    def _host(self, name: str) -> dict:
        for h in self.inventory()["hosts"]:
            if h["name"] == name:
                return h
        raise ProvisionError(f"host {name!r} is not in the bare-metal inventory")

    def target(self, host: dict) -> ssh.SSHTarget:
        if host.get("connection") == "local":  # the orchestrator's own host (local_host_inventory)
            return ssh.SSHTarget(host=host["address"], local=True)
        inv = self.inventory()
        o = {**inv["ssh"], **host.get("ssh", {})}
        ctl = ssh.control_dir_for(self.state_dir)
        return ssh.SSHTarget(host=host["address"], user=str(o.get("user", "root")), port=int(o.get("port", 22)),
                             key=str(o.get("key", "") or os.environ.get("SDC_KEY", "")),
                             known_hosts=str(o.get("known_hosts") or self.state_dir / "known_hosts"),
                             control_dir="" if os.environ.get("TK8S_SSH_MUX") == "0" else str(ctl),
                             extra_opts=tuple(o.get("options", ())))

    # ---- Provider API ----------------------------------------------------------------------
    def _pubkey(self) -> Path | None:
        key = self.inventory()["ssh"].get("key", "")
        if key and Path(os.path.expanduser(key) + ".pub").exists():
            return Path(os.path.expanduser(key) + ".pub")
        return None

    def env(self) -> dict[str, str]:
        inv = self.inventory()
        pub = self._pubkey()
        fp = keys.key_fingerprint(pub) if pub else None
        if not fp:
            raise ProvisionError("bare-metal inventory: ssh.key must name a private key with its .pub next to it")
        return {"SDC_URL": f"baremetal://{inv.get('source', self.cache)}",
                "SDC_ACCOUNT": str(inv["ssh"].get("user", "root")), "SDC_KEY_ID": fp}

    def find_key(self, key_id: str) -> str | None:
        dirs: list = []
        pub = self._pubkey()
        if pub:
            dirs.append(pub.parent)
        dirs.append("~/.ssh")
        return keys.find_key(key_id, dirs)

    def networks(self) -> list[Network]:
        return sorted((Network(n["name"], _uid("network", n["name"]), public=n["public"])
                       for n in self.inventory()["networks"]), key=lambda x: x.name)

    def packages(self) -> list[Package]:
        most = max(len(h["gpus"]) for h in self.inventory()["hosts"])
        out = [Package("bm-cpu", _uid("package", "bm-cpu"), 0, description="CPU-only slice of a host")]
        for g in SHAPES:
            if g <= most:
                out.append(Package(f"bm-{g}gpu", _uid("package", f"bm-{g}gpu"), g,
                                   description=f"{g}x MI355X (gfx950) slice of a host"))
        return sorted(out, key=lambda p: p.name)

    @property
    def default_package(self) -> str:  # type: ignore[override]
        return "bm-1gpu" if any(h["gpus"] for h in self.inventory()["hosts"]) else "bm-cpu"

    # ---- placement --------------------------------------------------------------------------
    # One machine per host (the kubeadm platform: one kubelet per OS, which owns all the host's
    # GPUs); False = machines are slices of hosts (the tk8s platform's node agents, and the
    # kubeadm platform's single-node mode, whose workers are GPU slots of the one host).
    whole_hosts = False

    def single_host(self) -> bool:
        """The inventory holds one host: the kubeadm platform then runs single-node (control plane
        and GPU worker on that host, kubeadm_platform.py) instead of one kubelet per machine."""
        return len(self.inventory()["hosts"]) == 1

    def _place(self, alloc: dict, name: str, role: str, ngpus: int) -> tuple[dict, list[int]]:
        hosts = self.inventory()["hosts"]
        used: dict[str, set] = {h["name"]: set() for h in hosts}
        load: dict[str, int] = {h["name"]: 0 for h in hosts}
        for rec in alloc.get("machines", {}).values():
            used.setdefault(rec["host"], set()).update(rec.get("gpus", []))
            load[rec["host"]] = load.get(rec["host"], 0) + 1
        if self.whole_hosts:
            free = [h for h in hosts if load[h["name"]] == 0 and len(h["gpus"]) >= ngpus]
            if role == "master":
                free.sort(key=lambda h: (h["role"] != "master", len(h["gpus"])))  # the master host, else the smallest
            if not free:
                raise ProvisionError(f"{name}: every machine needs a host of its own here (one kubelet per host) and no "
                                     f"free host has {ngpus} GPU(s); add hosts to the inventory, or use a one-host "
                                     "inventory (single-node mode: control plane and GPU worker on that host)")
            h = free[0]
            return h, ([] if role == "master" else list(h["gpus"]))
        if role == "master":
            h = next((h for h in hosts if h["role"] == "master"), hosts[0])
            return h, []
        if ngpus == 0:
            h = min(hosts, key=lambda x: (load[x["name"]], hosts.index(x)))
            return h, []
        for h in hosts:  # fill hosts in inventory order (keeps a job's GPUs on one xGMI island)
            free = [g for g in h["gpus"] if g not in used[h["name"]]]
            if len(free) >= ngpus:
                return h, free[:ngpus]
        total = sum(len(h["gpus"]) - len(used[h["name"]]) for h in hosts)
        raise ProvisionError(f"{name}: package needs {ngpus} GPU(s) on one host; {total} free across the inventory "
                             "(the bare-metal analogue of reaching the provisioning limit)")

    def _install(self, host: dict) -> tuple[str, str]:
        """The tk8s distribution and the interpreter path on ``host`` (once per host per run)."""
        with _install_guard:
            lock = _install_locks.setdefault(f"{self.state_dir}:{host['name']}", threading.Lock())
        with lock:
            t = self.target(host)
            rc, home, out = ssh.push_dist(t, REPO, self.inventory().get("dist_root", ".tk8s/dist"))
            if rc != 0:
                raise ProvisionError(f"{host['name']}: installing tk8s over ssh failed (rc={rc}): {out.strip()[-400:]}")
            py = self.inventory().get("python", "python3")
            rc, out = ssh.run(t, f"command -v {shlex.quote(py)}")
            if rc != 0 or not out.strip():
                raise ProvisionError(f"{host['name']}: no {py} on the host (the node runtime needs python3 >= 3.8)")
            return home, out.strip().splitlines()[-1]

    def create_machine(self, name: str, package: str, networks: list[str], image: str = "",
                       root_authorized_keys: str = "", tags: dict | None = None) -> Machine:
        pkg = self.package_by_id_or_name(package)
        nets = [self.network_by_id_or_name(n) for n in networks] or [self.network_by_id_or_name(self.default_network)]
        role = (tags or {}).get("role", "host")
        with file_lock(self.lock_file):
            alloc = read_json(self.alloc_file, {}) or {}
            if name in alloc.get("machines", {}):
                raise ProvisionError(f"machine {name} already exists")
            host, gpus = self._place(alloc, name, role, 0 if role == "master" else pkg.gpus)
            alloc.setdefault("machines", {})[name] = {"host": host["name"], "gpus": gpus, "state": "creating"}
            atomic_write_json(self.alloc_file, alloc)
        try:
            home, py = self._install(host)
            wd = f"{self.inventory()['workdir'].rstrip('/')}/machines/{name}"
            script = (f"mkdir -p {shlex.quote(wd)} && cd {shlex.quote(wd)} && mkdir -p run logs pods etc && "
                      f"printf '%s\\n' {shlex.quote(root_authorized_keys.strip())} > etc/authorized_keys && pwd")
            rc, out = ssh.run(self.target(host), script)
            if rc != 0:
                raise ProvisionError(f"{name}: preparing the machine on {host['name']} failed: {out.strip()[-400:]}")
            sandbox = out.strip().splitlines()[-1]
        except Exception:
            self._release(name)
            raise
        ips = [host["addresses"].get(n.name, host["address"]) for n in nets]
        m = Machine(name=name, id=_uid("machine", f"{host['name']}/{name}"), package=pkg.name,
                    networks=[n.id for n in nets], primaryip=ips[0], ips=ips, gpus=gpus, image=image,
                    tags={**(tags or {}), "tk8s_host": host["name"]}, sandbox=sandbox, home=home, python=py)
        with file_lock(self.lock_file):
            alloc = read_json(self.alloc_file, {}) or {}
            alloc.setdefault("machines", {})[name] = {"host": host["name"], "gpus": gpus, "state": "running",
                                                      "machine": m.to_dict()}
            atomic_write_json(self.alloc_file, alloc)
        return m

    def _release(self, name: str) -> None:
        with file_lock(self.lock_file):
            alloc = read_json(self.alloc_file, {}) or {}
            alloc.get("machines", {}).pop(name, None)
            atomic_write_json(self.alloc_file, alloc)

    def get_machine(self, name: str) -> Machine | None:
        rec = (read_json(self.alloc_file, {}) or {}).get("machines", {}).get(name)
        return Machine.from_dict(rec["machine"]) if rec and rec.get("machine") else None

    def list_machines(self) -> list[Machine]:
        recs = (read_json(self.alloc_file, {}) or {}).get("machines", {})
        return [Machine.from_dict(r["machine"]) for _, r in sorted(recs.items()) if r.get("machine")]

    def machine_env(self, m: Machine) -> dict[str, str]:
        env = {"TK8S_MACHINE": m.name, "TK8S_MACHINE_DIR": m.sandbox, "TK8S_MACHINE_IP": m.primaryip,
               "TK8S_MACHINE_GPUS": ",".join(map(str, m.gpus)), "TK8S_MACHINE_PACKAGE": m.package,
               "TK8S_HOME": m.home}
        if m.tags.get("tk8s_host"):  # the node label tk8s.amd.com/host: which machines share GPUs' host
            env["TK8S_HOST_ID"] = m.tags["tk8s_host"]
        return env

    def _target_of(self, m: Machine) -> ssh.SSHTarget:
        host = m.tags.get("tk8s_host")
        if not host:
            rec = (read_json(self.alloc_file, {}) or {}).get("machines", {}).get(m.name) or {}
            host = rec.get("host")
        if not host:
            raise ProvisionError(f"machine {m.name}: no host recorded")
        return self.target(self._host(host))

    def ansible_host_vars(self, m: Machine) -> dict:
        """Inventory variables that let a stock ansible-playbook reach and use this machine the way
        the in-repo engine does (ssh user/port/key, known-hosts policy, the node's tk8s install)."""
        t = self._target_of(m)
        hv = {"ansible_user": t.user, "ansible_port": t.port, "tk8s_home": m.home, "tk8s_machine_dir": m.sandbox,
              "tk8s_gpus": ",".join(map(str, m.gpus)),
              "ansible_python_interpreter": m.python or "python3"}
        if t.local:
            return {**hv, "ansible_connection": "local"}
        if t.key:
            hv["ansible_ssh_private_key_file"] = os.path.expanduser(t.key)
        if t.known_hosts:
            hv["ansible_ssh_common_args"] = f"-o UserKnownHostsFile={t.known_hosts} -o StrictHostKeyChecking=accept-new"
        return hv

    def exec(self, machine: Machine, command: str, timeout: float = 300, env: dict | None = None,
             stdin: bytes | None = None) -> tuple[int, str]:
        script = ssh.remote_script(command, cwd=machine.sandbox, env={**self.machine_env(machine), **(env or {})})
        return ssh.run(self._target_of(machine), script, timeout=timeout, stdin=stdin)

    def delete_machine(self, machine: Machine) -> None:
        """Stop everything the machine runs (daemons, pods: every pidfile's process group), remove
        its work dir, free its GPUs. Unreachable hosts keep their claim (so the GPUs are not handed
        out twice) and the error surfaces."""
        from ..executor import _SH_FUNCS, stop_group_script

        sb = machine.sandbox
        if sb and "/machines/" in sb:
            script = (_SH_FUNCS + "stopall() {\n"
                      "  for f in \"$@\"; do [ -f \"$f\" ] || continue; (\n" + stop_group_script('"$f"', 200) + "  ); done\n}\n"
                      f"cd {shlex.quote(sb)} 2>/dev/null || exit 0\n"
                      "stopall run/*.pid\nstopall pods/*/*.pid\n"
                      f"cd / && rm -rf -- {shlex.quote(sb)}\n")
            rc, out = ssh.run(self._target_of(machine), script, timeout=120)
            if rc == 255:
                raise ProvisionError(f"{machine.name}: host unreachable during delete: {out.strip()[-300:]}")
        self._release(machine.name)
