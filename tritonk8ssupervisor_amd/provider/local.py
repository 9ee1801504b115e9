"""Local bare-metal provider: worker "machines" are sandboxes on this MI355X host.

Replaces the Triton KVM of terraform/master/main.tf:1-11 / terraform/host/main.tf:1-11:

* a machine = a sandbox directory (``<state>/machines/<name>``) + its own loopback IP (one per
  network, from 127.0.<net>.0/24) + an exclusive slice of the host's GPUs (by package shape);
* ``networks()`` are loopback subnets; the default ``local-public`` plays Joyent-SDC-Public;
* ``packages()`` are worker shapes of the 8x MI355X node (``mi355x-<k>gpu``); the default
  ``mi355x-1gpu`` gives 8 workers x 1 GPU = all 8 GPUs allocatable (BASELINE.json configs 3-5).
  The master never takes GPUs (it only runs the control plane, like rancher/server).
* ``exec`` runs a command in the sandbox (remote-exec), ``delete_machine`` kills every process
  group recorded under the sandbox and frees its IPs and GPUs.

IP/GPU allocation is serialised by an flock on ``<state>/alloc.lock`` so concurrent creates
(the Terraform fan-out) are race-free, and claimed host-wide (``hostreg.py``) so clusters that
share the host never share an address or a GPU.
"""
from __future__ import annotations

import _socket as socket  # (the C module: inet_ntoa, gethostname, a bind probe -- utils/http1.py)
import getpass
import os
import subprocess
from pathlib import Path

from ..models.hostinfo import discover
from ..utils.fsutil import atomic_write_json, file_lock, read_json
from ..utils.ids import uuid5
from ..utils.procs import kill_pidfile
from . import keys
from .base import Machine, Network, Package, Provider, ProvisionError
from .hostreg import HostRegistry

_NS = "5f1c0d3e-8a4b-4c6e-9b1a-7e2f3d4c5b6a"

NETWORKS = [
    ("local-fabric", "127.0.2.0/24", False),
    ("local-public", "127.0.1.0/24", True),
    ("local-storage", "127.0.3.0/24", False),
]
# (name, gpus) ; cpus/memory derived from the host
SHAPES = [("cpu-only", 0), ("mi355x-1gpu", 1), ("mi355x-2gpu", 2), ("mi355x-4gpu", 4), ("mi355x-8gpu", 8)]


def _uid(kind: str, name: str) -> str:
    return uuid5(_NS, f"tk8s/{kind}/{name}")


def _loopback_multi_ok() -> bool:
    """Can we bind non-127.0.0.1 loopback addresses (true on stock Linux)?"""
    if os.environ.get("TK8S_SINGLE_IP") == "1":
        return False
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    try:
        s.bind(("127.0.1.254", 0))
        return True
    except OSError:
        return False
    finally:
        s.close()



def _ipv4_hosts(cidr: str):
    """The host addresses of an IPv4 network, in order -- ``ipaddress.ip_network(cidr).hosts()``
    as strings, without importing ipaddress on the bring-up path (prefixes /31 and /32, and
    anything that is not dotted-quad IPv4, go to ipaddress itself)."""
    addr, _, plen = cidr.partition("/")
    parts = addr.split(".")
    if len(parts) != 4 or not all(p.isdigit() and int(p) < 256 for p in parts) or not plen.isdigit() or int(plen) > 30:
        import ipaddress

        yield from (str(a) for a in ipaddress.ip_network(cidr).hosts())
        return
    n = int(plen)
    base = (int(parts[0]) << 24) | (int(parts[1]) << 16) | (int(parts[2]) << 8) | int(parts[3])
    mask = (0xFFFFFFFF << (32 - n)) & 0xFFFFFFFF
    if base & ~mask & 0xFFFFFFFF:
        raise ValueError(f"{cidr} has host bits set")
    for a in range(base + 1, base + (1 << (32 - n)) - 1):
        yield f"{a >> 24}.{(a >> 16) & 255}.{(a >> 8) & 255}.{a & 255}"

class LocalProvider(Provider):
    name = "local"
    default_network = "local-public"
    default_package = "mi355x-1gpu"
    colocated = True

    def __init__(self, state_dir: str | os.PathLike, key_dir: str | os.PathLike | None = None):
        self.state_dir = Path(state_dir).resolve()
        self.machines_dir = self.state_dir / "machines"
        self.key_dir = Path(key_dir) if key_dir else self.state_dir / "keys"
        self.alloc_file = self.state_dir / "alloc.json"
        self.lock_file = self.state_dir / "alloc.lock"
        self.host = HostRegistry()
        self._multi_ip = None
        self.preferred_gpus: list[int] = []  # an early burn-in is already validating these
        self._reserved: dict[str, tuple[list[str], list[int]]] = {}  # reserve(): name -> (ips, gpus)

    def prefer_gpus(self, gpus: list[int]) -> None:
        """Hand workers these GPUs first (when enough of them are free): the early burn-in
        (earlyburn.py) picked them before the allocator ran."""
        self.preferred_gpus = list(gpus)

    def _candidates(self, free: list[int], count: int) -> list[int]:
        pref = [g for g in free if g in self.preferred_gpus]
        return pref if len(pref) >= count else free

    # ---- inventory ----------------------------------------------------------------
    def env(self) -> dict[str, str]:
        _, _, fp = keys.ensure_cluster_key(self.key_dir)
        return {
            "SDC_URL": f"local://{socket.gethostname()}",
            "SDC_ACCOUNT": getpass.getuser(),
            "SDC_KEY_ID": fp,
        }

    def find_key(self, key_id: str) -> str | None:
        return keys.find_key(key_id, [self.key_dir, "~/.ssh"])

    def networks(self) -> list[Network]:
        return sorted((Network(n, _uid("network", n), subnet, pub) for n, subnet, pub in NETWORKS),
                      key=lambda x: x.name)

    def packages(self) -> list[Package]:
        cpus = os.cpu_count() or 8
        try:
            mem_mb = os.sysconf("SC_PAGE_SIZE") * os.sysconf("SC_PHYS_PAGES") // 2**20
        except (ValueError, OSError):
            mem_mb = 64 * 1024
        out = []
        for name, g in SHAPES:
            share = max(g, 1) / 8
            out.append(Package(name, _uid("package", name), gpus=g, cpus=max(1, int(cpus * share)),
                               memory_mb=int(mem_mb * share),
                               description=f"{g}x MI355X (gfx950) worker" if g else "CPU-only worker"))
        return sorted(out, key=lambda p: p.name)

    # ---- allocation ---------------------------------------------------------------
    def _multi(self) -> bool:
        if self._multi_ip is None:
            self._multi_ip = _loopback_multi_ok()
        return self._multi_ip

    @staticmethod
    def _host_gpus() -> bool:
        """Real GPUs are claimed host-wide; a fake inventory is private to each cluster."""
        return not os.environ.get("TK8S_FAKE_GPUS")

    _bound_cache: tuple[float, set[str]] | None = None

    @classmethod
    def _bound_ips_cached(cls, max_age: float = 2.0) -> set[str]:
        """_bound_ips() shared by the machines of one provisioning run: reading /proc/net costs
        ~1-4 ms and the allocations run one after another under the workspace lock."""
        import time

        c = cls._bound_cache
        now = time.monotonic()
        if c is None or now - c[0] > max_age:
            c = cls._bound_cache = (now, cls._bound_ips())
        return c[1]

    @staticmethod
    def _bound_ips() -> set[str]:
        """Loopback addresses something on this host already serves on (a TCP listener or a
        UDP socket bound to that address): a cluster the registry does not know about -- another
        user's, or one whose registry is gone -- still owns its master's DNS / ingress / API
        sockets there, and a new machine on the same address would answer for neither. (One
        regex pass over each table: a shared host lists thousands of sockets.)"""
        import re

        out: set[str] = set()
        # local address column "XXXXXX7F:PORT" (127.x.y.z, little-endian hex), then the remote
        # address, then the state (0A = LISTEN; any state for UDP)
        for table, state in (("/proc/net/tcp", rb"0A"), ("/proc/net/udp", rb"[0-9A-F]{2}")):
            try:
                with open(table, "rb") as f:
                    data = f.read()
            except OSError:
                continue
            for hexip in re.findall(rb"^ *\d+: ([0-9A-F]{6}7F):[0-9A-F]{4} [0-9A-F]{8}:[0-9A-F]{4} " + state,
                                    data, re.M):
                ip = socket.inet_ntoa(bytes.fromhex(hexip.decode())[::-1])
                if ip != "127.0.0.1":
                    out.add(ip)
        return out

    def _alloc_ips(self, alloc: dict, name: str, nets: list[Network], host: dict) -> list[str]:
        used = alloc.setdefault("ips", {})
        host_used = HostRegistry.taken(host, "ips") | (self._bound_ips_cached() if self._multi() else set())
        out = []
        for net in nets:
            if not self._multi():
                out.append("127.0.0.1")
                continue
            for ip in _ipv4_hosts(net.subnet):
                if ip not in used and ip not in host_used:
                    used[ip] = name
                    HostRegistry.claim(host, "ips", ip, self.alloc_file, name)
                    out.append(ip)
                    break
            else:
                raise ProvisionError(f"network {net.name} exhausted")
        return out

    def _alloc_gpus(self, alloc: dict, name: str, count: int, host: dict) -> list[int]:
        if count == 0:
            return []
        inv = discover()
        taken = {int(k) for k in alloc.setdefault("gpus", {})}
        if self._host_gpus():
            taken |= {int(k) for k in HostRegistry.taken(host, "gpus")}
        free = [g.ordinal for g in inv.gpus if g.ordinal not in taken]
        if len(free) >= count:
            free = self._candidates(free, count)
        if len(free) < count:
            raise ProvisionError(
                f"{name}: package needs {count} GPU(s) but only {len(free)} of {inv.count} are free "
                "(the local analogue of reaching the provisioning limit)")
        try:
            from ..ops import topo

            n = inv.count
            from ..agent.deviceplugin import link_matrix

            res = topo().preferred_allocation(n, link_matrix(inv.links), free, [], count)
            pick = list(res["devices"])
        except Exception:  # noqa: BLE001 - allocator module optional at provision time
            pick = free[:count]
        for g in pick:
            alloc["gpus"][str(g)] = name
            if self._host_gpus():
                HostRegistry.claim(host, "gpus", g, self.alloc_file, name)
        return pick

    def predict_gpus(self, per_machine: int, machines: int) -> list[int]:
        """The GPUs ``machines`` creates of ``per_machine`` GPUs each will take from what is free
        now (the same topology-aware picks as _alloc_gpus, made one after another)."""
        if per_machine <= 0 or machines <= 0:
            return []
        alloc = read_json(self.alloc_file, {}) or {}
        taken = {int(k) for k in alloc.get("gpus", {})}
        if self._host_gpus():
            with self.host.locked() as host:
                taken |= {int(k) for k in HostRegistry.taken(host, "gpus")}
        inv = discover()
        free = [g.ordinal for g in inv.gpus if g.ordinal not in taken]
        out: list[int] = []
        try:
            from ..agent.deviceplugin import link_matrix
            from ..ops import topo

            w = link_matrix(inv.links)
            for _ in range(machines):
                if len(free) < per_machine:
                    break
                pick = list(topo().preferred_allocation(inv.count, w, self._candidates(free, per_machine), [],
                                                        per_machine)["devices"])
                out += pick
                free = [g for g in free if g not in pick]
        except Exception:  # noqa: BLE001 - allocator module optional
            out = self._candidates(free, per_machine * machines)[: per_machine * machines]
        return sorted(out)

    # ---- lifecycle ----------------------------------------------------------------
    def reserve(self, machines: list[tuple[str, str, list[str], str]]) -> None:
        """Allocate the addresses and GPU slices of several machines -- (name, package, networks,
        role) -- under one take of the workspace and host locks and one write of the allocation
        table and the host registry, instead of one per machine (the engine's parallel creates
        queue on those locks: ~2-5 ms each, 9 machines deep at 8 workers). Best effort: if any
        machine cannot be allocated, nothing is reserved and each create allocates (and reports)
        on its own."""
        todo = []
        try:
            for name, package, networks, role in machines:
                nets = [self.network_by_id_or_name(n) for n in networks] or [
                    self.network_by_id_or_name(self.default_network)]
                todo.append((name, self.package_by_id_or_name(package), nets, role))
            with file_lock(self.lock_file):
                alloc = read_json(self.alloc_file, {}) or {}
                got = {}
                with self.host.locked() as host:
                    for name, pkg, nets, role in todo:
                        if name in alloc.get("machines", {}):
                            raise ProvisionError(f"machine {name} already exists")
                        ips = self._alloc_ips(alloc, name, nets, host)
                        gpus = self._alloc_gpus(alloc, name, 0 if role == "master" else pkg.gpus, host)
                        alloc.setdefault("machines", {})[name] = {"ips": ips, "gpus": gpus}
                        got[name] = (ips, gpus)
                    atomic_write_json(self.alloc_file, alloc)
                self._reserved.update(got)
        except (ProvisionError, OSError, KeyError, ValueError):
            return

    def release_reservation(self, name: str) -> None:
        """A reserved machine that will not be created after all (its create failed for good)."""
        if self._reserved.pop(name, None) is not None:
            self.delete_machine(Machine(name=name, id="", package="", networks=[], primaryip="", ips=[], gpus=[],
                                        image="", tags={}, sandbox=str(self.machines_dir / name)))

    def create_machine(self, name: str, package: str, networks: list[str], image: str = "",
                       root_authorized_keys: str = "", tags: dict | None = None) -> Machine:
        pkg = self.package_by_id_or_name(package)
        nets = [self.network_by_id_or_name(n) for n in networks] or [self.network_by_id_or_name(self.default_network)]
        role = (tags or {}).get("role", "host")
        sandbox = self.machines_dir / name
        if name in self._reserved:  # allocated with its siblings (reserve)
            ips, gpus = self._reserved.pop(name)
        else:
            with file_lock(self.lock_file):
                alloc = read_json(self.alloc_file, {}) or {}
                if name in alloc.get("machines", {}):
                    raise ProvisionError(f"machine {name} already exists")
                # the owner's alloc.json is written under the host lock too: a concurrent reaper
                # must never see a claim whose machine its owner does not list yet
                with self.host.locked() as host:
                    ips = self._alloc_ips(alloc, name, nets, host)
                    gpus = self._alloc_gpus(alloc, name, 0 if role == "master" else pkg.gpus, host)
                    alloc.setdefault("machines", {})[name] = {"ips": ips, "gpus": gpus}
                    atomic_write_json(self.alloc_file, alloc)
        for sub in ("run", "logs", "pods", "etc"):
            (sandbox / sub).mkdir(parents=True, exist_ok=True)
        if root_authorized_keys:
            (sandbox / "etc" / "authorized_keys").write_text(root_authorized_keys.rstrip() + "\n")
        m = Machine(name=name, id=_uid("machine", f"{name}/{ips[0]}"), package=pkg.name,
                    networks=[n.id for n in nets], primaryip=ips[0], ips=ips, gpus=gpus, image=image,
                    tags=dict(tags or {}), sandbox=str(sandbox))
        atomic_write_json(sandbox / "machine.json", m.to_dict())
        return m

    def get_machine(self, name: str) -> Machine | None:
        d = read_json(self.machines_dir / name / "machine.json")
        return Machine.from_dict(d) if d else None

    def list_machines(self) -> list[Machine]:
        out = []
        if self.machines_dir.is_dir():
            for d in sorted(self.machines_dir.iterdir()):
                m = self.get_machine(d.name)
                if m:
                    out.append(m)
        return out

    def machine_env(self, m: Machine) -> dict[str, str]:
        env = {
            "TK8S_MACHINE": m.name,
            "TK8S_MACHINE_DIR": m.sandbox,
            "TK8S_MACHINE_IP": m.primaryip,
            "TK8S_MACHINE_GPUS": ",".join(map(str, m.gpus)),
            "TK8S_MACHINE_PACKAGE": m.package,
        }
        try:  # the package's slice of the host: the node's capacity, enforced by agent/resources.py
            pkg = self.package_by_id_or_name(m.package)
            env.update(TK8S_MACHINE_CPUS=str(pkg.cpus), TK8S_MACHINE_MEMORY_MB=str(pkg.memory_mb))
        except Exception:  # noqa: BLE001 - an unknown package: the host's shape
            pass
        fake_hosts = int(os.environ.get("TK8S_FAKE_HOSTS", "0") or 0)
        if fake_hosts > 1:  # CPU tests: pretend the machines are spread over that many hosts
            digits = "".join(ch for ch in m.name if ch.isdigit()) or "0"
            env["TK8S_HOST_ID"] = f"fakehost{(int(digits) - 1) % fake_hosts}"
        return env

    def ansible_host_vars(self, m: Machine) -> dict:
        """Inventory variables for stock ansible-playbook: the machines are sandboxes of this host,
        so it connects locally; the tk8s modules find the sandbox and the install from these."""
        from pathlib import Path as _P

        return {"ansible_connection": "local", "tk8s_machine_dir": m.sandbox, "tk8s_gpus": ",".join(map(str, m.gpus)),
                "tk8s_home": str(_P(__file__).resolve().parents[2])}

    def exec(self, machine: Machine, command: str, timeout: float = 300, env: dict | None = None,
             stdin: bytes | None = None) -> tuple[int, str]:
        e = dict(os.environ)
        e.update(self.machine_env(machine))
        e.update(env or {})
        try:
            r = subprocess.run(["bash", "-c", command], cwd=machine.sandbox, env=e, capture_output=True,
                               input=stdin if stdin is not None else b"", timeout=timeout)
        except subprocess.TimeoutExpired as ex:
            return 124, f"timeout after {timeout}s: {ex}"
        return r.returncode, (r.stdout or b"").decode(errors="replace") + (r.stderr or b"").decode(errors="replace")

    def delete_machine(self, machine: Machine) -> None:
        sandbox = Path(machine.sandbox or self.machines_dir / machine.name)
        run = sandbox / "run"
        if run.is_dir():
            for pidfile in sorted(run.glob("*.pid")):
                kill_pidfile(pidfile, grace=2.0)
        # pods write their pidfiles under pods/<pod>/pid
        pods = sandbox / "pods"
        if pods.is_dir():
            for pidfile in sorted(pods.glob("*/*.pid")):
                kill_pidfile(pidfile, grace=1.0)
        with file_lock(self.lock_file):
            alloc = read_json(self.alloc_file, {}) or {}
            alloc.get("machines", {}).pop(machine.name, None)
            for k in ("ips", "gpus"):
                table = alloc.get(k, {})
                for key in [key for key, owner in table.items() if owner == machine.name]:
                    del table[key]
            atomic_write_json(self.alloc_file, alloc)
            with self.host.locked() as host:
                HostRegistry.release(host, self.alloc_file, machine.name)
        import shutil

        shutil.rmtree(sandbox, ignore_errors=True)
