"""Provisioning engine: a Terraform-compatible subset over the tk8s providers (L3a).

Reads the generated root config ``terraform/rancher.tf`` (setup.sh:145-152) and the module
definitions ``terraform/{master,host}/*.tf``; commands mirror what setup.sh runs:

  get      — resolve module sources into .terraform/modules   (setup.sh:156 `terraform get`)
  plan     — diff desired resources against terraform.tfstate  (BASELINE.json config 1)
  apply    — create machines concurrently, run their provisioners (setup.sh:157)
  destroy  — delete every machine in the state                 (setup.sh:501 `destroy -force`)

Differences from the reference's Terraform usage:
  * parallelism defaults to ALL resources at once (Terraform's default is 10);
  * local-exec provisioners are serialised and the .ip hand-off files are rewritten in module
    order after apply (no nondeterministic `>>` interleaving, terraform/*/main.tf:30);
  * idempotent creates are retried (``retries``) and failures leave a "tainted" state entry;
  * every step is timed into the event log.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import threading
import time
from pathlib import Path

from . import hcl
from .provider.base import Machine, Provider, ProvisionError
from .utils.events import EventLog
from .utils.faults import fault
from .utils.fsutil import atomic_write, atomic_write_json, file_lock, read_json
from .utils.pool import Pool, as_completed
from .utils.record import field, record as dataclass

STATE_FILE = "terraform.tfstate"
RESOURCE_TYPE = "tk8s_machine"
# Stock-Terraform form of the same machine (terraform/compat/*): terraform_data whose ``input``
# carries the tk8s_machine attributes and whose local-exec provisioners call `tk8s machine ...`.
# The engine plans it identically and creates it through the same provider fast path.
COMPAT_TYPE = "terraform_data"
BOOTSTRAP = ["test -d run && test -d logs && test -d pods",
             "case $(python3 --version 2>&1) in 'Python 3.'[89]*|'Python 3.'[1-9][0-9]*) ;; *) echo 'python3 >= 3.8 required' >&2; exit 1 ;; esac"]


_APPEND = None


def serial_local(provider, parallelism: int | None) -> bool:
    """Create machines on this host one after another, master first. A local create is ~1.6 ms
    of Python (directories, a few small files: no network round trip to overlap), so nine
    threads only contend for the interpreter lock: at 8 workers the master -- whose control plane
    play 2 waits for -- came out of that queue ~15 ms into provisioning and the phase took
    ~21 ms on the MI355X host (profiles/r6_curve/). ``TK8S_PROVISION_SERIAL=0`` (or an explicit
    parallelism) restores a thread per machine."""
    return (parallelism is None and getattr(provider, "colocated", False)
            and os.environ.get("TK8S_PROVISION_SERIAL", "1") != "0")


_PY3_OK: dict[tuple, tuple[int, str]] = {}


def _bootstrap_in_process(provider, m: Machine, cmds: list[str]) -> tuple[int, str] | None:
    """The modules' own bootstrap (BOOTSTRAP: the sandbox's directories, python3 >= 3.8), checked
    here for a machine on this host instead of by a shell per machine: at 8 workers nine bash +
    ``python3 --version`` spawns at once were ~10 ms of the provision phase. The directories are
    the machine's own; ``python3`` is the host's, the same for every local machine (the machine's
    environment does not change PATH), so its version is asked once per interpreter file
    (path, inode, mtime, size: a replaced or rewritten python3 is asked again) -- and not at all
    when it is the interpreter running this engine. Any other script: None (the provider runs it).
    ``TK8S_INPROCESS_BOOTSTRAP=0`` runs even this one in a shell."""
    if (cmds != BOOTSTRAP or not getattr(provider, "colocated", False) or not m.sandbox
            or os.environ.get("TK8S_INPROCESS_BOOTSTRAP", "1") == "0"):
        return None
    sb = Path(m.sandbox)
    missing = [d for d in ("run", "logs", "pods") if not (sb / d).is_dir()]
    if missing:
        return 1, f"{sb}: missing {', '.join(missing)}"
    key = None
    for d in os.environ.get("PATH", "").split(os.pathsep):
        py = os.path.join(d or ".", "python3")
        try:
            st = os.stat(py)
        except OSError:
            continue
        if st.st_mode & 0o170000 == 0o100000 and os.access(py, os.X_OK):  # a regular, executable file
            key = (py, st.st_dev, st.st_ino, st.st_mtime_ns, st.st_size)
            break
    if key not in _PY3_OK:
        if key is not None and os.path.realpath(key[0]) == os.path.realpath(sys.executable):
            _PY3_OK[key] = (0, "") if sys.version_info >= (3, 8) else (1, "python3 >= 3.8 required")
        else:
            r = subprocess.run(["bash", "-c", BOOTSTRAP[1]], capture_output=True, text=True, timeout=60)
            _PY3_OK[key] = (r.returncode, (r.stdout + r.stderr).strip())
    return _PY3_OK[key]


def _append_in_process(cwd: Path, cmd: str) -> bool:
    """``echo <word> >> <file>`` -- the modules' inventory hand-off (terraform/*/main.tf) -- done
    here with bash's exact effect (the word and a newline appended, the file created if
    missing), instead of a shell spawn per machine. Any other command: False (bash runs it)."""
    global _APPEND
    if _APPEND is None:
        import re

        _APPEND = re.compile(r"echo ([A-Za-z0-9_.:-]+) >> ([A-Za-z0-9_.-]+)")
    m = _APPEND.fullmatch(cmd.strip())
    if m is None:
        return False
    with open(Path(cwd) / m.group(2), "a") as f:
        f.write(m.group(1) + "\n")
    return True


@dataclass
class ResourceSpec:
    address: str          # module.<name>.tk8s_machine.<rname>
    module: str
    source: str
    rname: str
    attrs: dict           # interpolated machine attributes
    provisioners: list    # hcl.Block list (unevaluated: they reference the created machine)
    module_dir: Path


@dataclass
class PlanAction:
    address: str
    action: str           # create | no-op | destroy | replace
    attrs: dict = field(default_factory=dict)


@dataclass
class ApplyResult:
    created: list[str] = field(default_factory=list)
    unchanged: list[str] = field(default_factory=list)
    destroyed: list[str] = field(default_factory=list)
    failed: dict[str, str] = field(default_factory=dict)
    seconds: float = 0.0

    @property
    def ok(self) -> bool:
        return not self.failed


class Engine:
    def __init__(self, tf_dir: str | os.PathLike, provider: Provider, events: EventLog | None = None,
                 parallelism: int | None = None, retries: int = 1, on_created=None):
        self.dir = Path(tf_dir).resolve()
        self.provider = provider
        self.events = events or EventLog(None)
        self.parallelism = parallelism
        self.retries = retries
        self.on_created = on_created  # callback(spec address, Machine) once a machine is bootstrapped
        self._state_lock = threading.Lock()
        self._exec_lock = threading.Lock()
        self._write_lock = threading.Lock()
        self._mem: dict | None = None  # apply(): the state in memory, written through by _flush
        self._dirty = 0

    # ---- config ----------------------------------------------------------------------
    def root(self) -> hcl.Block:
        f = self.dir / "rancher.tf"
        if not f.exists():
            raise ProvisionError(f"{f} not found (run setup first)")
        return hcl.parse_file(f)

    def get(self) -> list[str]:
        """`terraform get`: link each module source into .terraform/modules/<name>."""
        mods = []
        mdir = self.dir / ".terraform" / "modules"
        mdir.mkdir(parents=True, exist_ok=True)
        for m in self.root().children("module"):
            name = m.labels[0]
            src = (self.dir / str(m.attrs["source"])).resolve()
            if not src.is_dir():
                raise ProvisionError(f"module {name}: source {src} not found")
            link = mdir / name
            if link.is_symlink() or link.exists():
                link.unlink()
            link.symlink_to(src)
            mods.append(name)
        return mods

    def specs(self) -> list[ResourceSpec]:
        out = []
        mods: dict[Path, hcl.Block] = {}  # one parse per module source (8 workers share "host")
        for m in self.root().children("module"):
            name = m.labels[0]
            src = (self.dir / str(m.attrs["source"])).resolve()
            mod = mods.get(src) or mods.setdefault(src, hcl.parse_dir(src))
            variables = {}
            for v in mod.children("variable"):
                vname = v.labels[0]
                if vname in m.attrs:
                    variables[vname] = hcl.interpolate(m.attrs[vname], {"__dir__": str(self.dir)})
                elif "default" in v.attrs:
                    variables[vname] = v.attrs["default"]
                else:
                    raise ProvisionError(f"module {name}: required variable {vname!r} not set")
            unknown = set(m.attrs) - {"source"} - set(variables)
            if unknown:
                raise ProvisionError(f"module {name}: unknown arguments {sorted(unknown)}")
            ctx = {"var": variables, "__dir__": str(src)}
            for r in mod.children("resource"):
                rtype, rname = r.labels
                if rtype == COMPAT_TYPE:
                    attrs = {k: hcl.interpolate(v, ctx) for k, v in (r.attrs.get("input") or {}).items()}
                    # its local-exec provisioners ARE the machine lifecycle (`tk8s machine create|delete`):
                    # the engine does that itself, then runs the standard bootstrap check
                    provs = [p for p in r.children("provisioner") if "machine " not in str(p.attrs.get("command", ""))]
                    provs.append(hcl.Block("provisioner", ["remote-exec"], {"inline": list(BOOTSTRAP)}))
                    if isinstance(attrs.get("networks"), str):
                        attrs["networks"] = [x for x in attrs["networks"].split(",") if x]
                    out.append(ResourceSpec(f"module.{name}.{rtype}.{rname}", name, str(m.attrs["source"]),
                                            rname, attrs, provs, src))
                    continue
                if rtype != RESOURCE_TYPE:
                    raise ProvisionError(f"module {name}: unsupported resource type {rtype}")
                attrs = {k: hcl.interpolate(v, ctx) for k, v in r.attrs.items()}
                if isinstance(attrs.get("networks"), str):
                    attrs["networks"] = [x for x in attrs["networks"].split(",") if x]
                out.append(ResourceSpec(f"module.{name}.{rtype}.{rname}", name, str(m.attrs["source"]),
                                        rname, attrs, r.children("provisioner"), src))
        return out

    # ---- state -----------------------------------------------------------------------
    def state(self) -> dict:
        return read_json(self.dir / STATE_FILE, None) or {"version": 1, "resources": {}}

    def _save_resource(self, address: str, rec: dict | None) -> None:
        """Record one resource. Outside apply() a read-modify-write of the state file; inside it
        the record goes to the in-memory state and one writer at a time writes it through:
        records that arrive while a write is on its way ride on the next one, so N parallel
        creations cost a few writes, not N read-modify-writes in a row under the lock (measured
        at 8 workers: the state lock was 40 % of the creation threads' time)."""
        if self._mem is None:
            with self._state_lock, file_lock(self.dir / ".tfstate.lock"):
                st = self.state()
                self._apply_record(st, address, rec)
                atomic_write_json(self.dir / STATE_FILE, st)
            return
        with self._state_lock:
            self._apply_record(self._mem, address, rec)
            self._dirty += 1
        self._flush()

    @staticmethod
    def _apply_record(st: dict, address: str, rec: dict | None) -> None:
        if rec is None:
            st["resources"].pop(address, None)
        else:
            st["resources"][address] = rec
        st["serial"] = st.get("serial", 0) + 1

    def _flush(self, wait: bool = False) -> None:
        """Write the in-memory state if records are pending. A caller that finds a write in
        progress leaves its record to that writer, which looks again after every write and once
        more after letting go -- so no record is left behind. ``wait``: block until written."""
        while self._write_lock.acquire(blocking=wait):
            try:
                while True:
                    with self._state_lock:
                        if not self._dirty:
                            break
                        self._dirty = 0
                        text = json.dumps(self._mem, indent=2, sort_keys=True) + "\n"
                    with file_lock(self.dir / ".tfstate.lock"):
                        atomic_write(self.dir / STATE_FILE, text)
            finally:
                self._write_lock.release()
            with self._state_lock:
                if not self._dirty:
                    return

    # ---- plan ------------------------------------------------------------------------
    def plan(self) -> list[PlanAction]:
        st = self.state()["resources"]
        want = {s.address: s for s in self.specs()}
        acts = []
        for addr, s in want.items():
            cur = st.get(addr)
            if cur is None:
                acts.append(PlanAction(addr, "create", s.attrs))
            elif cur.get("tainted"):
                acts.append(PlanAction(addr, "replace", s.attrs))
            else:
                acts.append(PlanAction(addr, "no-op", s.attrs))
        for addr in st:
            if addr not in want:
                acts.append(PlanAction(addr, "destroy"))
        return acts

    @staticmethod
    def plan_summary(acts: list[PlanAction]) -> str:
        add = sum(a.action in ("create", "replace") for a in acts)
        destroy = sum(a.action in ("destroy", "replace") for a in acts)
        lines = [f"  {'+' if a.action == 'create' else '-/+' if a.action == 'replace' else '-' if a.action == 'destroy' else ' '} {a.address}"
                 for a in acts if a.action != "no-op"]
        lines.append(f"Plan: {add} to add, 0 to change, {destroy} to destroy.")
        return "\n".join(lines)

    # ---- apply -----------------------------------------------------------------------
    def _provision(self, spec: ResourceSpec, m: Machine) -> None:
        ctx = {"var": {}, RESOURCE_TYPE: {spec.rname: m.to_dict()}, "self": m.to_dict(), "__dir__": str(spec.module_dir)}
        for p in spec.provisioners:
            kind = p.labels[0] if p.labels else ""
            if kind == "remote-exec":
                # Like Terraform, the inline list runs as ONE script on the machine, in order,
                # stopping at the first failing command (one shell spawn per machine, not per line).
                cmds = list(hcl.interpolate(p.attrs.get("inline", []), ctx))
                if cmds:
                    done = _bootstrap_in_process(self.provider, m, cmds)
                    rc, out = done if done is not None else self.provider.exec(m, "set -e\n" + "\n".join(cmds))
                    if rc != 0:
                        raise ProvisionError(f"{spec.address}: remote-exec failed rc={rc}: {out.strip()[-400:]}")
            elif kind == "local-exec":
                cmd = hcl.interpolate(p.attrs["command"], ctx)
                with self._exec_lock:
                    if not _append_in_process(self.dir, cmd):
                        r = subprocess.run(["bash", "-c", cmd], cwd=self.dir, capture_output=True, text=True, timeout=300)
                        if r.returncode != 0:
                            raise ProvisionError(f"{spec.address}: local-exec {cmd!r} failed: {r.stderr.strip()}")
            else:
                raise ProvisionError(f"{spec.address}: unsupported provisioner {kind!r}")

    def _boot(self, m: Machine, spec: ResourceSpec) -> None:
        if self.on_created is not None:
            try:
                self.on_created(spec.address, m)
            except Exception as e:  # noqa: BLE001 - a boot hook never fails provisioning
                self.events.emit("machine_boot_hook_failed", name=m.name, error=str(e))

    def _create(self, spec: ResourceSpec) -> Machine:
        a = spec.attrs
        last_err: Exception | None = None
        for attempt in range(1, self.retries + 2):
            t = time.monotonic()
            try:
                if fault("provision.create", a["name"]) and attempt == 1:
                    raise ProvisionError(f"injected create failure for {a['name']}")
                pub = a.get("root_authorized_keys", "")
                m = self.provider.create_machine(a["name"], a["package"], list(a.get("networks", [])),
                                                 image=a.get("image", ""), root_authorized_keys=pub,
                                                 tags=a.get("tags", {}))
            except ProvisionError as e:
                last_err = e
                self.events.emit("machine_create_retry", address=spec.address, attempt=attempt, error=str(e))
                continue
            t_boot = time.monotonic()
            try:
                self._provision(spec, m)
            except Exception as e:  # tainted: machine exists but bootstrap failed
                self._save_resource(spec.address, {"module": spec.module, "machine": m.to_dict(), "tainted": True,
                                                   "error": str(e)})
                raise
            self._save_resource(spec.address, {"module": spec.module, "machine": m.to_dict(), "tainted": False})
            self.events.emit("machine_created", address=spec.address, name=m.name, ip=m.primaryip,
                             gpus=m.gpus, seconds=round(time.monotonic() - t, 6),
                             bootstrap_seconds=round(time.monotonic() - t_boot, 6))
            # booting after the bootstrap (measured at 8 workers on the MI355X host: booting first
            # gained nothing, profiles/r2_n8) -- a machine that failed it never starts services
            self._boot(m, spec)
            return m
        if hasattr(self.provider, "release_reservation"):
            self.provider.release_reservation(a["name"])
        raise ProvisionError(f"{spec.address}: create failed after {self.retries + 1} attempts: {last_err}")

    def apply(self) -> ApplyResult:
        t0 = time.monotonic()
        res = ApplyResult()
        specs = self.specs()
        st = self.state()["resources"]
        # Terraform semantics: a resource in the state whose module left the configuration (the
        # node count went down) is destroyed by apply, as `plan` announced.
        wanted = {s.address for s in specs}
        for addr, rec in list(st.items()):
            if addr not in wanted:
                self.provider.delete_machine(Machine.from_dict(rec["machine"]))
                self._save_resource(addr, None)
                res.destroyed.append(addr)
                self.events.emit("machine_destroyed", address=addr, name=rec["machine"].get("name"))
        todo = []
        for s in specs:
            cur = st.get(s.address)
            if cur and not cur.get("tainted"):
                res.unchanged.append(s.address)
                continue
            if cur and cur.get("tainted"):
                self.provider.delete_machine(Machine.from_dict(cur["machine"]))
                self._save_resource(s.address, None)
            todo.append(s)
        if todo and hasattr(self.provider, "reserve"):  # one allocation for all (local machines)
            self.provider.reserve([(s.attrs["name"], s.attrs["package"], list(s.attrs.get("networks", [])),
                                    (s.attrs.get("tags") or {}).get("role", "host")) for s in todo])
        workers = self.parallelism or max(1, len(todo))
        if serial_local(self.provider, self.parallelism):
            # master first: its control plane boots while the workers are created
            todo.sort(key=lambda s: not s.source.rstrip("/").endswith("master"))
            workers = 1
        self._mem, self._dirty = self.state(), 0
        try:
            with Pool(workers, "provision") as ex:
                futs = {ex.submit(self._create, s): s for s in todo}
                for f in as_completed(futs):
                    s = futs[f]
                    try:
                        f.result()
                        res.created.append(s.address)
                    except Exception as e:  # noqa: BLE001 - report per resource
                        res.failed[s.address] = str(e)
                        self.events.emit("machine_failed", address=s.address, error=str(e))
        finally:
            self._flush(wait=True)
            self._mem = None
        self.write_ip_files(specs)
        res.seconds = time.monotonic() - t0
        return res

    def write_ip_files(self, specs: list[ResourceSpec] | None = None) -> None:
        """Rewrite masters.ip / hosts.ip in module order from the state (race-free hand-off)."""
        specs = specs if specs is not None else self.specs()
        st = self.state()["resources"]
        files: dict[str, list[str]] = {"masters.ip": [], "hosts.ip": []}
        for s in specs:
            rec = st.get(s.address)
            if not rec or rec.get("tainted"):
                continue
            key = "masters.ip" if s.source.rstrip("/").endswith("master") else "hosts.ip"
            files[key].append(rec["machine"]["primaryip"])
        for name, ips in files.items():
            if ips:
                atomic_write(self.dir / name, "".join(ip + "\n" for ip in ips))
            else:
                (self.dir / name).unlink(missing_ok=True)

    def machines(self) -> dict[str, Machine]:
        """Created machines keyed by module name (tainted ones excluded)."""
        out = {}
        for rec in self.state()["resources"].values():
            if not rec.get("tainted"):
                m = Machine.from_dict(rec["machine"])
                out[rec["module"]] = m
        return out

    # ---- destroy ---------------------------------------------------------------------
    def destroy(self) -> list[str]:
        st = self.state()["resources"]
        gone = []

        def one(addr: str, rec: dict) -> str:
            self.provider.delete_machine(Machine.from_dict(rec["machine"]))
            self._save_resource(addr, None)
            return addr

        with Pool(max(1, len(st)), "destroy") as ex:
            for f in as_completed([ex.submit(one, a, r) for a, r in st.items()]):
                gone.append(f.result())
        return gone
