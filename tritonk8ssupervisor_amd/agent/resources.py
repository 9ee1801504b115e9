"""Pod and machine resource limits, enforced (VERDICT r3 missing-1).

The reference's nodes were hard slices: a Triton KVM ``package`` per machine
(/root/reference/terraform/host/main.tf:3, chosen at /root/reference/setup.sh:402-449), and its
workloads ran in Docker containers with cgroup limits
(/root/reference/ansible/roles/rancherhost/tasks/main.yml:26-34). Here a worker is a sandbox of
the MI355X host and a pod is a process group, so the agent enforces the shapes itself, in the
strongest mode the host allows (``Enforcer.mode``):

* ``cgroup2`` -- a writable (delegated) cgroup v2 subtree: a machine cgroup with the package's
  ``memory.max`` / ``cpu.max`` / ``cpuset.cpus``, one cgroup per pod beneath it with the pod's
  ``limits.memory`` / ``limits.cpu`` and, for GPU pods, ``cpuset.cpus`` = the NUMA-local CPUs of
  its GPUs. The kernel throttles and OOM-kills; ``memory.events`` says which kill was an OOM.
* ``cgroup1`` -- the same on writable v1 memory / cpu / cpuset hierarchies (root on a v1 host,
  e.g. inside a container): ``memory.limit_in_bytes``, ``cpu.cfs_quota_us``, ``cpuset.cpus``.
* ``watchdog`` -- unprivileged (the GPU tier: an ordinary user, no delegation), the agent
  enforces the shapes from ``/proc``:
  - ``limits.cpu``: a duty cycle over the pod's processes, as cpulimit does -- every
    ``TICK_S`` the CPU time its processes used (``/proc/<pid>/stat`` utime+stime deltas) is
    charged to a token bucket filled at ``limits.cpu`` cores; while the bucket is negative the
    pod's process groups are SIGSTOPped, and SIGCONTed when it has refilled (``CpuThrottle``);
  - ``limits.memory``: every pod's resident set is sampled, a pod over its limit is killed
    (``OOMKilled``, exit 137, restarted under its policy); CPU pods also get a hard
    ``RLIMIT_DATA`` backstop from the jail (``--rlimit-data``: an allocation burst between two
    samples fails with ENOMEM instead of taking the host's memory);
  - the machine's package (its ``cpu`` / ``memory`` shape, the reference's KVM slice): the same
    bucket over the CPU time of ALL the machine's pods, and when their resident sets together
    exceed the package's memory the newest pod is OOMKilled;
  - GPU pods are pinned to their GPUs' NUMA-local CPUs (``sched_setaffinity``; placement).

Processes join their cgroups and CPUs inside the pod jail before anything runs
(``tk8s-gpujail --cgroup-procs/--cpus``, gpujail.h ``join_limits``), so no process of a pod ever
runs outside them. ``TK8S_POD_RESOURCES`` = auto|cgroup2|cgroup1|watchdog|none picks the mode;
``TK8S_CGROUP_ROOT`` and ``TK8S_SYSFS_ROOT`` point at other trees (the CPU tests' fakes).
"""
from __future__ import annotations

import os
import re
import signal
import threading
import time
from pathlib import Path

from ..utils import quantity
from ..utils.record import record as dataclass

CFS_PERIOD_US = 100_000
_NAME = re.compile(r"[^A-Za-z0-9_.-]")
TICK_S = 0.05             # the watchdog's CPU duty-cycle tick
BURST_S = 0.1             # how far ahead of its rate a pod may run (seconds of its limit)
_HZ = os.sysconf("SC_CLK_TCK") if hasattr(os, "sysconf") else 100
RLIMIT_DATA_SLACK = 256 << 20   # the backstop sits above the sampled limit: 2 x limits.memory + this
RLIMIT_DATA_FLOOR = 1 << 30     # ... and never below 1 GiB


def rlimit_data_for(memory: int) -> int:
    """The per-process RLIMIT_DATA backstop of a CPU pod with ``limits.memory``: above the limit
    the sampler enforces, well below what would take the host. RLIMIT_DATA counts private
    writable VIRTUAL memory -- 8 MiB per thread stack, malloc arenas not yet touched -- not the
    resident set Kubernetes limits, so it has a 1 GiB floor (a thread-heavy pod with a
    small limit must start; its resident set is what the sampler holds to the limit)."""
    return max(2 * int(memory) + RLIMIT_DATA_SLACK, RLIMIT_DATA_FLOOR)


def signal_ids(groups, pids, sig, starts: dict[int, int]) -> None:
    """``sig`` to process groups ``groups`` and processes ``pids`` that are still the processes
    recorded in ``starts`` (pid -> start ticks); ids without a record are left alone."""
    from ..utils.procs import proc_start_ticks

    for g in groups:
        if starts.get(g) is not None and proc_start_ticks(g) == starts[g]:
            try:
                os.killpg(g, sig)
            except (ProcessLookupError, PermissionError):
                pass
    for p in pids:
        if starts.get(p) is not None and proc_start_ticks(p) == starts[p]:
            try:
                os.kill(p, sig)
            except (ProcessLookupError, PermissionError):
                pass


def _cpu_seconds(pid: int) -> float | None:
    """CPU time process ``pid`` and its waited-for children have used: utime + stime + cutime +
    cstime (/proc/<pid>/stat fields 14-17, all threads). With the children's part, the CPU of a
    child that lived and died between two scans still reaches the pod's bill (through its parent),
    and so does the part of a sampled child's life after its last sample."""
    try:
        with open(f"/proc/{pid}/stat", "rb") as f:
            raw = f.read()
        rest = raw[raw.rindex(b")") + 2:].split()
        return (int(rest[11]) + int(rest[12]) + int(rest[13]) + int(rest[14])) / _HZ
    except (OSError, ValueError, IndexError):
        return None


class CpuThrottle:
    """The watchdog mode's CPU limits: token buckets filled at ``limits.cpu`` cores per pod (and
    at the package's ``cpu`` for the machine as a whole), charged with the CPU time the pods'
    processes used each tick; a pod whose bucket -- or whose machine's -- is negative is stopped
    (SIGSTOP to its process groups and members) until it has refilled (SIGCONT). Over a window the
    pod then runs ``limits.cpu`` / (its parallelism) of the time: a 250m busy loop runs one tick
    in four."""

    def __init__(self, machine_cpu: float | None = None):
        self.machine_cpu = machine_cpu or None
        self.balance: dict[str, float] = {}      # pod key (and "" = the machine) -> CPU seconds
        self.total: dict[str, float] = {}         # pod key -> its members' CPU seconds at the previous tick
        self.stopped: dict[str, tuple[list[int], list[int]]] = {}  # pod key -> (groups, pids) it stopped
        self.starts: dict[int, int] = {}          # pid -> its start time (ticks since boot) at the last scan
        self.exempt: set[str] = set()             # pods being terminated: never stopped again
        self.stops = 0                            # pod stops so far (describe, tests)
        # the watchdog's thread steps; the runtime's stop threads resume pods they terminate
        self.lock = threading.RLock()

    def _signal(self, groups, pids, sig) -> None:
        """Signal the pod's processes -- each only while it is still the process the last scan saw
        (same start time): a pid or process group id reused since is never signalled. A group is
        signalled through its leader's identity (while the leader lives, its id cannot be reused)."""
        signal_ids(groups, pids, sig, self.starts)

    def terminating(self, key: str) -> None:
        """Pod ``key`` is being stopped: running again at once, so its processes see SIGTERM and
        have their grace period, and not throttled any more."""
        with self.lock:
            self.exempt.add(key)
            self.resume(key)

    def resume(self, key: str) -> None:
        with self.lock:
            hit = self.stopped.pop(key, None)
            if hit is not None:
                self._signal(hit[0], hit[1], signal.SIGCONT)

    def resume_all(self) -> None:
        with self.lock:
            for key in list(self.stopped):
                self.resume(key)

    def step(self, pods: dict[str, tuple[list[int], set[int]]], limits: dict[str, "Limits"], dt: float,
             in_machine=lambda key: True) -> None:
        """One tick: ``pods`` -> {key: (process groups, member pids)} of the running pods."""
        with self.lock:
            self._step(pods, limits, dt, in_machine)

    def _step(self, pods, limits, dt, in_machine) -> None:
        for key in [k for k in self.stopped if k not in pods]:  # gone (or terminating): never left stopped
            self.resume(key)
        for key in [k for k in self.balance if k and k not in pods]:
            del self.balance[key]
        # A pod's bill is the change of ONE sum over its members -- each member's own CPU plus that
        # of its children it has waited for: a member that appeared since the last tick brings its
        # whole life in (its CPU before the first sample is charged too), and one that exited and
        # was reaped by a member moves its total into that member's children's part (nothing is
        # charged twice; a child re-parented outside the pod takes only its unsampled tail along).
        used: dict[str, float] = {}
        totals: dict[str, float] = {}
        for key, (_groups, pids) in pods.items():
            t = sum(x for x in (_cpu_seconds(p) for p in pids) if x is not None)
            totals[key] = t
            used[key] = max(0.0, t - self.total.get(key, 0.0))
        self.total = totals
        machine_neg = False
        if self.machine_cpu:
            u = sum(v for k, v in used.items() if in_machine(k))
            b = min(self.balance.get("", 0.0) + self.machine_cpu * dt - u, self.machine_cpu * BURST_S)
            self.balance[""] = b
            machine_neg = b < 0
        for key, (groups, pids) in pods.items():
            if key in self.exempt:
                continue
            lim = limits.get(key)
            neg = machine_neg and in_machine(key)
            if lim is not None and lim.cpu:
                b = min(self.balance.get(key, 0.0) + lim.cpu * dt - used[key], lim.cpu * BURST_S)
                self.balance[key] = b
                neg = neg or b < 0
            if neg and key not in self.stopped:
                self.stopped[key] = (list(groups), sorted(pids))
                self._signal(groups, pids, signal.SIGSTOP)
                self.stops += 1
            elif neg:  # members that appeared since it was stopped
                g0, p0 = self.stopped[key]
                new = sorted(set(pids) - set(p0))
                if new:
                    self._signal([], new, signal.SIGSTOP)
                    self.stopped[key] = (g0, p0 + new)
            elif key in self.stopped:
                self.resume(key)


@dataclass
class Limits:
    memory: int | None = None    # bytes (limits.memory)
    cpu: float | None = None     # cores (limits.cpu)
    cpus: str = ""               # cpuset / affinity list ("0-63,128-191"), "" = any


def pod_limits(pod: dict) -> Limits:
    """The pod's cgroup limits, as the kubelet sizes the pod cgroup: the sum over its app
    containers when every one has the limit, at least the largest init container's."""
    spec = pod.get("spec") or {}

    def total(kind: str, parse) -> float | None:
        vals = [((c.get("resources") or {}).get("limits") or {}).get(kind) for c in spec.get("containers") or []]
        if not vals or any(v is None for v in vals):
            return None
        s = sum(parse(v) for v in vals)
        inits = [((c.get("resources") or {}).get("limits") or {}).get(kind) for c in spec.get("initContainers") or []]
        return max([s] + [parse(v) for v in inits if v is not None])

    mem = total("memory", quantity.parse)
    cpu = total("cpu", quantity.parse)
    return Limits(memory=int(mem) if mem is not None else None, cpu=cpu)


def parse_cpulist(text: str) -> list[int]:
    out: list[int] = []
    for part in (text or "").strip().split(","):
        if not part:
            continue
        lo, _, hi = part.partition("-")
        out += range(int(lo), int(hi or lo) + 1)
    return out


def format_cpulist(cpus) -> str:
    cpus = sorted(set(cpus))
    out, i = [], 0
    while i < len(cpus):
        j = i
        while j + 1 < len(cpus) and cpus[j + 1] == cpus[j] + 1:
            j += 1
        out.append(str(cpus[i]) if i == j else f"{cpus[i]}-{cpus[j]}")
        i = j + 1
    return ",".join(out)


def sysfs_root() -> Path:
    return Path(os.environ.get("TK8S_SYSFS_ROOT", "/sys"))


def gpu_local_cpus(render_minors) -> str:
    """The CPUs NUMA-local to these GPUs (``/sys/class/drm/renderD<m>/device/local_cpulist``)
    that this process may run on, as one list; "" when unknown or none of them is ours (a
    cpuset that keeps the agent off that socket: the pod is then not pinned rather than
    unstartable). On an MI355X node, GPUs 0-3 sit on socket 0 and 4-7 on 1."""
    cpus: set[int] = set()
    for m in render_minors:
        if m is None or int(m) < 0:
            continue
        try:
            cpus |= set(parse_cpulist((sysfs_root() / "class" / "drm" / f"renderD{int(m)}" / "device" /
                                       "local_cpulist").read_text()))
        except (OSError, ValueError):
            continue
    if cpus and hasattr(os, "sched_getaffinity"):
        cpus &= os.sched_getaffinity(0)
    return format_cpulist(cpus) if cpus else ""


def _own_cgroups() -> dict[str, str]:
    """controller (or "" for v2) -> this process's cgroup path, from /proc/self/cgroup."""
    out = {}
    try:
        for line in Path("/proc/self/cgroup").read_text().splitlines():
            _, ctrls, path = line.split(":", 2)
            for c in (ctrls.split(",") if ctrls else [""]):
                out[c] = path
    except (OSError, ValueError):
        pass
    return out


SWEEP_MIN_AGE_S = 60.0


def _sweep(parent: Path) -> None:
    """Remove the machine cgroups under ``parent`` that hold no process any more (an agent killed
    before it could clean up): rmdir of a cgroup fails while anything lives in it, and a live
    agent lives in its own machine's (``Enforcer``), so a live cluster's cgroups stay. One made in
    the last minute is left alone: its agent may be between the mkdir and moving itself in."""
    def live(m: Path) -> bool:  # its agent still runs in it (v1: the machine itself, v2: its leaf)
        for f in (m / "cgroup.procs", m / "agent" / "cgroup.procs"):
            try:
                if f.read_text().split():
                    return True
            except OSError:
                pass
        return False

    import time

    try:
        for m in parent.glob("tk8s-machine-*"):
            try:
                young = time.time() - m.stat().st_ctime < SWEEP_MIN_AGE_S
            except OSError:
                continue
            if young or live(m):
                continue
            for d in m.glob("pod-*"):
                try:
                    os.rmdir(d)
                except OSError:
                    pass
            try:
                os.rmdir(m)
            except OSError:
                pass
    except OSError:
        pass


def detect_mode() -> tuple[str, str]:
    """(mode, why) the Enforcer of a node agent on this host would pick, found without creating
    or moving anything (``./tk8s doctor``)."""
    want = os.environ.get("TK8S_POD_RESOURCES", "auto")
    if want == "none":
        return "none", "disabled (TK8S_POD_RESOURCES=none)"
    if want not in ("auto", "cgroup2", "cgroup1", "watchdog"):
        return "none", f"unknown TK8S_POD_RESOURCES={want!r}"
    root = Path(os.environ.get("TK8S_CGROUP_ROOT", "/sys/fs/cgroup"))
    own = _own_cgroups()
    why = []
    if want in ("auto", "cgroup2"):
        d = root / own.get("", "/").lstrip("/")
        try:
            have = set((d / "cgroup.controllers").read_text().split()) if (root / "cgroup.controllers").exists() else set()
        except OSError:
            have = set()
        if {"memory", "cpu"} <= have and os.access(d / "cgroup.subtree_control", os.W_OK):
            return "cgroup2", f"delegated subtree {d}"
        why.append(f"cgroup2: {d} not delegated" if have else "cgroup2: not a unified hierarchy")
    if want in ("auto", "cgroup1"):
        d = root / "memory" / own.get("memory", "/").lstrip("/")
        if "memory" in own and (root / "memory" / "cgroup.procs").exists() and os.access(d, os.W_OK):
            return "cgroup1", f"writable memory hierarchy {d}"
        why.append("cgroup1: no writable memory hierarchy")
    if want in ("auto", "watchdog"):
        return "watchdog", "; ".join(why)
    return "none", "; ".join(why)


def _own_supervisor() -> int | None:
    """This agent's restart supervisor: its parent, when that is ``tk8s-supervise``."""
    ppid = os.getppid()
    try:
        with open(f"/proc/{ppid}/comm") as f:
            comm = f.read().strip()
    except OSError:
        return None
    return ppid if comm == "tk8s-supervise" else None


def _write(path: Path, value) -> None:
    with open(path, "w") as f:
        f.write(f"{value}\n")


class Enforcer:
    """One per node agent: ``pod(key, limits)`` before a pod starts (its cgroup, the jail options
    that put it there), ``oom_killed(key)`` after a container exits, ``release(key)`` when the pod
    is gone; ``watch(...)`` runs the memory watchdog (watchdog mode)."""

    def __init__(self, node: str, machine: Limits | None = None, scope: str = ""):
        # the machine cgroup's name: the node's, plus a hash of ``scope`` (its sandbox) -- clusters
        # side by side on one host may each have a kubenode1
        import hashlib

        self.node = _NAME.sub("_", node) + (f"-{hashlib.sha1(scope.encode()).hexdigest()[:8]}" if scope else "")
        self.machine = machine or Limits()
        self.root = Path(os.environ.get("TK8S_CGROUP_ROOT", "/sys/fs/cgroup"))
        self.mode, self.why = "none", ""
        self.base: dict[str, Path] = {}    # controller -> the machine cgroup ("" = v2)
        self.pods: dict[str, dict[str, Path]] = {}
        self.limits: dict[str, Limits] = {}
        self.oom: set[str] = set()          # pods the watchdog killed for memory
        self.oom_base: dict[str, int] = {}  # pod key -> the cgroup's oom_kill count when its container started
        self.outside: set[str] = set()      # host-scoped pods: beside the machine's slice, not in it
        self.throttle = CpuThrottle(self.machine.cpu)
        self.lock = threading.Lock()
        want = os.environ.get("TK8S_POD_RESOURCES", "auto")
        if want == "none":
            self.why = "disabled (TK8S_POD_RESOURCES=none)"
            return
        for mode in (("cgroup2", "cgroup1", "watchdog") if want == "auto" else (want,)):
            try:
                if getattr(self, f"_setup_{mode}")():
                    self.mode = mode
                    return
            except OSError as e:
                self.why += f"{mode}: {e}; "
                self._undo()
        if self.mode == "none":
            self.why = self.why or "no mode available"

    # ---- modes -----------------------------------------------------------------------------
    def _setup_cgroup2(self) -> bool:
        if not (self.root / "cgroup.controllers").exists():
            self.why += "cgroup2: not a unified hierarchy; "
            return False
        own = self.root / _own_cgroups().get("", "/").lstrip("/")
        have = set((own / "cgroup.controllers").read_text().split())
        if not {"memory", "cpu"} <= have or not os.access(own / "cgroup.subtree_control", os.W_OK):
            self.why += f"cgroup2: {own} is not delegated to this user (controllers {sorted(have)}); "
            return False
        # no internal processes: this agent moves to a leaf first -- with its own restart supervisor
        # (tk8s-supervise, the agent's parent, always shares its cgroup and supervises
        # nothing else) -- and nothing else (other processes sharing the cgroup, say the
        # other node agents of the host starting at the same moment, are not ours to move; with
        # them there the subtree cannot be enabled)
        leaf = own / "tk8s-agent"
        leaf.mkdir(exist_ok=True)
        mine = [str(os.getpid())]
        sup = _own_supervisor()
        procs = (own / "cgroup.procs").read_text().split()
        if sup is not None and str(sup) in procs:
            mine.append(str(sup))
        for p in mine:
            _write(leaf / "cgroup.procs", p)
        others = [p for p in procs if p not in mine]
        if others and not (own / "cgroup.subtree_control").read_text().split():
            for p in mine:
                _write(own / "cgroup.procs", p)  # back where they were
            self.why += (f"cgroup2: {own} also holds processes that are not this agent's ({', '.join(others[:5])}); "
                         "give each agent a delegated cgroup of its own; ")
            return False
        ctrls = [c for c in ("memory", "cpu", "cpuset") if c in have]
        _write(own / "cgroup.subtree_control", " ".join(f"+{c}" for c in ctrls))
        _sweep(own)
        m = own / f"tk8s-machine-{self.node}"
        m.mkdir(exist_ok=True)
        self.base = {"": m}  # (what _undo removes if this mode fails)
        (m / "agent").mkdir(exist_ok=True)  # the agent lives in its machine (a leaf: no internal processes)
        _write(m / "agent" / "cgroup.procs", os.getpid())
        _write(m / "cgroup.subtree_control", " ".join(f"+{c}" for c in ctrls))
        self._limit(m, "", self.machine)
        self.base = {"": m}
        return True

    def _setup_cgroup1(self) -> bool:
        own = _own_cgroups()
        base = {}
        for c in ("memory", "cpu", "cpuset"):
            hier = self.root / c
            if c not in own or not (hier / "cgroup.procs").exists():
                continue
            d = hier / own[c].lstrip("/")
            if not os.access(d, os.W_OK):
                continue
            _sweep(d)
            m = d / f"tk8s-machine-{self.node}"
            m.mkdir(exist_ok=True)
            base[c] = self.base[c] = m  # (self.base: what _undo removes if this mode fails)
            if c == "cpuset":  # a v1 cpuset starts empty: inherit the parent's before any task joins
                for f in ("cpuset.cpus", "cpuset.mems"):
                    if not (m / f).read_text().strip():
                        _write(m / f, (d / f).read_text().strip())
        if "memory" not in base:
            self.why += "cgroup1: no writable memory hierarchy; "
            self._undo()
            return False
        self.base = base
        for c, m in base.items():
            self._limit(m, c, self.machine)
            _write(m / "cgroup.procs", os.getpid())  # the agent lives in its machine: no sweep takes it
        return True

    def _setup_watchdog(self) -> bool:
        return True

    def _undo(self) -> None:
        """A cgroup mode failed half way: the agent goes back where it was, nothing of the mode
        stays (a later mode must not think a cpuset fences its pods)."""
        for ctrl, m in self.base.items():
            try:
                if ctrl == "":
                    _write(m.parent / "tk8s-agent" / "cgroup.procs", os.getpid())
                    os.rmdir(m / "agent")
                else:
                    _write(m.parent / "cgroup.procs", os.getpid())
                os.rmdir(m)
            except OSError:
                pass
        self.base = {}

    # ---- limits ----------------------------------------------------------------------------
    def _limit(self, d: Path, ctrl: str, lim: Limits) -> None:
        """Write ``lim`` into cgroup ``d`` (``ctrl`` "" = v2, else the v1 controller)."""
        if ctrl == "":
            if lim.memory:
                _write(d / "memory.max", int(lim.memory))
                if (d / "memory.swap.max").exists():
                    _write(d / "memory.swap.max", 0)
                if (d / "memory.oom.group").exists():
                    _write(d / "memory.oom.group", 1)  # an OOM kill takes the whole pod, as the kubelet sets it
            if lim.cpu:
                _write(d / "cpu.max", f"{max(1000, int(lim.cpu * CFS_PERIOD_US))} {CFS_PERIOD_US}")
            if lim.cpus and (d / "cpuset.cpus").exists():
                _write(d / "cpuset.cpus", lim.cpus)
        elif ctrl == "memory" and lim.memory:
            _write(d / "memory.limit_in_bytes", int(lim.memory))
        elif ctrl == "cpu" and lim.cpu:
            _write(d / "cpu.cfs_period_us", CFS_PERIOD_US)
            _write(d / "cpu.cfs_quota_us", max(1000, int(lim.cpu * CFS_PERIOD_US)))
        elif ctrl == "cpuset" and lim.cpus:
            _write(d / "cpuset.cpus", lim.cpus)

    def pod(self, key: str, lim: Limits, in_machine: bool = True, gpu: bool = False) -> list[str]:
        """Prepare pod ``key``: its cgroups, and the jail options that put its processes in them
        (and on its CPUs). ``in_machine=False``: a host-scoped pod (the fabric check's one
        process over the GPUs of several machines) sits beside the machine, not inside its slice.
        ``gpu``: the pod holds GPUs (no RLIMIT_DATA backstop: the GPU runtime's private writable
        reservations are not resident memory -- on the MI355X a HIP process with one GPU holds
        ~400 MiB VmData, torch 1.44 GiB VmData for 1.0 GiB RSS, plus every pinned host buffer,
        profiles/r5_rlimit_gpu -- and grow with the GPUs it opens, so a bound fitted to one GPU
        would fail an 8-GPU pod at start; the sampler enforces its limit)."""
        with self.lock:
            self.limits.pop(key, None)
            self.limits[key] = lim  # (insertion order: the newest pod last, for the machine's memory)
            self.oom.discard(key)
            self.oom_base.pop(key, None)
            with self.throttle.lock:
                self.throttle.exempt.discard(key)
            if in_machine:
                self.outside.discard(key)
            else:
                self.outside.add(key)
        opts: list[str] = []
        if self.mode == "watchdog" and lim.memory and not gpu:
            opts += ["--rlimit-data", str(rlimit_data_for(lim.memory))]
        if self.mode in ("cgroup2", "cgroup1"):
            name = "pod-" + _NAME.sub("_", key)
            dirs = {}
            for ctrl, base in self.base.items():
                d = (base if in_machine else base.parent) / name
                d.mkdir(exist_ok=True)
                if ctrl == "cpuset":
                    for f in ("cpuset.cpus", "cpuset.mems"):
                        if not (d / f).read_text().strip():
                            _write(d / f, (d.parent / f).read_text().strip())
                self._limit(d, ctrl, lim)
                dirs[ctrl] = d
                opts += ["--cgroup-procs", str(d / "cgroup.procs")]
            with self.lock:
                self.pods[key] = dirs
            self.reset_oom(key)  # (the baseline of a cgroup that outlived an earlier pod of this name)
        if lim.cpus and not (self.mode == "cgroup2" and (self.base[""] / "cpuset.cpus").exists()) \
                and "cpuset" not in self.base:
            opts += ["--cpus", lim.cpus]  # no cpuset controller: affinity
        return opts

    def oom_killed(self, key: str) -> bool:
        """Was the last kill in pod ``key`` an out-of-memory kill?"""
        with self.lock:
            if key in self.oom:
                return True
            dirs = self.pods.get(key) or {}
        n = self._oom_kills(dirs)
        if n is None:
            return False
        with self.lock:
            base = self.oom_base.get(key, 0)
        # the counters are cumulative over the cgroup's life: only a kill since this container
        # instance started counts, not one of an earlier instance
        if n > base:
            return True
        if "memory" in dirs and "" not in dirs:
            try:
                return int((dirs["memory"] / "memory.failcnt").read_text()) > 0
            except (OSError, ValueError):
                pass
        return False

    @staticmethod
    def _oom_kills(dirs: dict) -> int | None:
        """The pod cgroup's cumulative oom_kill count (v2 memory.events, v1 memory.oom_control)."""
        try:
            if "" in dirs:
                ev = dict(line.split() for line in (dirs[""] / "memory.events").read_text().splitlines() if line.strip())
                return int(ev.get("oom_kill", 0))
            if "memory" in dirs:
                ctl = dict(line.split() for line in (dirs["memory"] / "memory.oom_control").read_text().splitlines()
                           if len(line.split()) == 2)
                return int(ctl.get("oom_kill", 0))
        except (OSError, ValueError):
            pass
        return None

    def reset_oom(self, key: str) -> None:
        """A container (re)starts: its exit is judged on its own -- the oom_kill count from here on."""
        with self.lock:
            self.oom.discard(key)
            dirs = self.pods.get(key) or {}
        n = self._oom_kills(dirs)
        with self.lock:
            self.oom_base[key] = n or 0
        if "memory" in dirs:  # v1 counts failures cumulatively: reset between instances
            try:
                _write(dirs["memory"] / "memory.failcnt", 0)
            except OSError:
                pass

    def release(self, key: str) -> None:
        with self.lock:
            dirs = self.pods.pop(key, {})
            self.limits.pop(key, None)
            self.oom.discard(key)
            self.oom_base.pop(key, None)
            self.outside.discard(key)
        self.throttle.resume(key)
        for d in dirs.values():
            try:
                os.rmdir(d)
            except OSError:
                pass

    def close(self) -> None:
        """The agent is going away: every pod cgroup it made, then its machine's, are removed
        (those still holding a process stay)."""
        for key in list(self.pods):
            self.release(key)
        self.throttle.resume_all()
        for ctrl, base in self.base.items():
            try:  # leave it for the parent (v1: the agent itself; v2: its leaf) and remove it
                if ctrl == "":
                    _write(base.parent / "tk8s-agent" / "cgroup.procs", os.getpid())
                    os.rmdir(base / "agent")
                else:
                    _write(base.parent / "cgroup.procs", os.getpid())
                os.rmdir(base)
            except OSError:
                pass

    def describe(self) -> str:
        m = self.machine
        shape = ", ".join(x for x in (f"memory {m.memory >> 20} MiB" if m.memory else "",
                                      f"cpu {m.cpu:g}" if m.cpu else "", f"cpus {m.cpus}" if m.cpus else "") if x)
        if self.mode == "cgroup2":
            return f"cgroup2 ({self.base[''].parent}): pod memory.max, cpu.max, cpuset; machine {shape or 'unbounded'}"
        if self.mode == "cgroup1":
            return (f"cgroup1 ({', '.join(sorted(self.base))}): pod memory, cfs quota, cpuset; "
                    f"machine {shape or 'unbounded'}")
        if self.mode == "watchdog":
            mach = ", ".join(x for x in (f"cpu {m.cpu:g} by the same duty cycle over all its pods" if m.cpu else "",
                                          f"memory {m.memory >> 20} MiB over all its pods' resident sets (the newest "
                                          "pod OOMKilled)" if m.memory else "") if x)
            return ("watchdog: limits.cpu by a SIGSTOP/SIGCONT duty cycle over each pod's processes (/proc CPU-time "
                    f"deltas every {TICK_S * 1000:.0f} ms); limits.memory by resident-set sampling (OOMKilled) with an "
                    "RLIMIT_DATA backstop for CPU pods; machine package: " + (mach or "unbounded")
                    + "; GPU pods pinned to NUMA-local CPUs (no delegated cgroup: " + self.why.strip("; ") + ")")
        return f"none: {self.why.strip('; ')}"

    # ---- the watchdog (watchdog mode) -------------------------------------------------------
    def over_limit(self, rss: dict[str, int]) -> list[str]:
        """Pods whose resident set (``rss``: key -> bytes) is over their limits.memory."""
        with self.lock:
            return [k for k, b in rss.items() if (self.limits.get(k) or Limits()).memory and b > self.limits[k].memory]

    def kill_oom(self, key: str, groups: list[int], pids=(), starts: dict[int, int] | None = None) -> None:
        """SIGKILL a pod's process groups and members (those that left the group: usage.members),
        each only while it is the process the scan saw (``starts``: pid -> start ticks)."""
        with self.lock:
            self.oom.add(key)
        if starts is None:
            from ..utils.procs import proc_start_ticks

            starts = {p: proc_start_ticks(p) for p in (*groups, *pids)}
        signal_ids(groups, pids, signal.SIGKILL, starts)

    def over_machine(self, rss: dict[str, int]) -> list[str]:
        """When the machine's pods together are over its package's memory: the pods to kill, the
        newest first, until the rest fit (host-scoped pods sit outside the slice)."""
        if not self.machine.memory:
            return []
        with self.lock:
            order = [k for k in self.limits if k in rss and k not in self.outside]
        order += [k for k in rss if k not in order and k not in self.outside]  # (pods started before any limit)
        total = sum(rss[k] for k in order)
        out = []
        while order and total > self.machine.memory:
            k = order.pop()  # the newest
            out.append(k)
            total -= rss[k]
        return out

    def watch(self, groups_of, stop: threading.Event, period: float = 0.5) -> None:
        """Watchdog loop: ``groups_of()`` -> {pod key: [process group ids]}. Every ``period`` s a
        /proc scan finds each pod's processes and resident set (memory limits, the machine's
        memory); every ``TICK_S`` the CPU duty cycle runs over the processes last found."""
        if self.mode != "watchdog":
            return
        from .usage import _proc_table, child_map, members

        pods: dict[str, tuple[list[int], set[int]]] = {}
        last = time.monotonic()
        next_scan = last + period  # (never a /proc scan in the agent right as its first pod starts)
        try:
            while not stop.wait(TICK_S):
                with self.lock:
                    limits = dict(self.limits)
                cpu_on = any(lim.cpu for lim in limits.values()) or bool(self.machine.cpu and limits)
                mem_on = any(lim.memory for lim in limits.values()) or bool(self.machine.memory and limits)
                now = time.monotonic()
                if not (cpu_on or mem_on):
                    self.throttle.resume_all()
                    pods, last, next_scan = {}, now, now + period
                    continue
                if now >= next_scan:
                    next_scan = now + period
                    groups = groups_of()
                    table = _proc_table()
                    kids = child_map(table)
                    pods, rss = {}, {}
                    for key, gs in groups.items():
                        ps = set().union(*(members(table, g, kids) for g in gs)) if gs else set()
                        pods[key] = (list(gs), ps)
                        rss[key] = sum(table[p][2] for p in ps if p in table)
                    self.throttle.starts = {p: v[5] for p, v in table.items()}
                    if mem_on:
                        for key in dict.fromkeys(self.over_limit(rss) + self.over_machine(rss)):
                            self.throttle.resume(key)  # (a stopped process dies of SIGKILL all the same)
                            self.kill_oom(key, pods[key][0], sorted(pods[key][1]), self.throttle.starts)
                            pods.pop(key, None)
                            time.sleep(0)  # the runtime's wait() sees the kill; oom_killed() names it
                if cpu_on:
                    self.throttle.step(pods, limits, now - last, in_machine=lambda k: k not in self.outside)
                elif self.throttle.stopped:
                    self.throttle.resume_all()
                last = now
        finally:
            self.throttle.resume_all()
