#!/usr/bin/env python3
"""Headline benchmark: wall-clock of ``./setup.sh`` -> all nodes Ready on the MI355X host.

Metric (BASELINE.json): "wall-clock (s) ./setup.sh -> all nodes Ready; 1/2/4/8 workers".
``--gpus N`` brings up 1 master + N workers with the ``mi355x-1gpu`` package, i.e. one
MI355X per worker, so N workers make N x ``amd.com/gpu`` allocatable (weak scaling: the
per-worker work is fixed, the cluster grows with N).

One *step* is one complete, non-interactive bring-up in a fresh workspace:

    ./setup.sh --answers <N workers, mi355x-1gpu> --yes
      configure -> provision (terraform/{master,host}) -> ansible/clusterUp.yml
      (rocmsetup, control plane + environment, worker join + device plugin)
      -> every worker heartbeating AND validated on its GPU (tk8s-probe: gfx950 discovery,
         1 GiB HBM write, 256 MiB MD5; the benchmarks.md analogues) -> amd.com/gpu == N
      -> (N >= 2) RCCL all-reduce Job over all N GPUs, one rank per GPU, checked exactly

``value`` is the wall-clock from launching ``./setup.sh`` to the moment it prints
``ALL NODES READY`` (bench.py streams its stdout and timestamps that line): interpreter
start-up, provisioning, the playbook, the control plane, agent joins and per-GPU validation
are all inside. The step brackets (``ms_per_step``) cover the whole ``./setup.sh`` process,
which after Ready also runs the RCCL all-reduce Job over all N GPUs (N >= 2), reported as
``rccl_check_s`` / ``rccl_peak_busbw_gbps``. The teardown (``./setup.sh -c``) after each
step runs outside the timed brackets, followed by a ``--settle`` pause (default 1 s on a GPU
host): the amdgpu driver releases an exited GPU process asynchronously, and a new process that
starts the HIP runtime within ~0.1-0.2 s of that exit waits for it (``hsa_init`` 45-65 ms on a
settled host vs 100-230 ms right after one; profiles/r1_init_costs/init_costs3.json). Without the
pause every step after the first would also time the previous step's GPU teardown, which a real
``./setup.sh`` never sees. The per-step runtime start is reported (``hip_init_ms_steps``). The reference publishes no
bring-up time (BASELINE.json ``published: {}``); ``vs_baseline`` is quoted against the
51 s of fixed sleeps in the reference's bring-up path, a floor the
reference can never go below (setup.sh:36,41,46; terraform/*/main.tf:22;
ansible/roles/ranchermaster/tasks/main.yml:25).

A timed step whose post-Ready RCCL check fails is left out of ``value`` and listed in
``post_ready_errors`` (its Ready time stood, the cluster did not). The first such failure
(warmup steps included) turns the RCCL check off for every later step -- recorded once as
``fabric_disabled_after_step`` with the error's tail -- so a broken fabric costs one bounded
check (``--rccl-op-timeout``, 20 s per wait inside the ranks), never one per step. After the headline, a
single-rank run also measures BASELINE.json configs[1], ``curve_config2``: 1 master + 1/2/4/8
``cpu-only`` workers (no GPU, no device plugin), ``--curve-steps`` timed bring-ups per point.

Multi-GPU launch (driver): ``torch.distributed.run --nproc-per-node N bench.py --gpus N``.
Rank 0 drives the bring-up (it is the operator's shell); every rank joins the barriers
and synchronises its own device around the timed region; the time reported is the MAX
over ranks.
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent
if str(REPO) not in sys.path:
    sys.path.insert(0, str(REPO))

BASELINE_FLOOR_S = 51.0  # reference fixed-sleep floor
METRIC = "wall-clock (s) ./setup.sh → all nodes Ready; 1/2/4/8 workers"


def _free_port() -> int:
    from tritonk8ssupervisor_amd.utils.net import pick_port

    return pick_port("127.0.0.1")


class Dist:
    """Barrier + device sync across the torchrun ranks.

    The barrier runs over gloo (host sockets) even on GPUs: an RCCL barrier would leave ranks
    1..N-1 spinning a kernel on their GPUs -- and a proxy thread on the CPU -- for the whole timed
    bring-up, on the very GPUs the bring-up is validating (and, after Ready, next to the
    cluster's own RCCL fabric check). Each side of a step is still bracketed by
    torch.cuda.synchronize() on every rank's device."""

    def __init__(self):
        self.rank = int(os.environ.get("RANK", "0"))
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.torch = None
        self.cuda = False
        self.pg = False
        try:
            import torch

            self.torch = torch
            self.cuda = torch.cuda.is_available()
        except Exception:  # noqa: BLE001 - torch is optional for the CPU bring-up
            pass
        if self.world > 1 and self.torch is not None:
            import torch.distributed as dist

            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            if self.cuda:
                self.torch.cuda.set_device(self.local_rank)
            dist.init_process_group("gloo")
            self.pg = True

    def sync(self) -> None:
        if self.cuda:
            self.torch.cuda.synchronize()
        if self.pg:
            import torch.distributed as dist

            dist.barrier()
        if self.cuda:
            self.torch.cuda.synchronize()

    def max(self, v: float) -> float:
        if not self.pg:
            return v
        import torch.distributed as dist

        t = self.torch.tensor([v], dtype=self.torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def bcast_obj(self, obj):
        if not self.pg:
            return obj
        import torch.distributed as dist

        box = [obj]
        dist.broadcast_object_list(box, src=0)
        return box[0]

    def close(self) -> None:
        if self.pg:
            import torch.distributed as dist

            dist.destroy_process_group()


def make_workspace(root: Path) -> Path:
    from tritonk8ssupervisor_amd.orchestrator import init_workspace

    init_workspace(root)
    for f in ("setup.sh", "tk8s", "kubectl"):
        shutil.copy2(REPO / f, root / f)
    return root


def child_env(fake_gpus: int | None) -> dict:
    env = dict(os.environ)
    env["PYTHONPATH"] = os.pathsep.join([str(REPO)] + [p for p in env.get("PYTHONPATH", "").split(os.pathsep) if p])
    env["TK8S_PYTHON"] = sys.executable
    # the torchrun rank env must not leak into the cluster's own processes
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK", "ROLE_WORLD_SIZE",
              "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID", "TORCHELASTIC_RESTART_COUNT",
              "TORCHELASTIC_MAX_RESTARTS", "TORCHELASTIC_USE_AGENT_STORE", "TORCHELASTIC_ERROR_FILE",
              "GROUP_WORLD_SIZE", "ROLE_NAME", "OMP_NUM_THREADS_SET"):
        env.pop(k, None)
    if fake_gpus is not None:
        env["TK8S_FAKE_GPUS"] = str(fake_gpus)
    # the RCCL fabric Job (after Ready, N >= 2) logs its init and P2P channel setup, so the JSON's
    # rccl_last_step.transport says what the channels ran over (P2P/IPC vs SHM/NET)
    env.setdefault("NCCL_DEBUG", "INFO")
    env.setdefault("NCCL_DEBUG_SUBSYS", "INIT,P2P")
    return env


def private_registry(env: dict, root: Path) -> None:
    """The bench measures one cluster: claims left on the host by other clusters (say, a test run
    that leaked one) must not keep its GPUs from it."""
    env.setdefault("TK8S_HOST_REGISTRY", str(root / "hostreg"))


KFD_PROC = Path("/sys/class/kfd/kfd/proc")


class KfdCensus:
    """Which processes hold the KFD (``/sys/class/kfd/kfd/proc/<pid>``: every process of the
    host with the GPU driver open, this box's other tenants included) during one bring-up,
    sampled every ``period`` s from before ./setup.sh starts (the previous step's settle pause,
    outside the timed brackets) until its Ready line.
    A slow runtime start (``hsa_init``) of the burn-in is then attributed to what changed in
    the KFD process set just before it: a process exiting (the driver
    tears its GPU state down; a runtime starting meanwhile waits for it), one starting, or
    nothing visible (a driver-internal cause)."""

    def __init__(self, period: float = 0.005):
        self.period = period
        self.events: list[tuple[float, str, str]] = []   # (unix time, "start"|"exit", pid)
        self.initial: set[str] = set()
        self._stop = None
        self._th = None

    @staticmethod
    def snapshot() -> set[str] | None:
        try:
            return {e for e in os.listdir(KFD_PROC) if e.isdigit()}
        except OSError:
            return None

    def start(self) -> "KfdCensus":
        import threading

        first = self.snapshot()
        if first is None:
            return self
        self.initial = first
        self._stop = threading.Event()

        def loop():
            prev = first
            while not self._stop.is_set():
                cur = self.snapshot() or set()
                t = time.time()
                self.events += [(t, "start", p) for p in sorted(cur - prev)]
                self.events += [(t, "exit", p) for p in sorted(prev - cur)]
                prev = cur
                self._stop.wait(self.period)

        self._th = threading.Thread(target=loop, name="kfd-census", daemon=True)
        self._th.start()
        return self

    def stop(self) -> None:
        if self._stop is not None:
            self._stop.set()
            self._th.join(1.0)

    def report(self, spawned_unix: float | None, own_pids: set[str], window: float = 0.3) -> dict:
        """KFD process changes in the ``window`` s before the burn-in was spawned and during its
        runtime start; own_pids: the KFD pids this bring-up's own processes are known by."""
        if self._stop is None:
            return {"available": False}
        out = {"available": True, "present_at_launch": len(self.initial)}
        if spawned_unix is None:
            return out
        lo = spawned_unix - window
        near = [{"dt_ms": round((t - spawned_unix) * 1e3, 1), "what": what, "pid": int(p),
                 "own": p in own_pids} for t, what, p in self.events if t >= lo]
        out["changes"] = near[:40]
        return out


def slow_start_cause(census: dict, runtime_init_ms: float | None, limit_ms: float = 50.0) -> str | None:
    """One line naming what most likely delayed a runtime start over ``limit_ms``."""
    if runtime_init_ms is None or runtime_init_ms <= limit_ms:
        return None
    if not census.get("available"):
        return "unknown: /sys/class/kfd/kfd/proc not readable here"
    window = runtime_init_ms + 1.0  # changes up to the end of the runtime start count
    ch = [c for c in census.get("changes", []) if c["dt_ms"] <= window]
    # The KFD names processes by their pid on the host; inside a container the burn-in's own pid
    # differs, so its entry is recognised by when it appears: as its runtime start ends (within
    # about one sample of the census, 5 ms).
    ours = [c for c in ch if c["what"] == "start" and not c["own"] and abs(c["dt_ms"] - runtime_init_ms) <= 6.0]
    if ours:
        ch = [c for c in ch if c is not ours[0]]
    exits = [c for c in ch if c["what"] == "exit" and c["dt_ms"] <= 0]
    foreign_exit = [c for c in exits if not c["own"]]
    if foreign_exit:
        c = foreign_exit[-1]
        return f"foreign KFD process {c['pid']} exited {-c['dt_ms']:.0f} ms before the burn-in spawned"
    if exits:
        c = exits[-1]
        return f"this bring-up's KFD process {c['pid']} exited {-c['dt_ms']:.0f} ms before the burn-in spawned"
    held = [c for c in ch if c["what"] == "exit" and 0 < c["dt_ms"] and ours and abs(c["dt_ms"] - ours[0]["dt_ms"]) <= 6.0]
    if held:  # its KFD open completed the moment another process's KFD state was released
        c = held[-1]
        return (f"waited for KFD process {c['pid']}'s release: it went away {c['dt_ms']:.0f} ms into the start, "
                f"as the burn-in's own KFD process appeared")
    starts = [c for c in ch if c["what"] == "start" and not c["own"]]
    if starts:
        c = starts[0]
        return f"foreign KFD process {c['pid']} started {c['dt_ms']:+.0f} ms around the burn-in spawn"
    late_exits = [c for c in ch if c["what"] == "exit"]
    if late_exits:
        c = late_exits[0]
        return f"KFD process {c['pid']} exited {c['dt_ms']:.0f} ms into the burn-in's runtime start"
    return "no KFD process change within 0.3 s before or during the start (driver-internal)"


def _probe_libraries() -> list[str]:
    """The shared libraries the GPU burn-in (tk8s-hsaprobe) maps, as the dynamic loader resolves
    them -- the files a first bring-up on a fresh machine reads from disk."""
    probe = REPO / "tritonk8ssupervisor_amd" / "bin" / "tk8s-hsaprobe"
    try:
        out = subprocess.run(["ldd", str(probe)], capture_output=True, text=True, timeout=10).stdout
    except (OSError, subprocess.SubprocessError):
        return []
    libs = [probe.as_posix()]
    for line in out.splitlines():
        parts = line.split("=>")
        if len(parts) == 2 and parts[1].strip().startswith("/"):
            libs.append(parts[1].split("(")[0].strip())
    return libs


def page_cache_residency(paths: list[str]) -> dict:
    """Fraction of each file's pages in the page cache (mincore(2) over a read-only map): what a
    cold first run has to read from disk. Outside the timed region; {} where it cannot be asked."""
    import ctypes
    import mmap

    try:
        libc = ctypes.CDLL(None, use_errno=True)
        libc.mmap.restype = ctypes.c_void_p
        libc.mmap.argtypes = (ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_long)
        libc.munmap.argtypes = (ctypes.c_void_p, ctypes.c_size_t)
        libc.mincore.argtypes = (ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p)
    except (OSError, AttributeError):
        return {}
    page = mmap.PAGESIZE
    out, total, resident = {}, 0, 0
    for p in paths:
        try:
            fd = os.open(p, os.O_RDONLY)
        except OSError:
            continue
        try:
            size = os.fstat(fd).st_size
            if size == 0:
                continue
            addr = libc.mmap(None, size, mmap.PROT_READ, mmap.MAP_SHARED, fd, 0)
            if addr in (None, ctypes.c_void_p(-1).value):
                continue
            try:
                npages = (size + page - 1) // page
                vec = (ctypes.c_ubyte * npages)()
                if libc.mincore(ctypes.c_void_p(addr), size, vec) != 0:
                    continue
                res = sum(b & 1 for b in vec)
            finally:
                libc.munmap(ctypes.c_void_p(addr), size)
            out[os.path.basename(p)] = {"mib": round(size / 2**20, 1), "resident": round(res / npages, 3)}
            total += npages
            resident += res
        finally:
            os.close(fd)
    if total:
        out["_all"] = {"mib": round(total * page / 2**20, 1), "resident": round(resident / total, 3)}
    return out


def slowest_tasks(events: Path, launched_unix: float | None = None, top: int = 6) -> list[dict]:
    """The slowest playbook tasks and provisioning steps of one bring-up (its .tk8s/events.jsonl),
    and the CLI's own start (launch -> its first event): where a slow step's time went, kept in
    the JSON line for the cold first run."""
    out = []
    try:
        for k, line in enumerate(events.read_text().splitlines()):
            e = json.loads(line)
            if k == 0 and launched_unix and e.get("ts"):
                out.append({"what": "CLI start: interpreter + imports (launch -> first event)",
                            "s": round(e["ts"] - launched_unix, 4)})
            if e.get("event") in ("task", "phase_end") and isinstance(e.get("seconds"), (int, float)):
                out.append({"what": e.get("task") or f"phase {e.get('phase')}", "s": round(e["seconds"], 4),
                            **({"timing_ms": e["timing_ms"]} if e.get("timing_ms") else {})})
    except (OSError, ValueError):
        return []
    return sorted(out, key=lambda x: -x["s"])[:top]


def evict_page_cache(paths: list[str]) -> dict:
    """Drop these files' clean pages from the page cache (posix_fadvise DONTNEED: no privilege
    needed, nothing but the cache changes), so the next bring-up reads them from disk -- a first
    ./setup.sh on a machine that has never run it."""
    n, size = 0, 0
    for p in paths:
        try:
            fd = os.open(p, os.O_RDONLY)
        except OSError:
            continue
        try:
            size += os.fstat(fd).st_size
            os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
            n += 1
        except OSError:
            pass
        finally:
            os.close(fd)
    return {"files": n, "mib": round(size / 2**20, 1)}


def one_bringup(ws: Path, n: int, args, env: dict, log, census: KfdCensus | None = None, package: str | None = None,
                rccl: str | None = None) -> dict:
    answers = {"nodes": n, "package": package or args.package, "name": "k8s bench", "confirm": "yes"}
    (ws / "answers.json").write_text(json.dumps(answers))
    cmd = ["./setup.sh", "--answers", "answers.json", "--yes", "--json", "--port", str(_free_port()),
           "--timeout", str(args.timeout), "--rccl-timeout", str(args.rccl_timeout)]
    if args.no_validate:
        cmd.append("--no-validate")
    if rccl or args.rccl:
        cmd += ["--rccl", rccl or args.rccl]
    if getattr(args, "rccl_op_timeout", None):
        cmd += ["--rccl-op-timeout", str(args.rccl_op_timeout)]
    import threading

    census = census or KfdCensus()
    t0 = time.perf_counter()
    launched_unix = time.time()
    p = subprocess.Popen(cmd, cwd=ws, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, bufsize=1,
                         start_new_session=True)
    lines: list[str] = []
    ready_at: list[float] = []
    eof_at: list[float] = []

    def reader():  # stream: the READY line is timestamped as it is printed
        for line in p.stdout:
            if not ready_at and line.startswith("ALL NODES READY"):
                ready_at.append(time.perf_counter() - t0)
                census.stop()
            lines.append(line)
        eof_at.append(time.perf_counter() - t0)

    th = threading.Thread(target=reader, name="setup-stdout", daemon=True)
    th.start()
    killed: list[bool] = []

    def watchdog():  # the bound holds even when setup.sh hangs without printing anything
        killed.append(True)
        try:
            os.killpg(p.pid, 9)
        except OSError:
            pass

    # a blocking wait (waitpid), with the bound on a timer: Popen.wait(timeout=...) polls with a
    # backoff capped at 50 ms, which quantised every step's time
    dog = threading.Timer(args.timeout + 120, watchdog)
    dog.daemon = True
    dog.start()
    try:
        rc = p.wait()
    finally:
        dog.cancel()
    wall = time.perf_counter() - t0
    census.stop()
    th.join(10)
    if killed:
        lines.append(f"\n[bench] ./setup.sh killed after {args.timeout + 120:.0f}s\n")
    t_ready = ready_at[0] if ready_at else None
    out = "".join(lines)
    log.write(out)
    log.flush()
    if t_ready is None:
        raise RuntimeError(f"./setup.sh exited {rc} before every node was Ready:\n{out[-3000:]}")
    post_ready = (eof_at[0] if eof_at else wall) - t_ready
    if rc != 0:
        # Ready was reached (the metric); what failed afterwards is the RCCL fabric check. Keep
        # the measurement and report the failure instead of dropping the whole step.
        return {"wall_seconds": wall, "ready_wall_seconds": t_ready, "post_ready_seconds": post_ready, "phases": {},
                "post_ready_error": f"exit {rc}: " + out.strip()[-1500:]}
    summary = json.loads(out.strip().splitlines()[-1])
    summary["wall_seconds"] = wall
    summary["launched_unix"] = launched_unix
    summary["ready_wall_seconds"] = t_ready
    summary["post_ready_seconds"] = post_ready
    hb = summary.get("host_burnin") or {}
    own = {str(x) for x in (hb.get("pid"), hb.get("kfd_pid")) if x}
    summary["kfd_census"] = census.report(hb.get("spawned_unix"), own)
    summary["slow_start_cause"] = slow_start_cause(summary["kfd_census"], hb.get("runtime_init_ms"))
    hb = summary.get("host_burnin") or {}
    spawned = hb.get("spawned_unix")
    if spawned:  # how long after the launch of ./setup.sh the GPU burn-in process started
        summary["burnin_spawn_ms"] = round((spawned - launched_unix) * 1e3, 2)
        if hb.get("main_unix_ms"):  # exec + dynamic loading until the probe's main()
            summary["burnin_exec_ms"] = round(hb["main_unix_ms"] - spawned * 1e3, 2)
        if hb.get("seen_unix") and hb.get("main_unix_ms") and hb.get("total_ms") is not None:
            # from the probe's result to setup noticing it
            summary["burnin_notice_ms"] = round(hb["seen_unix"] * 1e3 - hb["main_unix_ms"] - hb["total_ms"], 2)
    return summary


def teardown(ws: Path, env: dict, log) -> float:
    t0 = time.perf_counter()
    p = subprocess.run(["./setup.sh", "-c", "--yes"], cwd=ws, env=env, stdout=subprocess.PIPE,
                       stderr=subprocess.STDOUT, text=True, timeout=120)
    log.write(p.stdout)
    log.flush()
    if p.returncode != 0:
        raise RuntimeError(f"./setup.sh -c exited {p.returncode}:\n{p.stdout[-2000:]}")
    return time.perf_counter() - t0


def _stats(xs: list[float]) -> dict:
    srt = sorted(xs)
    mid = len(srt) // 2
    return {"mean_s": round(sum(xs) / len(xs), 4),
            "median_s": round(srt[mid] if len(srt) % 2 else (srt[mid - 1] + srt[mid]) / 2, 4),
            "min_s": round(srt[0], 4), "max_s": round(srt[-1], 4)}


def series(root: Path, name: str, n: int, args, env: dict, log, steps: int, warmup: int = 1, settle: float = 0.0,
           rccl: str | None = None, env_over: dict | None = None) -> dict:
    """``warmup`` untimed then ``steps`` timed bring-ups of 1 master + ``n`` workers of the
    headline's package, each bracketed like a headline step, teardown and workspace outside."""
    step_env = dict(env, **(env_over or {}))
    ready, proc, fabric, rccl_s, last = [], [], [], [], {}
    for i in range(warmup + steps):
        ws = root / f"{name}{i}"
        make_workspace(ws)
        t0 = time.perf_counter()
        s = one_bringup(ws, n, args, step_env, log, rccl=rccl)
        dt = time.perf_counter() - t0
        teardown(ws, env, log)
        shutil.rmtree(ws, ignore_errors=True)
        if s.get("post_ready_error"):
            raise RuntimeError(f"{name} step {i}: {s['post_ready_error'][-800:]}")
        if i >= warmup:
            ready.append(s["ready_wall_seconds"])
            proc.append(dt)
            fabric.append(s["wall_seconds"])
            rccl_s.append(s.get("phases", {}).get("rccl", 0.0))
            last = s
        if settle > 0:
            time.sleep(settle)
    return {"steps": steps, "warmup": warmup, "ready": _stats(ready), "process": _stats(proc),
            "setup_exit": _stats(fabric), "rccl_phase_mean_s": round(sum(rccl_s) / len(rccl_s), 4),
            "last": last}


CURVE_NODES = (1, 2, 4, 8)


def mean_phases(per_step: list[dict]) -> dict:
    """Mean seconds per bring-up phase over a point's timed steps."""
    out: dict[str, float] = {}
    for ph in per_step:
        for k, v in ph.items():
            if isinstance(v, (int, float)):
                out[k] = out.get(k, 0.0) + v / len(per_step)
    return {k: round(v, 4) for k, v in out.items()}


def mean_tasks(per_step: list[list[dict]], top: int = 6) -> list[dict]:
    """A point's slowest tasks: each task's mean over the steps that listed it (slowest_tasks of
    each step), slowest first."""
    acc: dict[str, list[float]] = {}
    for step in per_step:
        for t in step:
            acc.setdefault(t["what"], []).append(t["s"])
    n = max(len(per_step), 1)
    rows = [{"what": k, "mean_s": round(sum(v) / n, 4), "steps": len(v)} for k, v in acc.items()]
    return sorted(rows, key=lambda r: -r["mean_s"])[:top]


def config2_curve(root: Path, args, env: dict, log, steps: int, warmup: int = 1) -> dict:
    """BASELINE.json configs[1]: 1 master + N ``cpu-only`` workers (no GPU, no device plugin),
    N = 1/2/4/8 -- the worker-count curve of the bring-up itself, measurable on a 1-GPU box. Each
    point: ``warmup`` untimed bring-ups then ``steps`` timed ones, each bracketed like the
    headline's (the whole ./setup.sh process; value = launch -> ALL NODES READY), teardown and
    workspace creation outside the brackets."""
    points = []
    t_curve = time.perf_counter()
    for n in getattr(args, "curve_workers", None) or CURVE_NODES:
        ready, proc, phases, tasks = [], [], [], []
        for i in range(warmup + steps):
            ws = root / f"curve{n}-{i}"
            make_workspace(ws)
            t0 = time.perf_counter()
            s = one_bringup(ws, n, args, env, log, package="cpu-only", rccl="off")
            dt = time.perf_counter() - t0
            if i >= warmup:  # where this point's time went, read before the teardown
                phases.append(s.get("phases") or {})
                tasks.append(slowest_tasks(ws / ".tk8s" / "events.jsonl", s.get("launched_unix"), top=12))
                if getattr(args, "keep_events", None) and (ws / ".tk8s" / "events.jsonl").exists():
                    Path(args.keep_events).mkdir(parents=True, exist_ok=True)
                    shutil.copy2(ws / ".tk8s" / "events.jsonl", Path(args.keep_events) / f"curve{n}-{i}.events.jsonl")
            teardown(ws, env, log)
            shutil.rmtree(ws, ignore_errors=True)
            if i >= warmup:
                ready.append(s["ready_wall_seconds"])
                proc.append(dt)
        srt = sorted(ready)
        points.append({"workers": n, "steps": steps, "mean_s": round(sum(ready) / len(ready), 4),
                       "median_s": round(srt[len(srt) // 2] if len(srt) % 2 else (srt[len(srt) // 2 - 1] + srt[len(srt) // 2]) / 2, 4),
                       "min_s": round(srt[0], 4), "max_s": round(srt[-1], 4),
                       "ms_per_step": round(sum(proc) / len(proc) * 1000.0, 2), "gpus_allocatable": s.get("gpus_allocatable"),
                       "nodes": s.get("nodes"), "phases_s": mean_phases(phases),
                       "slowest_tasks": mean_tasks(tasks)})
    return {"config": "BASELINE.json configs[1]: 1 master + N cpu-only workers, no GPU device plugin",
            "package": "cpu-only", "warmup": warmup, "points": points,
            "wall_s": round(time.perf_counter() - t_curve, 3),
            "scaling_8_vs_1": round(points[-1]["mean_s"] / points[0]["mean_s"], 3)
            if len(points) > 1 and points[0]["workers"] == 1 and points[-1]["workers"] == 8 else None,
            # the same ratio of the medians: one slow step among 5 moves the means' ratio by ~0.1
            "scaling_8_vs_1_median": round(points[-1]["median_s"] / points[0]["median_s"], 3)
            if len(points) > 1 and points[0]["workers"] == 1 and points[-1]["workers"] == 8 else None}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1, help="workers (one MI355X each)")
    ap.add_argument("--steps", type=int, default=10)  # one 150 ms KFD wait (another process's release) moves a 3-step mean by 50 ms
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--package", default="mi355x-1gpu")
    ap.add_argument("--timeout", type=float, default=300.0, help="bound on one bring-up's readiness wait (s)")
    ap.add_argument("--no-validate", action="store_true", help="skip per-worker GPU validation (not the headline)")
    ap.add_argument("--rccl", choices=["on", "off"], default=None)
    ap.add_argument("--rccl-timeout", type=float, default=120.0, help="bound on the post-Ready RCCL Job (s)")
    ap.add_argument("--rccl-op-timeout", type=float, default=None,
                    help="bound on each wait inside an RCCL rank (default: ./setup.sh's, 20 s)")
    ap.add_argument("--fake-gpus", type=int, default=None,
                    help="CPU rehearsal: N fake gfx950 devices (default: fake 8 when no GPU is present)")
    ap.add_argument("--workdir", default=None, help="parent of the per-step workspaces (default: a tempdir)")
    ap.add_argument("--log", default=None, help="append setup.sh output here")
    ap.add_argument("--keep-events", default=None, help="copy each step's .tk8s/events.jsonl into this directory")
    ap.add_argument("--back-to-back", type=int, default=None,
                    help="after the timed steps, this many extra bring-ups with NO settle pause (a rebuild right "
                         "after a teardown), reported separately as back_to_back_* (default: 2 with real GPUs)")
    ap.add_argument("--curve-steps", type=int, default=5,
                    help="timed steps per point of the cpu-only worker curve (BASELINE configs[1], 1/2/4/8 workers) "
                         "run after the headline on a single-rank run; 0 skips it")
    ap.add_argument("--curve-workers", type=lambda s: [int(x) for x in s.split(",") if x.strip()], default=None,
                    help="the curve's worker counts, comma separated (default 1,2,4,8)")
    ap.add_argument("--plain-steps", type=int, default=5,
                    help="timed bring-ups with TK8S_SHORTCUTS=0 (every start-up shortcut off), reported as "
                         "plain_path_s on a single-rank run; 0 skips them")
    ap.add_argument("--fabric-steps", type=int, default=None,
                    help="timed bring-ups with --rccl on, reported as fabric_validated_s (launch -> ./setup.sh exits "
                         "after a passing RCCL all-reduce Job); default 5 with real GPUs, 0 with fake ones")
    ap.add_argument("--cold-evict", action="store_true",
                    help="before the cold first run, evict every file a bring-up reads from the page cache "
                         "(posix_fadvise DONTNEED), so it also reads them from disk")
    ap.add_argument("--settle", type=float, default=None,
                    help="pause after each teardown, outside the timed region, so the driver has released the "
                         "previous step's GPU processes (default: 1.0 s with real GPUs, 0 with fake ones)")
    args = ap.parse_args(argv)

    d = Dist()
    n = args.gpus
    fake = args.fake_gpus
    if fake is None and not d.cuda and not _has_kfd_gpus():
        fake = max(8, n)
    settle = args.settle if args.settle is not None else (0.0 if fake else 1.0)
    root = Path(args.workdir) if args.workdir else Path(tempfile.mkdtemp(prefix="tk8s-bench-", dir=os.environ.get("TMPDIR", "/tmp")))
    root.mkdir(parents=True, exist_ok=True)
    times: list[float] = []
    excluded: list[dict] = []   # timed steps whose post-Ready RCCL check failed
    summaries: list[dict] = []
    teardown_s: list[float] = []
    ready_times: list[float] = []
    err = None
    # what the cold first run starts from: the byte-code cache the tree came
    # with, and how much of the burn-in's shared libraries the page cache already holds
    cold_start_state: dict = {}
    if d.rank == 0:
        pyc = REPO / "build" / "pycache"
        cold_start_state = {"build_pycache_files_at_start": sum(1 for _ in pyc.rglob("*.pyc")) if pyc.is_dir() else 0,
                            "probe_libs_page_cache_at_start": page_cache_residency(_probe_libraries())}
        from tritonk8ssupervisor_amd.utils.build_native import build

        build()  # incremental; no-op when the in-tree build is current
    env = child_env(fake)
    private_registry(env, root)
    log = open(args.log, "a") if (args.log and d.rank == 0) else open(os.devnull, "w")
    b2b = args.back_to_back if args.back_to_back is not None else (0 if fake else 2)
    b2b_ready: list[float] = []
    b2b_detail: list[dict] = []
    cold: dict | None = None
    # the first post-Ready fabric failure turns the RCCL check off for every later
    # step (recorded once), so a broken fabric costs one deadline, not one per step
    fabric_disabled: dict | None = None
    total = args.warmup + args.steps
    census = KfdCensus().start() if d.rank == 0 else None
    try:
        for i in range(total + b2b):
            timed = args.warmup <= i < total
            extra = i >= total
            ws = root / f"step{i}"
            if d.rank == 0:
                make_workspace(ws)
            d.sync()
            t0 = time.perf_counter()
            s = None
            if d.rank == 0 and err is None:
                step_env = env
                if i == 0 and args.warmup > 0:
                    # the first step runs cold: empty byte-code and parse caches, i.e. a user's
                    # first ./setup.sh on a fresh install
                    step_env = dict(env, PYTHONPYCACHEPREFIX=str(root / "cold-pycache"),
                                    TK8S_YAML_CACHE=str(root / "cold-cache"))
                    if args.cold_evict:  # ... and on a machine whose disk cache has never seen it
                        from tritonk8ssupervisor_amd.utils.build_native import bringup_files

                        files = bringup_files(env, relative=False)
                        cold_start_state["evicted"] = evict_page_cache(files)
                        cold_start_state["bringup_files_page_cache_after_evict"] = (
                            page_cache_residency(files).get("_all"))
                try:
                    if i == 0 and args.warmup > 0:
                        cold_start_state.update(loadavg_1m=round(os.getloadavg()[0], 2),
                                                cpus=len(os.sched_getaffinity(0)))
                    s = one_bringup(ws, n, args, step_env, log, census,
                                    rccl="off" if fabric_disabled is not None else None)
                    if s.get("post_ready_error") and fabric_disabled is None:
                        fabric_disabled = {"after_step": i, "kind": "timed" if timed else "back-to-back" if extra
                                           else "warmup", "error_tail": s["post_ready_error"][-800:]}
                    if i == 0 and args.warmup > 0:
                        cold = s
                        cold["slowest_tasks"] = slowest_tasks(ws / ".tk8s" / "events.jsonl", s.get("launched_unix"))
                except Exception as e:  # noqa: BLE001 - reported after the collective
                    err = str(e)
            d.sync()
            dt = time.perf_counter() - t0
            err = d.bcast_obj(err)
            if d.rank == 0:
                if args.keep_events and (ws / ".tk8s" / "events.jsonl").exists():
                    Path(args.keep_events).mkdir(parents=True, exist_ok=True)
                    shutil.copy2(ws / ".tk8s" / "events.jsonl", Path(args.keep_events) / f"step{i}.events.jsonl")
                try:
                    teardown_s.append(teardown(ws, env, log))
                except Exception as e:  # noqa: BLE001 - a failed step is already reported
                    if err is None:
                        err = str(e)
                shutil.rmtree(ws, ignore_errors=True)
                if census is not None:
                    census.stop()
                census = KfdCensus().start()  # the next step's census starts before its settle pause
                if settle > 0 and i + 1 < total:  # no pause before the back-to-back steps / between them
                    time.sleep(settle)
            err = d.bcast_obj(err)
            if err is not None:
                if extra:  # a failed back-to-back step does not void the measurement
                    err = None
                break
            if extra:
                b2b_ready.append(d.max(s["ready_wall_seconds"] if s else 0.0))
                if s is not None:  # where a rebuild right after a teardown spends its extra time
                    hb = s.get("host_burnin") or {}
                    b2b_detail.append({"ready_s": s.get("ready_wall_seconds"), "burnin_runtime_init_ms": hb.get("runtime_init_ms"),
                                       "burnin_total_ms": hb.get("total_ms"), "previous_teardown_s": teardown_s[-2] if len(teardown_s) > 1 else None,
                                       "phases_s": {k: round(v, 4) for k, v in (s.get("phases") or {}).items()},
                                       "slow_start_cause": slow_start_cause(s.get("kfd_census") or {}, hb.get("runtime_init_ms")),
                                       "kfd_census": s.get("kfd_census")})
            if timed:
                bad = d.bcast_obj(bool(s and s.get("post_ready_error")) if d.rank == 0 else None)
                if bad:  # Ready was reached but the post-Ready fabric check failed: flagged, not counted
                    excluded.append({"step": i, "error": s["post_ready_error"][-600:] if s else ""})
                else:
                    times.append(d.max(dt))
                    ready_times.append(d.max(s["ready_wall_seconds"] if s else 0.0))
                    if s is not None:
                        summaries.append(s)
            if d.rank == 0:
                kind = "timed" if timed else "back-to-back" if extra else "warmup"
                print(f"[bench] step {i} ({kind}): {dt:.3f}s", file=sys.stderr, flush=True)
    finally:
        if census is not None:
            census.stop()
        log.close()
        if d.rank == 0 and not args.workdir:
            shutil.rmtree(root, ignore_errors=True)
    d.close()
    if d.rank != 0:
        return 0 if err is None else 1
    if err is None and not times:
        err = f"every timed step failed its post-Ready RCCL check: {excluded[-1]['error'] if excluded else ''}"
    if err is not None:
        print(json.dumps({"metric": METRIC, "value": None, "error": err[-2000:],
                          **({"excluded_steps": excluded} if excluded else {})}))
        return 1
    curve = None
    if args.curve_steps > 0 and d.world == 1:
        croot = Path(tempfile.mkdtemp(prefix="tk8s-curve-", dir=os.environ.get("TMPDIR", "/tmp")))
        try:
            with open(args.log, "a") if args.log else open(os.devnull, "w") as clog:
                curve = config2_curve(croot, args, env, clog, args.curve_steps)
        except Exception as e:  # noqa: BLE001 - the headline stands; the curve says why it is missing
            curve = {"error": str(e)[-1500:]}
        finally:
            shutil.rmtree(croot, ignore_errors=True)
    plain = fabric = None
    fabric_steps = args.fabric_steps if args.fabric_steps is not None else (0 if fake else 5)
    off = "off" if fabric_disabled is not None else None
    if d.world == 1 and (args.plain_steps > 0 or fabric_steps > 0):
        xroot = Path(tempfile.mkdtemp(prefix="tk8s-extra-", dir=os.environ.get("TMPDIR", "/tmp")))
        with open(args.log, "a") if args.log else open(os.devnull, "w") as xlog:
            if args.plain_steps > 0:
                try:
                    plain = series(xroot, "plain", n, args, env, xlog, args.plain_steps, settle=settle,
                                   rccl=off, env_over={"TK8S_SHORTCUTS": "0"})
                except Exception as e:  # noqa: BLE001 - the headline stands; the key says why it is missing
                    plain = {"error": str(e)[-1500:]}
            if fabric_steps > 0 and fabric_disabled is not None:
                fabric = {"skipped": f"the fabric check failed after step {fabric_disabled['after_step']}",
                          "error_tail": fabric_disabled["error_tail"]}
            elif fabric_steps > 0:
                try:
                    fabric = series(xroot, "fabric", n, args, env, xlog, fabric_steps, settle=settle, rccl="on")
                    # one more, untimed, with RCCL's INIT/P2P log on: the rank's transport record
                    # (which channels it built) without logging inside the timed steps
                    logged = series(xroot, "fabric-logged", n, args, env, xlog, 1, warmup=0, settle=settle, rccl="on",
                                    env_over={"NCCL_DEBUG": "INFO", "NCCL_DEBUG_SUBSYS": "INIT,P2P"})
                    fabric["transport_logged_run"] = (logged["last"].get("rccl") or {}).get("transport")
                except Exception as e:  # noqa: BLE001
                    fabric = {"error": str(e)[-1500:]}
        shutil.rmtree(xroot, ignore_errors=True)
    step_mean = sum(times) / len(times)
    mean = sum(ready_times) / len(ready_times)
    ready = [s["ready_seconds"] for s in summaries if s.get("ready_seconds") is not None]
    phases: dict[str, float] = {}
    for s in summaries:
        for k, v in s.get("phases", {}).items():
            phases[k] = phases.get(k, 0.0) + v / len(summaries)
    last = summaries[-1] if summaries else {}
    hip_init = []
    for s in summaries:
        v = [float(a["hip-init-ms"]) for a in (s.get("validation") or {}).values() if a.get("hip-init-ms")]
        hip_init.append(max(v) if v else None)
    out = {
        "metric": METRIC,
        "value": round(mean, 4),
        "unit": "s",
        "n_gpus": n,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(step_mean * 1000.0, 2),
        "higher_is_better": False,
        "scaling": "weak",
        "vs_baseline": round(mean / BASELINE_FLOOR_S, 5),
        "baseline": {"value": BASELINE_FLOOR_S, "what": "reference bring-up fixed-sleep floor (BASELINE.md); "
                     "the reference publishes no bring-up time"},
        "vs_baseline_note": "vs the reference's fixed-sleep floor (51 s of sleeps in its cloud-VM path), NOT "
                            "like-for-like: this bring-up creates no VM, pulls no image and starts no container "
                            "(local sandboxes on the GPU host)",
        "dtype": "fp32",
        "data": "synthetic" + (" (fake GPUs: CPU rehearsal, not a GPU measurement)" if fake else ""),
        "config": {"model": f"1 master + {n} workers x {args.package}", "global_batch": n, "seq_len": 0,
                   "parallelism": f"workers{n}", "validate": not args.no_validate,
                   "rccl": (args.rccl or ("on" if n >= 2 else "off"))},
        "value_definition": "wall-clock from launching ./setup.sh to its 'ALL NODES READY' line (every worker "
                            "heartbeating, GPU-validated, amd.com/gpu allocatable); mean over the timed steps",
        "step_definition": "whole ./setup.sh process (also runs the RCCL fabric check when n_gpus >= 2), "
                           "barrier + device sync on every rank on both sides, MAX over ranks",
        # what persists between steps (all of it per-user and content-checked; every step still
        # creates its machines, starts every process and runs every GPU validation kernel)
        "host_caches": "Python byte code (build/pycache), parsed YAML of the unchanged playbook/role/"
                       "manifest files and rewritten Jinja expressions (~/.local/state/tk8s; entries carry "
                       "their source text); filled by the warmup steps",
        "min_s": round(min(ready_times), 4),
        "max_s": round(max(ready_times), 4),
        "median_s": round(sorted(ready_times)[len(ready_times) // 2] if len(ready_times) % 2
                          else sum(sorted(ready_times)[len(ready_times) // 2 - 1:len(ready_times) // 2 + 1]) / 2, 4),
        "setup_process_s": round(step_mean, 4),
        # from the Ready line to ./setup.sh's exit (the RCCL fabric check, the summary): with
        # value, what ms_per_step is made of
        "post_ready_s": round(sum(s.get("post_ready_seconds", 0.0) for s in summaries) / len(summaries), 4)
        if summaries else None,
        "cold_first_run_s": round(cold["ready_wall_seconds"], 4) if cold else None,
        "cold_first_run_what": "step 0 (a warmup step) with empty byte-code and parse caches: a first "
                               "./setup.sh on a fresh install" if cold else None,
        # where the cold first run's time went, and what it started from
        "cold_first_run_phases_s": {k: round(v, 4) for k, v in (cold.get("phases") or {}).items()} if cold else None,
        "cold_first_run_burnin": {k: v for k, v in (
            ("runtime_init_ms", (cold.get("host_burnin") or {}).get("runtime_init_ms")),
            ("total_ms", (cold.get("host_burnin") or {}).get("total_ms")),
            ("spawn_ms", cold.get("burnin_spawn_ms")), ("exec_ms", cold.get("burnin_exec_ms")),
            ("notice_ms", cold.get("burnin_notice_ms")))} if cold else None,
        "cold_first_run_kfd_census": cold.get("kfd_census") if cold else None,
        "cold_first_run_slowest_tasks": cold.get("slowest_tasks") if cold else None,
        "cold_first_run_slow_start_cause": cold.get("slow_start_cause") if cold else None,
        "cold_first_run_start_state": cold_start_state or None,
        "rccl_check_s": round(sum(s.get("phases", {}).get("rccl", 0.0) for s in summaries) / len(summaries), 4)
        if summaries else None,
        "ready_s_inside_setup": round(sum(ready) / len(ready), 4) if ready else None,
        "teardown_s": round(sum(teardown_s) / len(teardown_s), 4) if teardown_s else None,
        "phases_s": {k: round(v, 4) for k, v in phases.items()},
        "gpus_allocatable": last.get("gpus_allocatable"),
        "nodes_validated": last.get("nodes_validated"),
        "rccl_peak_busbw_gbps": (last.get("rccl") or {}).get("peak_busbw_gbps"),
        # the fabric check of the last step, for the multi-GPU runs: communicator start-up, how
        # unevenly the ranks came up, the channel transports RCCL logged, the Job's shape
        "rccl_last_step": {k: (last.get("rccl") or {}).get(k) for k in (
            "ok", "nranks", "pods", "gpus_per_pod", "comm_init_ms_max", "sweep_ms_max", "init_spread_ms", "transport",
            "rccl_library", "peak_algbw_gbps", "fabric", "sweep", "op_timeout_s")}
        if last.get("rccl") else None,
        "xgmi_last_step": last.get("xgmi"),
        "validation_last_step": last.get("validation"),
        "hip_init_ms_steps": hip_init,
        "settle_s": settle,
        "burnin_runtime_init_ms_steps": [(s.get("host_burnin") or {}).get("runtime_init_ms") for s in summaries],
        "burnin_runtime_steps": [(s.get("host_burnin") or {}).get("runtime") for s in summaries],
        "burnin_device_wall_ms_max_steps": [max((s.get("host_burnin") or {}).get("device_wall_ms") or [0.0]) or None
                                            for s in summaries],
        "burnin_peers_ms_steps": [(s.get("host_burnin") or {}).get("peers_ms") for s in summaries],
        # how long before Ready the burn-in's result was seen: near 0, the GPU burn-in (not the
        # control-plane / agent chain) set the step's Ready time
        "burnin_result_before_ready_ms_steps": [
            round((s["launched_unix"] + s["ready_wall_seconds"] - s["host_burnin"]["seen_unix"]) * 1e3, 1)
            if (s.get("host_burnin") or {}).get("seen_unix") and s.get("launched_unix") and s.get("ready_wall_seconds")
            else None for s in summaries],
        "burnin_total_ms_steps": [(s.get("host_burnin") or {}).get("total_ms") for s in summaries],
        "burnin_spawn_ms_steps": [s.get("burnin_spawn_ms") for s in summaries],
        "burnin_exec_ms_steps": [s.get("burnin_exec_ms") for s in summaries],
        "burnin_notice_ms_steps": [s.get("burnin_notice_ms") for s in summaries],
        # every timed step whose runtime start took > 50 ms, with what the KFD process census saw
        "slow_start_cause": {str(args.warmup + i): s["slow_start_cause"] for i, s in enumerate(summaries)
                             if s.get("slow_start_cause")},
        "kfd_census_available": any((s.get("kfd_census") or {}).get("available") for s in summaries),
    }
    if b2b_ready:
        out["back_to_back"] = {"steps": len(b2b_ready), "mean_s": round(sum(b2b_ready) / len(b2b_ready), 4),
                               "max_s": round(max(b2b_ready), 4), "per_step": b2b_detail,
                               "what": "./setup.sh -c && ./setup.sh with no settle pause: Ready includes the driver "
                                       "still releasing the previous bring-up's GPU processes"}
    if fabric_disabled is not None:  # the steps after it ran with --rccl off
        out["fabric_disabled_after_step"] = fabric_disabled["after_step"]
        out["fabric_disabled"] = fabric_disabled
        out["config"]["rccl"] = f"on until step {fabric_disabled['after_step']}, then off (fabric check failed)"
    if excluded:  # timed steps left out of value: Ready, then the post-Ready RCCL check failed
        out["post_ready_errors"] = {"count": len(excluded), "excluded_steps": [x["step"] for x in excluded],
                                    "last": excluded[-1]["error"]}
    if curve is not None:
        out["curve_config2"] = curve
    if plain is not None:  # the bring-up with every start-up shortcut off
        out["plain_path_s"] = plain.get("ready", {}).get("mean_s")
        out["plain_path"] = {k: v for k, v in plain.items() if k != "last"}
        out["plain_path"]["what"] = ("TK8S_SHORTCUTS=0: every start-up shortcut of docs/architecture.md off "
                                     "(early burn-in, zygotes, caches, fast parsers, -S, inline tasks, ...)")
    if fabric is not None and "skipped" in fabric:
        out["fabric_validated_s"] = None
        out["fabric_validated"] = fabric
    elif fabric is not None:  # launch -> a passing RCCL all-reduce Job, N GPUs
        last_rccl = (fabric.get("last") or {}).get("rccl") or {}
        out["fabric_validated_s"] = fabric.get("setup_exit", {}).get("mean_s")
        out["fabric_validated"] = {k: v for k, v in fabric.items() if k != "last"}
        out["fabric_validated"].update({
            "what": "--rccl on: wall-clock from launching ./setup.sh to its exit after the RCCL all-reduce Job "
                    "over every GPU passed its exact check",
            "rccl": {k: last_rccl.get(k) for k in ("ok", "nranks", "pods", "comm_init_ms_max", "sweep_ms_max", "init_spread_ms", "rccl_library",
                                                   "peak_busbw_gbps", "peak_algbw_gbps", "fabric", "sweep",
                                                   "op_timeout_s", "transport")}})
    print(json.dumps(out), flush=True)
    return 0


def _has_kfd_gpus() -> bool:
    try:
        from tritonk8ssupervisor_amd.models.hostinfo import discover

        return discover().count > 0
    except Exception:  # noqa: BLE001
        return False


if __name__ == "__main__":
    sys.exit(main())
