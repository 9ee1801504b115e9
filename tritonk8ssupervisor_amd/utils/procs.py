"""Daemon process management (the local analogue of `docker run -d --restart=unless-stopped`).

Daemons run in their own session/process group so teardown can signal the whole tree, and
their pid/pgid is recorded in a pidfile under the owning machine's sandbox. Nothing here ever
uses ``os.exec*`` in-process: every program starts as a child (the GPU-box rule that processes
which initialised the GPU must not exec; spawners here never touch the GPU anyway).
"""
from __future__ import annotations

import contextlib
import errno
import json
import os
import signal
import subprocess
import time
from pathlib import Path


def plain_argv(argv: list[str], env: dict | None = None) -> list[str]:
    """``argv`` without the ``-S`` after a Python interpreter when the site-skipping shortcut is
    off (``TK8S_SHORTCUTS=0`` / ``TK8S_SKIP_SITE=0``, in ``env`` or this process's environment)."""
    e = env if env is not None else os.environ
    if e.get("TK8S_SKIP_SITE", "1") != "0" and e.get("TK8S_SHORTCUTS", "1") != "0":
        return argv
    out = []
    for i, a in enumerate(argv):
        if a == "-S" and i > 0 and os.path.basename(argv[i - 1]).startswith("python"):
            continue
        out.append(a)
    return out


def spawn_daemon(argv: list[str], *, env: dict | None = None, cwd: str | None = None,
                 log_path: str | None = None, pidfile: str | None = None) -> subprocess.Popen:
    argv = plain_argv(argv, env)
    log = open(log_path, "ab", buffering=0) if log_path else subprocess.DEVNULL
    try:
        p = subprocess.Popen(argv, env=env, cwd=cwd, stdin=subprocess.DEVNULL, stdout=log,
                             stderr=subprocess.STDOUT, start_new_session=True, close_fds=True)
    finally:
        if log_path:
            log.close()
    if pidfile:
        Path(pidfile).parent.mkdir(parents=True, exist_ok=True)
        from .fsutil import atomic_write_json

        atomic_write_json(pidfile, {"pid": p.pid, "pgid": p.pid, "argv": argv, "started": time.time(),
                                    "start": proc_start_ticks(p.pid)})
    return p


def proc_start_ticks(pid: int) -> int | None:
    """When the process started (``/proc/<pid>/stat`` field 22, clock ticks since boot): with the
    pid, an identity that a reused pid does not share. None if there is no such process."""
    try:
        with open(f"/proc/{int(pid)}/stat") as f:
            return int(f.read().rsplit(")", 1)[1].split()[19])
    except (OSError, ValueError, IndexError):
        return None


def pidfile_owner_alive(info: dict) -> bool:
    """Is the process a pidfile names still the one that wrote it? Its recorded start time must
    match; a pidfile without one (written by an older tk8s) must name a tk8s process. A pidfile
    that outlived a reboot or a failed run must never get an unrelated process group signalled
    (ADVICE r2)."""
    pid = int(info.get("pid") or 0)
    now = proc_start_ticks(pid) if pid > 0 else None
    if now is None:
        return False
    if info.get("start") is not None:
        return int(info["start"]) == now
    try:
        with open(f"/proc/{pid}/cmdline", "rb") as f:
            cmd = f.read().replace(b"\0", b" ")
    except OSError:
        return False
    return any(k in cmd for k in (b"tk8s", b"tritonk8ssupervisor"))


def pid_alive(pid: int) -> bool:
    if pid <= 0:
        return False
    try:
        os.kill(pid, 0)
    except OSError as e:
        return e.errno == errno.EPERM
    # a zombie child of ours still "exists"; reap if possible
    with contextlib.suppress(ChildProcessError, OSError):
        r, _ = os.waitpid(pid, os.WNOHANG)
        if r == pid:
            return False
    try:
        with open(f"/proc/{pid}/stat") as f:
            return f.read().split(")")[-1].split()[0] != "Z"
    except OSError:
        return True


def read_pidfile(pidfile: str | os.PathLike) -> dict | None:
    try:
        return json.loads(Path(pidfile).read_text())
    except (OSError, ValueError):
        return None


def group_alive(pgid: int) -> bool:
    """True while the process group has a member that is not a zombie. A daemon reparented to
    an init that reaps lazily lingers as a zombie, which `killpg(pgid, 0)` still counts."""
    try:
        os.killpg(pgid, 0)
    except ProcessLookupError:
        return False
    except PermissionError:
        return True
    try:
        pids = [d for d in os.listdir("/proc") if d.isdigit()]
    except OSError:
        return True
    for d in pids:
        try:
            with open(f"/proc/{d}/stat", "rb") as f:
                rest = f.read().rsplit(b")", 1)[1].split()
        except (OSError, IndexError):
            continue
        if len(rest) > 2 and int(rest[2]) == pgid and rest[0] != b"Z":
            return True
    return False


def kill_group(pgid: int, grace: float = 3.0, term: bool = True) -> bool:
    """SIGTERM the process group (unless ``term`` is False: the caller already did), wait up to
    `grace` s, then SIGKILL. True if it was alive."""
    try:
        os.killpg(pgid, signal.SIGTERM if term else 0)
    except ProcessLookupError:
        return False
    except PermissionError:
        return False
    deadline = time.monotonic() + grace
    delay = 0.001
    while time.monotonic() < deadline:
        with contextlib.suppress(ChildProcessError, OSError):
            os.waitpid(-pgid, os.WNOHANG)
        if not group_alive(pgid):
            return True
        time.sleep(delay)
        delay = min(delay * 2, 0.02)
    with contextlib.suppress(ProcessLookupError, PermissionError):
        os.killpg(pgid, signal.SIGKILL)
    # until the kernel has torn it down (its sockets and addresses are free for the next owner)
    deadline = time.monotonic() + 2.0
    while time.monotonic() < deadline and group_alive(pgid):
        with contextlib.suppress(ChildProcessError, OSError):
            os.waitpid(-pgid, os.WNOHANG)
        time.sleep(0.005)
    return True


def kill_pidfile(pidfile: str | os.PathLike, grace: float = 3.0) -> bool:
    """Stop the process group a pidfile names -- only if its process is still the one that wrote
    the pidfile (pidfile_owner_alive); a stale pidfile is just removed."""
    info = read_pidfile(pidfile)
    if isinstance(info, int):  # a bare pid (the burn-in's)
        info = {"pid": info}
    if not isinstance(info, dict) or not info.get("pid"):
        return False
    if not pidfile_owner_alive(info):
        with contextlib.suppress(FileNotFoundError):
            Path(pidfile).unlink()
        return False
    alive = kill_group(int(info.get("pgid") or info["pid"]), grace)
    with contextlib.suppress(FileNotFoundError):
        Path(pidfile).unlink()
    return alive


def wait_for_file_text(path: str | os.PathLike, needle: str, timeout: float, interval: float = 0.01) -> bool:
    """Poll a log file until it contains `needle` (the `docker logs | grep "Listening on"` wait)."""
    deadline = time.monotonic() + timeout
    while time.monotonic() < deadline:
        with contextlib.suppress(OSError):
            if needle in Path(path).read_text(errors="replace"):
                return True
        time.sleep(interval)
    return False
