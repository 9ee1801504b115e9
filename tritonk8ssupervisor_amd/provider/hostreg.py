"""Host-wide claims on the local provider's loopback IPs and GPUs.

A cloud never hands two VMs the same address, nor two tenants the same device. On one MI355X
host the local provider plays that cloud for every cluster the host runs, so each workspace's
own ``alloc.json`` is not enough: two clusters brought up side by side (two users, or parallel
test workers) would both take 127.0.1.1 for their master -- and with it the same DNS, ingress
and NodePort sockets -- and both claim GPU 0. This registry is the host's view: one JSON file
under a per-user directory (``$TK8S_HOST_REGISTRY``, default ``${TMPDIR:-/tmp}/tk8s-host-<uid>``),
guarded by an flock and always taken *inside* the workspace lock (workspace, then host: no
lock-order inversion).

A claim records who holds it (workspace ``alloc.json``, machine name, creating pid). It is
reaped when its owner no longer lists the machine (torn down, or the workspace deleted), or when
the creating process is gone and no process of the machine's sandbox is alive (a bring-up that
crashed and was never torn down), so a dead cluster never strands an address or a GPU.
"""
from __future__ import annotations

import contextlib
import os
from pathlib import Path

from ..utils.fsutil import atomic_write_json, file_lock, read_json
from ..utils.procs import pid_alive, read_pidfile


def registry_dir() -> Path:
    from ..earlyburn import registry_dir as path  # one definition: the early burn-in reads it too

    return Path(path())


def _sandbox_alive(sandbox: Path) -> bool:
    for pattern in ("run/*.pid", "pods/*/*.pid"):
        for pidfile in sandbox.glob(pattern):
            info = read_pidfile(pidfile)
            pid = info.get("pid") if isinstance(info, dict) else info
            with contextlib.suppress(TypeError, ValueError):
                if pid_alive(int(pid or 0)):
                    return True
    return False


def _stale(claim: dict, owners: dict | None = None) -> bool:
    """``owners``: allocation tables already read during this reap (one read per workspace, not
    one per claimed machine)."""
    alloc_file = Path(claim.get("alloc", ""))
    machine = claim.get("machine", "")
    if owners is None or str(alloc_file) not in owners:
        owner = read_json(alloc_file, {}) or {}
        if owners is not None:
            owners[str(alloc_file)] = owner
    else:
        owner = owners[str(alloc_file)]
    if machine not in owner.get("machines", {}):
        return True
    if pid_alive(int(claim.get("pid") or 0)):
        return False
    return not _sandbox_alive(alloc_file.parent / "machines" / machine)


class HostRegistry:
    def __init__(self, path: str | os.PathLike | None = None):
        self.dir = Path(path) if path else registry_dir()
        self.file = self.dir / "claims.json"
        self.lock_file = self.dir / "claims.lock"

    @contextlib.contextmanager
    def locked(self) -> Iterator[dict]:
        """The claim table under the host lock, reaped of dead owners; written back on exit."""
        self.dir.mkdir(parents=True, exist_ok=True, mode=0o700)
        with file_lock(self.lock_file):
            table = read_json(self.file, {}) or {}
            before = repr(table)
            tables: dict[str, dict] = {}
            for kind in ("ips", "gpus"):
                claims = table.setdefault(kind, {})
                owners: dict[tuple, bool] = {}
                for key in list(claims):
                    c = claims[key]
                    k = (c.get("alloc"), c.get("machine"), c.get("pid"))
                    if k not in owners:
                        owners[k] = _stale(c, tables)
                    if owners[k]:
                        del claims[key]
            yield table
            if repr(table) != before or not self.file.exists():
                atomic_write_json(self.file, table)

    @staticmethod
    def claim(table: dict, kind: str, key: str, alloc_file: Path, machine: str) -> None:
        table.setdefault(kind, {})[str(key)] = {"alloc": str(alloc_file), "machine": machine, "pid": os.getpid()}

    @staticmethod
    def taken(table: dict, kind: str) -> set[str]:
        return set(table.get(kind, {}))

    @staticmethod
    def release(table: dict, alloc_file: Path, machine: str) -> None:
        for kind in ("ips", "gpus"):
            claims = table.get(kind, {})
            for key in [k for k, c in claims.items() if c.get("alloc") == str(alloc_file) and c.get("machine") == machine]:
                del claims[key]
