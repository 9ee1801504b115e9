"""Race-free filesystem helpers.

The reference appends machine IPs from concurrent Terraform provisioners with ``>>``
(terraform/master/main.tf:29-31), so ``masters.ip``/``hosts.ip`` order is nondeterministic
(SURVEY.md §5.2). Everything here is atomic (tmp + rename) or serialised by an flock.
"""
from __future__ import annotations

import contextlib
import fcntl
import json
import os
from pathlib import Path


def _mkstemp(p: Path) -> tuple[int, str]:
    """tempfile.mkstemp's contract (a new 0600 file, exclusive create) without importing
    tempfile (random, bisect, weakref ...) on the bring-up path."""
    while True:
        tmp = str(p.parent / f".{p.name}.{os.urandom(6).hex()}.tmp")
        try:
            return os.open(tmp, os.O_WRONLY | os.O_CREAT | os.O_EXCL | os.O_CLOEXEC, 0o600), tmp
        except FileExistsError:
            continue


def atomic_write(path: str | os.PathLike, data: str | bytes, mode: int | None = None, durable: bool = False) -> None:
    """Write ``data`` to ``path`` atomically (readers see the old or the new file, never half).

    ``durable`` adds an fsync before the rename (survives power loss, ~2 ms per file). Bring-up
    state does not need it: a crashed run is cleaned or resumed, and the rename alone already
    guarantees that no reader ever sees a torn file."""
    p = Path(path)
    p.parent.mkdir(parents=True, exist_ok=True)
    fd, tmp = _mkstemp(p)
    try:
        with os.fdopen(fd, "wb") as f:
            f.write(data.encode() if isinstance(data, str) else data)
            if durable:
                f.flush()
                os.fsync(f.fileno())
        if mode is not None:
            os.chmod(tmp, mode)
        os.replace(tmp, p)
    except BaseException:
        with contextlib.suppress(FileNotFoundError):
            os.unlink(tmp)
        raise


def atomic_write_json(path: str | os.PathLike, obj: Any) -> None:
    atomic_write(path, json.dumps(obj, indent=2, sort_keys=True) + "\n")


def read_json(path: str | os.PathLike, default: Any = None) -> Any:
    try:
        with open(path, "rb") as f:
            return json.loads(f.read() or b"null")
    except FileNotFoundError:
        return default


@contextlib.contextmanager
def file_lock(path: str | os.PathLike) -> Iterator[None]:
    """Exclusive advisory lock on ``path`` (created if missing)."""
    p = Path(path)
    p.parent.mkdir(parents=True, exist_ok=True)
    with open(p, "a+") as f:
        fcntl.flock(f.fileno(), fcntl.LOCK_EX)
        try:
            yield
        finally:
            fcntl.flock(f.fileno(), fcntl.LOCK_UN)


def locked_append_line(path: str | os.PathLike, line: str) -> None:
    """Append one line under a lock (the safe form of ``echo ip >> hosts.ip``)."""
    p = Path(path)
    with file_lock(str(p) + ".lock"):
        with open(p, "a") as f:
            f.write(line.rstrip("\n") + "\n")
            f.flush()


def remove_paths(paths: list[str | os.PathLike]) -> list[str]:
    """rm -rf each path; returns the ones that existed."""
    removed = []
    for p in paths:
        p = Path(p)
        if p.is_symlink() or p.is_file():
            p.unlink()
            removed.append(str(p))
        elif p.is_dir():
            import shutil  # only for directories: not on the bring-up path

            shutil.rmtree(p, ignore_errors=True)
            removed.append(str(p))
    return removed
