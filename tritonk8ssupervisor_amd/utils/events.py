"""JSONL event log with monotonic per-phase timestamps.

The reference never measures its own bring-up (no timers); phases here are
timed so the BASELINE metric (``./setup.sh`` -> all nodes Ready) falls out of the log.
"""
from __future__ import annotations

import contextlib
import json
import os
import threading
import time
from pathlib import Path

_lock = threading.Lock()


class EventLog:
    """One JSON line per event, appended through a descriptor opened once with O_APPEND: one
    ``write`` per event, atomic against the other threads and processes appending to the same
    file, and no open/close per event (which, behind one lock, cost the nine creation threads of
    an 8-worker bring-up a third of their time). A log whose file was removed under it (a
    workspace cleaned and made again) opens the new one."""

    def __init__(self, path: str | os.PathLike | None, echo: bool = False):
        self.path = Path(path) if path else None
        self.echo = echo
        self.t0 = time.monotonic()
        self.phases: dict[str, float] = {}
        self._fd = -1
        if self.path:
            self.path.parent.mkdir(parents=True, exist_ok=True)

    def _descriptor(self) -> int:
        fd = self._fd
        if fd >= 0:
            try:
                if os.fstat(fd).st_nlink > 0:
                    return fd
            except OSError:
                pass
        with _lock:
            if self._fd == fd:  # not reopened by another thread meanwhile
                if fd >= 0:
                    with contextlib.suppress(OSError):
                        os.close(fd)
                self._fd = os.open(self.path, os.O_WRONLY | os.O_APPEND | os.O_CREAT | os.O_CLOEXEC, 0o644)
            return self._fd

    def emit(self, event: str, **fields: Any) -> dict:
        rec = {"ts": time.time(), "t": round(time.monotonic() - self.t0, 6), "event": event, **fields}
        if self.path:
            line = (json.dumps(rec, sort_keys=True, default=str) + "\n").encode()
            try:
                os.write(self._descriptor(), line)
            except FileNotFoundError:  # its directory went away (a clean): the event is dropped
                pass
        if self.echo:
            print(f"[{rec['t']:8.3f}s] {event} " + " ".join(f"{k}={v}" for k, v in fields.items()), flush=True)
        return rec

    @contextlib.contextmanager
    def phase(self, name: str, **fields: Any) -> Iterator[None]:
        t = time.monotonic()
        self.emit("phase_start", phase=name, **fields)
        ok = False
        try:
            yield
            ok = True
        finally:
            dt = time.monotonic() - t
            self.phases[name] = dt
            self.emit("phase_end", phase=name, seconds=round(dt, 6), ok=ok)


def read_events(path: str | os.PathLike) -> list[dict]:
    out = []
    with contextlib.suppress(FileNotFoundError):
        with open(path) as f:
            for line in f:
                line = line.strip()
                if line:
                    out.append(json.loads(line))
    return out
