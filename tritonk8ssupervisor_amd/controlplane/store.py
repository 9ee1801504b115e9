"""Versioned object store with watch (the etcd + apiserver core of the control plane).

Single-threaded (one asyncio loop owns it), so no locks: every mutation bumps a global
resourceVersion, is appended to a bounded history and wakes long-poll watchers. Persistence, as
etcd does it: every mutation goes to a write-ahead journal (one JSON line, written before the
request that caused it is answered), and a periodic snapshot compacts it; a control plane that
restarts -- SIGTERM or SIGKILL alike -- loads the snapshot and replays the journal, so no
acknowledged write is lost.
"""
from __future__ import annotations

import asyncio
import copy
import json as _json
import time
from collections import deque
from typing import Any, Callable, Iterable

from ..utils.fsutil import atomic_write_json, read_json
from ..utils.ids import uuid4

HISTORY = 50_000


def now_iso() -> str:
    return time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())


class Conflict(Exception):
    pass


class Store:
    def __init__(self):
        self.rv = 0
        self.objs: dict[str, dict[str, dict]] = {}
        self.history: deque[tuple[int, str, str, dict]] = deque(maxlen=HISTORY)
        self._waiters: list[asyncio.Future] = []
        self.listeners: list[Callable[[str, str, dict], None]] = []
        self.type_meta: dict[str, tuple[str, str]] = {}  # kind -> (apiVersion, Kind) stamped on put
        self.kind_rv: dict[str, int] = {}  # kind -> resourceVersion of its last write (caches key on it)
        self._journal = None                # open write-ahead journal (open_journal), None = in memory only
        self.meta: dict[str, int] = {}      # persisted with the objects: the server's name sequence ("seq")

    # ---- reads ------------------------------------------------------------------------
    def get(self, kind: str, key: str) -> dict | None:
        return self.objs.get(kind, {}).get(key)

    def list(self, kind: str, pred: Callable[[dict], bool] | None = None) -> list[dict]:
        items = self.objs.get(kind, {}).values()
        return [o for o in items if pred is None or pred(o)]

    def keys(self, kind: str) -> Iterable[str]:
        return list(self.objs.get(kind, {}).keys())

    def version(self, *kinds: str) -> tuple[int, ...]:
        """The last write to each of ``kinds``: an index over them is current while this is."""
        return tuple(self.kind_rv.get(k, 0) for k in kinds)

    # ---- writes -----------------------------------------------------------------------
    def _notify(self, kind: str, etype: str, obj: dict) -> None:
        self.history.append((self.rv, kind, etype, obj))
        for fn in list(self.listeners):
            fn(kind, etype, obj)
        waiters, self._waiters = self._waiters, []
        for f in waiters:
            if not f.done():
                f.set_result(None)

    async def wait_change(self, timeout: float) -> None:
        """Sleep until the next mutation (or timeout)."""
        if timeout <= 0:
            return
        f = asyncio.get_running_loop().create_future()
        self._waiters.append(f)
        try:
            await asyncio.wait_for(f, timeout)
        except asyncio.TimeoutError:
            pass

    def put(self, kind: str, key: str, obj: dict, expect_rv: str | None = None) -> dict:
        table = self.objs.setdefault(kind, {})
        old = table.get(key)
        if expect_rv is not None and old is not None and old["metadata"].get("resourceVersion") != expect_rv:
            raise Conflict(f"{kind}/{key}: resourceVersion {expect_rv} is stale")
        self.rv += 1
        tm = self.type_meta.get(kind)
        if tm is not None:
            obj.setdefault("apiVersion", tm[0])
            obj.setdefault("kind", tm[1])
        md = obj.setdefault("metadata", {})
        md["resourceVersion"] = str(self.rv)
        md.setdefault("uid", old["metadata"]["uid"] if old else uuid4())
        md.setdefault("creationTimestamp", old["metadata"].get("creationTimestamp") if old else now_iso())
        table[key] = obj
        self.kind_rv[kind] = self.rv
        self._log("put", kind, key, obj)
        self._notify(kind, "MODIFIED" if old else "ADDED", obj)
        return obj

    def patch(self, kind: str, key: str, fn: Callable[[dict], None]) -> dict | None:
        cur = self.get(kind, key)
        if cur is None:
            return None
        new = copy.deepcopy(cur)
        fn(new)
        return self.put(kind, key, new)

    def delete(self, kind: str, key: str) -> dict | None:
        table = self.objs.get(kind, {})
        old = table.pop(key, None)
        if old is not None:
            self.rv += 1
            old = copy.deepcopy(old)
            old["metadata"]["resourceVersion"] = str(self.rv)
            self.kind_rv[kind] = self.rv
            self._log("del", kind, key, None)
            self._notify(kind, "DELETED", old)
        return old

    # ---- watch ------------------------------------------------------------------------
    def events_since(self, since: int, kind: str | None, pred: Callable[[dict], bool] | None = None) -> list[dict]:
        out = []
        for rv, k, etype, obj in reversed(self.history):  # newest first; stop at `since`
            if rv <= since:
                break
            if (kind is None or k == kind) and (pred is None or pred(obj)):
                out.append({"type": etype, "kind": k, "object": obj, "resourceVersion": rv})
        out.reverse()
        return out

    async def wait_events(self, since: int, kind: str | None, timeout: float,
                          pred: Callable[[dict], bool] | None = None) -> list[dict]:
        deadline = time.monotonic() + timeout
        while True:
            ev = self.events_since(since, kind, pred)
            left = deadline - time.monotonic()
            if ev or left <= 0:
                return ev
            await self.wait_change(left)

    async def wait_until(self, cond: Callable[[], Any], timeout: float) -> Any:
        """Long-poll helper: re-evaluate `cond` after every mutation until truthy or timeout."""
        deadline = time.monotonic() + timeout
        while True:
            v = cond()
            left = deadline - time.monotonic()
            if v or left <= 0:
                return v
            await self.wait_change(min(left, 1.0))

    # ---- persistence ------------------------------------------------------------------
    def _log(self, op: str, kind: str, key: str, obj: dict | None) -> None:
        if self._journal is not None:
            self._journal.write(_json.dumps({"rv": self.rv, "op": op, "kind": kind, "key": key, "obj": obj,
                                             "seq": self.meta.get("seq", 0)}, separators=(",", ":")) + "\n")
            self._journal.flush()  # in the kernel before the write is acknowledged: a killed process loses nothing

    def open_journal(self, path) -> int:
        """Replay the journal at ``path`` onto what ``restore`` loaded (entries past the snapshot's
        resourceVersion; a torn last line is ignored), then keep appending to it. Returns the
        number of entries replayed."""
        import os

        n = 0
        good = 0  # the end of the last whole entry: appends go on from there, past a torn tail
        try:
            with open(path, "rb") as f:
                while True:
                    raw = f.readline()
                    if not raw:
                        break
                    try:
                        e = _json.loads(raw)
                    except ValueError:
                        break  # the tail a kill cut short
                    if not raw.endswith(b"\n"):
                        break  # (a whole object without its newline: cut short all the same)
                    good = f.tell()
                    if e["rv"] <= self.rv:
                        continue
                    table = self.objs.setdefault(e["kind"], {})
                    if e["op"] == "put":
                        table[e["key"]] = e["obj"]
                    else:
                        table.pop(e["key"], None)
                    self.rv = e["rv"]
                    self.kind_rv[e["kind"]] = self.rv
                    self.meta["seq"] = max(self.meta.get("seq", 0), int(e.get("seq") or 0))
                    n += 1
        except FileNotFoundError:
            pass
        if os.path.exists(path) and os.path.getsize(path) > good:
            os.truncate(path, good)  # or the next replay would stop at the torn line, before these
        self._journal = open(path, "a", buffering=1 << 16)
        os.chmod(path, 0o600)
        return n

    def snapshot(self, path) -> None:
        atomic_write_json(path, {"rv": self.rv, "objs": self.objs, "meta": self.meta})
        if self._journal is not None:  # compaction: the snapshot holds everything up to self.rv
            self._journal.truncate(0)
            self._journal.seek(0)

    def restore(self, path) -> bool:
        d = read_json(path)
        if not d:
            return False
        self.rv = int(d.get("rv", 0))
        self.objs = d.get("objs", {})
        self.meta = dict(d.get("meta") or {})
        self.kind_rv = {k: self.rv for k in self.objs}
        return True
