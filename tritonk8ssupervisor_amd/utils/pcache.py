"""A small persistent string -> marshal-able cache shared by the processes of this user
(``state_home()``, ``$XDG_STATE_HOME/tk8s``: the same root as utils/yamlio.py's parse cache;
``TK8S_YAML_CACHE=off`` disables both).

For derived data that is expensive to compute the first time in every process but identical
across bring-ups -- e.g. the templating engine's rewrite of a Jinja expression needs the stdlib
tokenizer, whose first use compiles a large regex (~4 ms on the MI355X host). The table is
loaded once per process (one marshal read); a miss computes, and the new entry is merged into
the file (read, update, atomic replace), so steady state never writes. Bounded: the table is
dropped when it outgrows ``limit`` entries.
"""
from __future__ import annotations

import marshal
import os
import threading


def state_home() -> str:
    """Where tk8s keeps what it reads back on the operator's next run -- parse and rewrite caches,
    the image store: ``$XDG_STATE_HOME/tk8s`` (default ``~/.local/state/tk8s``). Not under
    ``~/.cache``: pods may write there (their own caches), and a poisoned entry here would run as
    the operator; the home around it is read-only to pods (agent._jail_layers)."""
    base = os.environ.get("XDG_STATE_HOME") or os.path.join(os.path.expanduser("~"), ".local", "state")
    return os.path.join(base, "tk8s")


class PersistentCache:
    def __init__(self, name: str, limit: int = 20000):
        self.name, self.limit = name, limit
        self._table: dict | None = None
        self._lock = threading.Lock()

    def _path(self) -> str | None:
        d = os.environ.get("TK8S_YAML_CACHE", "")
        if d == "off":
            return None
        if d:
            return os.path.join(d, f"{self.name}.marshal")
        return os.path.join(state_home(), f"{self.name}.marshal")

    def _load(self) -> dict:
        if self._table is None:
            table = {}
            path = self._path()
            if path:
                try:
                    with open(path, "rb") as f:
                        got = marshal.load(f)
                    if isinstance(got, dict):
                        table = got
                except (OSError, ValueError, EOFError, TypeError):
                    pass
            self._table = table
        return self._table

    def get(self, key: str):
        with self._lock:
            return self._load().get(key)

    def put(self, key: str, value) -> None:
        with self._lock:
            table = self._load()
            table[key] = value
            path = self._path()
            if not path:
                return
            try:
                blob = marshal.dumps(table if len(table) <= self.limit else {key: value})
            except ValueError:
                table.pop(key, None)
                return
            try:
                os.makedirs(os.path.dirname(path), exist_ok=True)
                tmp = f"{path}.{os.getpid()}.{threading.get_ident()}.tmp"
                with open(tmp, "wb") as f:
                    f.write(blob)
                os.replace(tmp, path)
            except OSError:
                pass
