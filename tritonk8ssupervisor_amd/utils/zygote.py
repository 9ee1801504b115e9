"""Zygote processes (earlyburn): an interpreter started early that waits for its arguments.

The control plane and node agent zygotes import everything while the bring-up provisions, then
wait here for the JSON their boot hook writes atomically once the machine exists.
"""
from __future__ import annotations

import json
import os
import signal
import time


def await_json(path: str, timeout: float | None = None, want: type = dict):
    """Wait for ``path`` to hold a JSON value of type ``want`` (written atomically by a boot
    hook); past the timeout, stop the supervisor (a zygote of a failed bring-up) and exit."""
    if timeout is None:
        timeout = float(os.environ.get("TK8S_ZYGOTE_TIMEOUT", "120"))
    deadline = time.monotonic() + timeout
    t_fast = time.monotonic() + 2.0
    while True:
        try:
            with open(path) as f:
                v = json.load(f)
            if isinstance(v, want):
                return v
        except (OSError, ValueError):
            pass
        if time.monotonic() > deadline:
            parent = os.getppid()
            try:
                with open(f"/proc/{parent}/comm") as f:
                    if f.read().strip() == "tk8s-supervise":
                        os.kill(parent, signal.SIGTERM)
            except OSError:
                pass
            raise SystemExit(0)
        # 1 ms while a bring-up is on its way (the arguments normally arrive within ~0.1 s, on the
        # critical path), 50 ms once it is clearly not coming (a failed bring-up's leftover)
        time.sleep(0.001 if time.monotonic() < t_fast else 0.05)
