"""Environment-driven fault injection (the reference has none).

``TK8S_FAULTS`` is a comma list of ``point[@target][:arg]`` entries, e.g.::

    TK8S_FAULTS="provision.create@kubenode2,agent.crash@kubenode1:1,cp.dashboard_delay:2.0"

Points consult :func:`fault` with their target (machine / node name); ``arg`` is returned
(``True`` when absent). A ``:N`` count on ``agent.crash`` style points is interpreted by the
caller (e.g. crash only the first N times, tracked via a file so restarts see it).
"""
from __future__ import annotations

import os


def _parse(spec: str) -> list[tuple[str, str | None, str | None]]:
    out = []
    for item in filter(None, (s.strip() for s in spec.split(","))):
        arg = None
        if ":" in item:
            item, arg = item.split(":", 1)
        target = None
        if "@" in item:
            item, target = item.split("@", 1)
        out.append((item, target, arg))
    return out


def fault(point: str, target: str | None = None) -> str | bool | None:
    """Returns the fault's argument (or True) if ``point`` is armed for ``target``, else None."""
    spec = os.environ.get("TK8S_FAULTS", "")
    if not spec:
        return None
    for p, t, arg in _parse(spec):
        if p == point and (t is None or t == target):
            return arg if arg is not None else True
    return None


class InjectedFault(RuntimeError):
    pass


def maybe_fail(point: str, target: str | None = None) -> None:
    if fault(point, target) is not None:
        raise InjectedFault(f"injected fault {point}@{target}")
