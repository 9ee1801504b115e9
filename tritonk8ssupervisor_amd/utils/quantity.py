"""Kubernetes resource quantities (``500m``, ``2``, ``1.5Gi``, ``100M``, ``1e3``) and the forms the
metrics API prints (``cpu: 250m`` / ``123456n``, ``memory: 1024Ki``)."""
from __future__ import annotations

import re

_SUFFIX = {"n": 1e-9, "u": 1e-6, "m": 1e-3, "": 1.0, "k": 1e3, "M": 1e6, "G": 1e9, "T": 1e12, "P": 1e15, "E": 1e18,
           "Ki": 2.0 ** 10, "Mi": 2.0 ** 20, "Gi": 2.0 ** 30, "Ti": 2.0 ** 40, "Pi": 2.0 ** 50, "Ei": 2.0 ** 60}
_Q = re.compile(r"^([+-]?(?:\d+\.?\d*|\.\d+)(?:[eE][+-]?\d+)?)(n|u|m|k|M|G|T|P|E|Ki|Mi|Gi|Ti|Pi|Ei)?$")


def parse(q) -> float:
    """A quantity as a plain number (cores for CPU, bytes for memory)."""
    if isinstance(q, (int, float)):
        return float(q)
    m = _Q.match(str(q).strip())
    if not m:
        raise ValueError(f"not a quantity: {q!r}")
    return float(m.group(1)) * _SUFFIX[m.group(2) or ""]


def cpu(cores: float) -> str:
    """Cores as the metrics API writes them: nanocores."""
    return f"{max(0, int(round(cores * 1e9)))}n"


def memory(nbytes: float) -> str:
    return f"{max(0, int(nbytes) // 1024)}Ki"
