"""Port mapping for a cluster whose daemons may run without root.

Everything of a local cluster lives on this host's loopback addresses, so nothing but privilege
stops a pod or a Service from using its real port -- except that ports below 1024 need root (or
CAP_NET_BIND_SERVICE). When the cluster runs as an ordinary user (the GPU hosts here do), every
privileged port P is shifted to ``PRIV_PORT_BASE + P`` (80 -> 20080) on *both* sides: the Service
proxy and ingress listen there, the built-in apps (apps/) bind there, Service env vars advertise
it. ``TK8S_REMAP_PRIVILEGED_PORTS`` = ``auto`` (default: remap unless root) | ``1`` | ``0``.
"""
from __future__ import annotations

import os

PRIV_PORT_BASE = 20000


def remap_privileged() -> bool:
    v = os.environ.get("TK8S_REMAP_PRIVILEGED_PORTS", "auto").strip().lower()
    if v in ("1", "true", "yes", "on"):
        return True
    if v in ("0", "false", "no", "off"):
        return False
    return os.geteuid() != 0


def host_port(port: int) -> int:
    """The port a cluster process actually binds for the cluster-visible ``port``."""
    port = int(port)
    return PRIV_PORT_BASE + port if 0 < port < 1024 and remap_privileged() else port
