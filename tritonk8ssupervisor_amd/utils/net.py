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
NODE_PORT_LOW = 30000  # Service NodePorts: 30000-32767 (controlplane/k8s_api.py)


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


def _ephemeral_low() -> int:
    try:
        with open("/proc/sys/net/ipv4/ip_local_port_range") as f:
            return int(f.read().split()[0])
    except (OSError, ValueError, IndexError):
        return 32768


def pick_port(host: str = "127.0.0.1", tries: int = 64) -> int:
    """A free TCP port for a daemon that binds it a moment later (the cluster's API port).

    Drawn between the remapped privileged ports and the NodePort range (30000-32767, which the
    Service proxy binds), and below the kernel's ephemeral range. ``bind(0)``
    returns a port from the ephemeral range, and every outgoing connection on the host draws its
    source port from the same range; between the pick and the daemon's bind another process can
    take it (EADDRINUSE, seen on the shared GPU box). Below the range only another explicit
    picker can. Falls back to ``bind(0)`` when no candidate binds."""
    import _socket  # (not ``socket``: its enum set-up is ~1.5 ms of the bring-up, utils/http1.py)

    lo, hi = PRIV_PORT_BASE + 1024, min(_ephemeral_low(), NODE_PORT_LOW) - 1
    for _ in range(tries if hi - lo >= 256 else 0):
        p = lo + int.from_bytes(os.urandom(4), "little") % (hi - lo + 1)
        s = _socket.socket(_socket.AF_INET, _socket.SOCK_STREAM)
        try:
            s.bind((host, p))
            return p
        except OSError:
            continue
        finally:
            s.close()
    s = _socket.socket(_socket.AF_INET, _socket.SOCK_STREAM)
    try:
        s.bind((host, 0))
        return s.getsockname()[1]
    finally:
        s.close()
