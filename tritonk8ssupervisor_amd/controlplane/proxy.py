"""Service proxy (the kube-proxy role) for the single-host local provider.

Every machine of a local cluster lives on this host, on its own loopback address, and every pod
gets its own loopback IP from its node's podCIDR (agent, ``POD_IP``). A Service therefore needs
one listener per exposed address, not one per node, so the control plane runs them on its own
event loop:

* ``ClusterIP``:    ``spec.clusterIP:port`` (allocated from 127.96.0.0/16)
* ``NodePort``:     additionally ``<master IP>:nodePort`` and ``127.0.0.1:nodePort`` (30000-32767)
* ``LoadBalancer``: additionally ``<master IP>:port``, published as
  ``status.loadBalancer.ingress[0].ip`` — the Guestbook walkthrough of the reference
  (docs/detailed.md:329-364) exposed its frontend exactly this way.

Connections go round-robin to the Service's endpoints: Running pods of the same
project/namespace whose labels match ``spec.selector``, at ``status.podIP:targetPort``; with
``sessionAffinity: ClientIP`` a client address keeps its endpoint for
``sessionAffinityConfig.clientIP.timeoutSeconds`` (10800) after its last connection.
"""
from __future__ import annotations

import asyncio
import itertools
import time
from typing import Callable


class ServiceProxy:
    def __init__(self, endpoints: Callable[[str, str], list[tuple[str, int]]], log: Callable[[str], None] = print,
                 affinity: Callable[[str], float] | None = None):
        self.endpoints = endpoints          # (service key, port name/number) -> [(ip, port)]
        self.log = log
        self.affinity = affinity            # service key -> ClientIP affinity timeout in s (0: none)
        self._sticky: dict[tuple[str, str, str], tuple[tuple[str, int], float]] = {}
        self.listeners: dict[tuple[str, str, int], asyncio.AbstractServer] = {}  # (svc key, host, port)
        self._rr: dict[tuple[str, str], itertools.count] = {}

    async def sync(self, wanted: dict[tuple[str, str, int], str]) -> None:
        """wanted: (service key, bind host, bind port) -> service port key. Opens/closes listeners."""
        for k in [k for k in self.listeners if k not in wanted]:
            srv = self.listeners.pop(k)
            srv.close()
            try:
                await srv.wait_closed()
            except Exception:  # noqa: BLE001 - closing is best effort
                pass
        for k, port_key in wanted.items():
            if k in self.listeners:
                continue
            svc, host, port = k
            try:
                self.listeners[k] = await asyncio.start_server(
                    lambda r, w, svc=svc, pk=port_key: self._conn(svc, pk, r, w), host, port, reuse_address=True)
            except OSError as e:
                self.log(f"service {svc}: cannot listen on {host}:{port}: {e}")

    async def close(self) -> None:
        await self.sync({})

    async def _conn(self, svc: str, port_key: str, reader: asyncio.StreamReader, writer: asyncio.StreamWriter) -> None:
        eps = self.endpoints(svc, port_key)
        if not eps:
            writer.close()
            return
        n = next(self._rr.setdefault((svc, port_key), itertools.count()))
        order = [eps[(n + i) % len(eps)] for i in range(len(eps))]
        ttl = self.affinity(svc) if self.affinity is not None else 0
        client = (writer.get_extra_info("peername") or ("?",))[0]
        if ttl:
            hit = self._sticky.get((svc, port_key, client))
            if hit and hit[1] > time.monotonic() and hit[0] in order:
                order.remove(hit[0])
                order.insert(0, hit[0])  # the client's endpoint, while it is still one
        up_r = up_w = None
        for host, port in order:  # round robin, skipping endpoints that refuse
            try:
                up_r, up_w = await asyncio.wait_for(asyncio.open_connection(host, port), 5.0)
                break
            except (OSError, asyncio.TimeoutError):
                continue
        if up_w is None:
            writer.close()
            return
        if ttl:
            self._sticky[(svc, port_key, client)] = ((host, port), time.monotonic() + ttl)
        await asyncio.gather(_pump(reader, up_w), _pump(up_r, writer), return_exceptions=True)
        for w in (writer, up_w):
            w.close()


async def _pump(src: asyncio.StreamReader, dst: asyncio.StreamWriter) -> None:
    try:
        while True:
            data = await src.read(1 << 16)
            if not data:
                break
            dst.write(data)
            await dst.drain()
    finally:
        try:
            if dst.can_write_eof():
                dst.write_eof()
            else:
                dst.close()
        except (OSError, RuntimeError):
            dst.close()
