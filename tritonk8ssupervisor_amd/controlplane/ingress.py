"""HTTP ingress controller (the ``ingress-controller`` / lb-service-rancher container of the
reference's Rancher Kubernetes stack, docs/img/infrastructure-containers.png).

``networking.k8s.io/v1`` Ingress objects route HTTP by host and path to Services. The control
plane runs one listener on the master address (port 80, shifted by utils.net.host_port when not
root) and, per request: match the rules (exact host beats the default, ``Exact`` beats
``Prefix``, longer paths beat shorter), pick a ready endpoint of the backend Service round-robin,
and forward the request with ``Connection: close`` (one request per upstream connection, so
keep-alive clients are re-routed on every request) plus ``X-Forwarded-*`` headers.
"""
from __future__ import annotations

import asyncio
import itertools
from typing import Callable
from urllib.parse import urlsplit

from .proxy import _pump

Route = tuple[str, str, str, str, str]  # (host or "", path, pathType, service key, service port key)


def match_route(routes: list[Route], host: str, path: str) -> tuple[str, str] | None:
    host = host.split(":", 1)[0].lower()
    best = None
    for r_host, r_path, ptype, svc, port_key in routes:
        if r_host and r_host.lower() != host:
            continue
        if ptype == "Exact":
            ok = path == r_path
        else:
            base = r_path.rstrip("/")
            ok = not base or path == base or path.startswith(base + "/")
        if ok:
            score = (1 if r_host else 0, 1 if ptype == "Exact" else 0, len(r_path))
            if best is None or score > best[0]:
                best = (score, svc, port_key)
    return (best[1], best[2]) if best else None


def _reply(writer: asyncio.StreamWriter, status: str, text: str) -> None:
    body = text.encode()
    writer.write(f"HTTP/1.1 {status}\r\nContent-Type: text/plain\r\nContent-Length: {len(body)}\r\n"
                 "Connection: close\r\n\r\n".encode() + body)


class IngressController:
    def __init__(self, routes: Callable[[], list[Route]], endpoints: Callable[[str, str], list[tuple[str, int]]],
                 log: Callable[[str], None] = print):
        self.routes = routes
        self.endpoints = endpoints
        self.log = log
        self.server: asyncio.AbstractServer | None = None
        self.address: tuple[str, int] | None = None
        self._rr = itertools.count()

    async def ensure(self, host: str, port: int, wanted: bool) -> None:
        """Listen while at least one Ingress exists; stop when the last one is deleted."""
        if wanted and self.server is None:
            try:
                self.server = await asyncio.start_server(self._conn, host, port, reuse_address=True)
                self.address = (host, port)
            except OSError as e:
                self.log(f"ingress: cannot listen on {host}:{port}: {e}")
        elif not wanted and self.server is not None:
            await self.close()

    async def close(self) -> None:
        if self.server is not None:
            self.server.close()
            try:
                await self.server.wait_closed()
            except Exception:  # noqa: BLE001 - closing is best effort
                pass
            self.server, self.address = None, None

    async def _conn(self, reader: asyncio.StreamReader, writer: asyncio.StreamWriter) -> None:
        try:
            head = await asyncio.wait_for(reader.readuntil(b"\r\n\r\n"), 30.0)
        except (asyncio.IncompleteReadError, asyncio.LimitOverrunError, asyncio.TimeoutError, ConnectionError):
            writer.close()
            return
        lines = head.decode("latin-1").split("\r\n")
        try:
            method, target, version = lines[0].split(" ", 2)
        except ValueError:
            _reply(writer, "400 Bad Request", "bad request line\n")
            writer.close()
            return
        headers = [ln for ln in lines[1:] if ln]
        host = next((ln.split(":", 1)[1].strip() for ln in headers if ln.lower().startswith("host:")), "")
        route = match_route(self.routes(), host, urlsplit(target).path or "/")
        if route is None:
            _reply(writer, "404 Not Found", "default backend - 404\n")
            writer.close()
            return
        eps = self.endpoints(*route)
        up_r = up_w = None
        n = next(self._rr)
        for i in range(len(eps)):
            ep_host, ep_port = eps[(n + i) % len(eps)]
            try:
                up_r, up_w = await asyncio.wait_for(asyncio.open_connection(ep_host, ep_port), 5.0)
                break
            except (OSError, asyncio.TimeoutError):
                continue
        if up_w is None:
            _reply(writer, "503 Service Unavailable", "no healthy upstream\n")
            writer.close()
            return
        peer = (writer.get_extra_info("peername") or ("", 0))[0]
        keep = [ln for ln in headers if ln.split(":", 1)[0].strip().lower() not in ("connection", "keep-alive")]
        out = [f"{method} {target} {version}", *keep, "Connection: close", f"X-Forwarded-For: {peer}",
               f"X-Forwarded-Host: {host}", "X-Forwarded-Proto: http"]
        up_w.write(("\r\n".join(out) + "\r\n\r\n").encode("latin-1"))
        await asyncio.gather(_pump(reader, up_w), _pump(up_r, writer), return_exceptions=True)
        for w in (writer, up_w):
            w.close()
