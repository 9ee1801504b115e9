"""Minimal asyncio HTTP/1.1 server (stdlib only; keep-alive; long-poll friendly).

Why not FastAPI/uvicorn: the control plane's start-up time is on the critical path of the
bring-up metric (the reference waits up to 300 s for Rancher to log "Listening on",
ansible/roles/ranchermaster/tasks/main.yml:14-20); importing this module costs milliseconds.
"""
from __future__ import annotations

import asyncio
import json
import re
import time
import traceback
from typing import Any, AsyncIterator, Awaitable, Callable
from urllib.parse import parse_qs, unquote, urlsplit

from ..utils.record import field, record as dataclass

REASONS = {101: "Switching Protocols", 200: "OK", 201: "Created", 202: "Accepted", 204: "No Content", 400: "Bad Request",
           401: "Unauthorized", 403: "Forbidden", 404: "Not Found", 405: "Method Not Allowed",
           409: "Conflict", 422: "Unprocessable Entity", 500: "Internal Server Error",
           503: "Service Unavailable", 504: "Gateway Timeout"}


@dataclass
class Request:
    method: str
    path: str
    query: dict[str, str]
    headers: dict[str, str]
    body: bytes
    peer: str = ""
    raw_query: str = ""

    def q_all(self, key: str) -> list[str]:
        """Every value of a repeated query parameter (``?command=ls&command=-l``)."""
        return parse_qs(self.raw_query, keep_blank_values=True).get(key, [])

    def json(self) -> Any:
        if not self.body:
            return {}
        try:
            return json.loads(self.body)
        except ValueError as e:
            raise HttpError(400, f"invalid JSON body: {e}") from e

    def q(self, key: str, default: str | None = None) -> str | None:
        return self.query.get(key, default)

    @property
    def bearer(self) -> str | None:
        a = self.headers.get("authorization", "")
        return a[7:].strip() if a.lower().startswith("bearer ") else None


@dataclass
class Response:
    status: int = 200
    body: Any = None
    headers: dict[str, str] = field(default_factory=dict)
    content_type: str | None = None

    def encode(self) -> tuple[bytes, str]:
        if isinstance(self.body, (bytes, bytearray)):
            return bytes(self.body), self.content_type or "application/octet-stream"
        if isinstance(self.body, str):
            return self.body.encode(), self.content_type or "text/plain; charset=utf-8"
        if self.body is None:
            return b"", self.content_type or "text/plain"
        return (json.dumps(self.body, separators=(",", ":"), default=str).encode(),
                self.content_type or "application/json")


@dataclass
class StreamResponse:
    """A chunked response whose body is produced over time (a Kubernetes watch stream)."""
    chunks: AsyncIterator[bytes]
    status: int = 200
    content_type: str = "application/json"
    headers: dict[str, str] = field(default_factory=dict)


@dataclass
class WebSocketResponse:
    """Switch the connection to a WebSocket (RFC 6455) and hand it to ``session(ws)``: what
    ``kubectl exec`` speaks since Kubernetes 1.29 (subprotocol v5.channel.k8s.io / v4.channel.k8s.io)."""
    session: Callable[["WebSocket"], Awaitable[None]]
    protocol: str = ""


class WebSocket:
    """Server side of an RFC 6455 connection: binary/text frames, client masking, ping/pong,
    close. Messages only (no fragments sent; incoming fragments are reassembled)."""

    def __init__(self, reader: asyncio.StreamReader, writer: asyncio.StreamWriter):
        self.reader, self.writer = reader, writer
        self.closed = False
        self._send_lock = asyncio.Lock()  # several tasks send (port-forward: one per port)

    async def send(self, data: bytes, opcode: int = 0x2) -> None:
        n = len(data)
        head = bytes([0x80 | opcode])
        if n < 126:
            head += bytes([n])
        elif n < 1 << 16:
            head += bytes([126]) + n.to_bytes(2, "big")
        else:
            head += bytes([127]) + n.to_bytes(8, "big")
        async with self._send_lock:
            self.writer.write(head + data)
            await self.writer.drain()

    async def recv(self) -> bytes | None:
        """The next message's payload; None once the client closed."""
        buf = b""
        while True:
            h = await self.reader.readexactly(2)
            fin, opcode = h[0] & 0x80, h[0] & 0x0F
            n = h[1] & 0x7F
            if n == 126:
                n = int.from_bytes(await self.reader.readexactly(2), "big")
            elif n == 127:
                n = int.from_bytes(await self.reader.readexactly(8), "big")
            if n > 64 << 20:
                raise HttpError(413, "websocket frame too large")
            mask = await self.reader.readexactly(4) if h[1] & 0x80 else b""
            data = await self.reader.readexactly(n)
            if mask and n:  # unmask as one big-integer XOR (port-forward moves MBs through here)
                m = (mask * (n // 4 + 1))[:n]
                data = (int.from_bytes(data, "little") ^ int.from_bytes(m, "little")).to_bytes(n, "little")
            if opcode == 0x8:
                self.closed = True
                return None
            if opcode == 0x9:
                await self.send(data, 0xA)
                continue
            if opcode == 0xA:
                continue
            buf += data
            if fin:
                return buf

    async def close(self, code: int = 1000) -> None:
        if not self.closed:
            self.closed = True
            try:
                await self.send(code.to_bytes(2, "big"), 0x8)
            except (ConnectionError, RuntimeError):
                pass


def websocket_accept(key: str) -> str:
    import base64
    import hashlib

    return base64.b64encode(hashlib.sha1((key + "258EAFA5-E914-47DA-95CA-C5AB0DC85B11").encode()).digest()).decode()


class HttpError(Exception):
    def __init__(self, status: int, message: str, body: Any = None):
        super().__init__(message)
        self.status = status
        self.message = message
        self.custom_body = body is not None
        self.body = body if body is not None else {"type": "error", "status": status, "message": message}


Handler = Callable[..., Awaitable[Response | Any]]


_PREFIX = re.compile(r"[^.^$*+?{}\[\]|()\\]*")


def _literal_prefix(pattern: str) -> str:
    """The literal text every match of ``pattern`` starts with: up to the first regex
    metacharacter, less a character a quantifier makes optional."""
    n = _PREFIX.match(pattern).end()
    if n and n < len(pattern) and pattern[n] in "*?{":
        n -= 1
    return pattern[:n]


_SEG = re.compile(r"/((?:\([^()]*\)|[^/()])*)")      # one path segment; a group may hold "/"
_LIT = re.compile(r"[A-Za-z0-9_.:\-]+")
_GROUP = re.compile(r"\(\?P<(\w+)>(.*)\)")
_CHOICE = re.compile(r"[A-Za-z0-9_\-]+(?:\|[A-Za-z0-9_\-]+)*")


def _segments(pattern: str):
    """A path pattern made of ``/``-separated literal segments (dots taken literally), named
    segments ``(?P<n>[^/]+)``, named choices ``(?P<n>a|b)`` and a final ``(?P<n>.+)``, with an
    optional trailing ``/?``, as ``(spec, trailing_slash_allowed)``; None for anything else
    (matched as a regex)."""
    trailing = pattern.endswith("/?")
    body = pattern[:-2] if trailing else pattern
    parts = _SEG.findall(body)
    if not parts or "".join("/" + x for x in parts) != body:
        return None
    spec = []
    last = len(parts) - 1
    for i, part in enumerate(parts):
        g = _GROUP.fullmatch(part)
        if g is not None:
            name, expr = g.groups()
            if expr == "[^/]+":
                spec.append(("param", name))
            elif expr == ".+" and i == last and not trailing:
                spec.append(("rest", name))
            elif _CHOICE.fullmatch(expr):
                spec.append(("choice", name, frozenset(expr.split("|"))))
            else:
                return None
        elif _LIT.fullmatch(part):
            spec.append(("lit", part))
        else:
            return None
    return tuple(spec), trailing


def _match_segments(spec, segs: list[str]):
    out = {}
    for i, s in enumerate(spec):
        if s[0] == "rest":
            rest = "/".join(segs[i:])
            if not rest:
                return None
            out[s[1]] = rest
            return out
        if i >= len(segs):
            return None
        seg = segs[i]
        if s[0] == "lit":
            if seg != s[1]:
                return None
        elif s[0] == "param":
            if not seg:
                return None
            out[s[1]] = seg
        elif seg not in s[2]:
            return None
        else:
            out[s[1]] = seg
    return out if len(segs) == len(spec) else None


_UNSET = object()


class Router:
    """Method + path-pattern routes, tried in order. Patterns built from plain segments (nearly
    all of the control plane's ~120) are matched segment by segment, without a regex; the rest
    are compiled. Either form is worked out the first time a path carrying the route's literal
    prefix reaches it. Compiling
    every route up front was 3.8 ms of the daemon's start on the MI355X host
    (profiles/r5_cp_trace/), and compiling on first use moved most of it into the bring-up's
    first workload request -- both on its critical path."""

    def __init__(self):
        # [method, literal prefix, pattern, compiled regex or None, handler, segment spec or None
        #  (_UNSET until a path first reaches the route)]
        self.routes: list[list] = []
        self._by_first: dict[str, list[list]] | None = None  # first path segment -> its routes, in order
        self._any_first: list[list] = []                      # routes whose first segment is not literal

    def add(self, method: str, pattern: str, handler: Handler) -> None:
        self.routes.append([method, _literal_prefix(pattern), pattern, None, handler, _UNSET])
        self._by_first = None

    @staticmethod
    def _first(prefix: str, pattern: str) -> str | None:
        """The route's literal first path segment, or None when a path of any first segment could
        match it."""
        if not prefix.startswith("/"):
            return None
        end = prefix.find("/", 1)
        if end > 0:
            return prefix[1:end]
        return prefix[1:] if prefix == pattern and len(prefix) > 1 else None

    def _index(self) -> None:
        firsts = [self._first(r[1], r[2]) for r in self.routes]
        keys = {f for f in firsts if f is not None}
        self._by_first = {k: [r for r, f in zip(self.routes, firsts) if f is None or f == k] for k in keys}
        self._any_first = [r for r, f in zip(self.routes, firsts) if f is None]

    def route(self, method: str, pattern: str):
        def deco(fn):
            self.add(method, pattern, fn)
            return fn
        return deco

    def match(self, method: str, path: str):
        allowed = False
        segs = path.split("/")[1:] if path.startswith("/") else None
        segs_t = segs[:-1] if segs and len(segs) > 1 and segs[-1] == "" else segs
        if self._by_first is None:
            self._index()
        routes = self._by_first.get(segs[0], self._any_first) if segs else self._any_first
        for r in routes:
            if not path.startswith(r[1]):
                continue
            seg = r[5]
            if seg is _UNSET:
                seg = r[5] = _segments(r[2])
            if seg is not None:
                if segs is None:
                    continue
                ps = segs_t if seg[1] else segs
                if len(ps) != len(seg[0]) and seg[0][-1][0] != "rest":
                    continue
                groups = _match_segments(seg[0], ps)
                if groups is None:
                    continue
            else:
                rx = r[3]
                if rx is None:
                    rx = r[3] = re.compile("^" + r[2] + "$")
                mt = rx.match(path)
                if not mt:
                    continue
                groups = mt.groupdict()
            m = r[0]
            if m == method or (m == "GET" and method == "HEAD"):
                return r[4], {k: unquote(v) for k, v in groups.items()}
            allowed = True
        if allowed:
            raise HttpError(405, f"method {method} not allowed on {path}")
        raise HttpError(404, f"no route for {method} {path}")


async def _read_request(reader: asyncio.StreamReader, peer: str) -> Request | None:
    try:
        head = await reader.readuntil(b"\r\n\r\n")
    except (asyncio.IncompleteReadError, ConnectionError):
        return None
    except asyncio.LimitOverrunError:
        raise HttpError(400, "headers too large")
    lines = head.decode("latin-1").split("\r\n")
    try:
        method, target, _ = lines[0].split(" ", 2)
    except ValueError:
        raise HttpError(400, "bad request line")
    headers = {}
    for line in lines[1:]:
        if ":" in line:
            k, v = line.split(":", 1)
            headers[k.strip().lower()] = v.strip()
    body = b""
    n = int(headers.get("content-length", "0") or 0)
    if n:
        body = await reader.readexactly(n)
    u = urlsplit(target)
    query = {k: v[-1] for k, v in parse_qs(u.query, keep_blank_values=True).items()}
    return Request(method.upper(), u.path or "/", query, headers, body, peer, u.query)


class HttpServer:
    def __init__(self, router: Router, on_error: Callable[[str], None] | None = None,
                 error_body: Callable[[str, HttpError], Any] | None = None,
                 observe: Callable[[str, str, bool, int, float], None] | None = None):
        self.router = router
        self.observe = observe  # (method, path, watch, status, seconds) of every request
        self.on_error = on_error
        self.error_body = error_body  # path, error -> body (e.g. a Kubernetes Status on API paths)
        self.server: asyncio.base_events.Server | None = None

    def _error(self, path: str, e: HttpError) -> Response:
        body = e.body
        if self.error_body is not None and not e.custom_body:
            body = self.error_body(path, e)
        return Response(e.status, body)

    async def _handle(self, reader: asyncio.StreamReader, writer: asyncio.StreamWriter) -> None:
        peer = "%s:%s" % (writer.get_extra_info("peername") or ("?", 0))[:2]
        try:
            while True:
                try:
                    req = await _read_request(reader, peer)
                except HttpError as e:
                    await self._send(writer, Response(e.status, e.body), keep=False, head=False)
                    return
                if req is None:
                    return
                t0 = time.perf_counter()
                try:
                    handler, params = self.router.match(req.method, req.path)
                    res = await handler(req, **params)
                    if not isinstance(res, (Response, StreamResponse, WebSocketResponse)):
                        res = Response(200, res)
                except HttpError as e:
                    res = self._error(req.path, e)
                except Exception as e:  # noqa: BLE001 - keep the server alive
                    if self.on_error:
                        self.on_error(traceback.format_exc())
                    res = self._error(req.path, HttpError(500, repr(e)))
                if self.observe is not None:
                    self.observe(req.method, req.path, req.query.get("watch") in ("1", "true"),
                                 101 if isinstance(res, WebSocketResponse) else getattr(res, "status", 200),
                                 time.perf_counter() - t0)
                keep = req.headers.get("connection", "").lower() != "close"
                if isinstance(res, WebSocketResponse):
                    hdr = ["HTTP/1.1 101 Switching Protocols", "Upgrade: websocket", "Connection: Upgrade",
                           f"Sec-WebSocket-Accept: {websocket_accept(req.headers.get('sec-websocket-key', ''))}"]
                    if res.protocol:
                        hdr.append(f"Sec-WebSocket-Protocol: {res.protocol}")
                    writer.write(("\r\n".join(hdr) + "\r\n\r\n").encode("latin-1"))
                    await writer.drain()
                    ws = WebSocket(reader, writer)
                    try:
                        await res.session(ws)
                    finally:
                        await ws.close()
                    return
                if isinstance(res, StreamResponse):
                    await self._stream(writer, res, keep=keep)
                else:
                    await self._send(writer, res, keep=keep, head=req.method == "HEAD")
                if not keep:
                    return
        except (ConnectionError, asyncio.IncompleteReadError):
            return
        finally:
            try:
                writer.close()
            except Exception:  # noqa: BLE001
                pass

    @staticmethod
    async def _send(writer: asyncio.StreamWriter, res: Response, keep: bool, head: bool) -> None:
        body, ctype = res.encode()
        hdr = [f"HTTP/1.1 {res.status} {REASONS.get(res.status, 'Status')}",
               f"Content-Type: {ctype}", f"Content-Length: {len(body)}",
               f"Connection: {'keep-alive' if keep else 'close'}"]
        hdr += [f"{k}: {v}" for k, v in res.headers.items()]
        writer.write(("\r\n".join(hdr) + "\r\n\r\n").encode("latin-1") + (b"" if head else body))
        await writer.drain()

    @staticmethod
    async def _stream(writer: asyncio.StreamWriter, res: StreamResponse, keep: bool) -> None:
        hdr = [f"HTTP/1.1 {res.status} {REASONS.get(res.status, 'Status')}", f"Content-Type: {res.content_type}",
               "Transfer-Encoding: chunked", "Cache-Control: no-cache, private",
               f"Connection: {'keep-alive' if keep else 'close'}"]
        hdr += [f"{k}: {v}" for k, v in res.headers.items()]
        writer.write(("\r\n".join(hdr) + "\r\n\r\n").encode("latin-1"))
        await writer.drain()
        try:
            async for chunk in res.chunks:
                if chunk:
                    writer.write(b"%x\r\n%s\r\n" % (len(chunk), chunk))
                    await writer.drain()
        finally:
            aclose = getattr(res.chunks, "aclose", None)
            if aclose is not None:
                await aclose()
        writer.write(b"0\r\n\r\n")
        await writer.drain()

    async def start(self, host: str, port: int) -> tuple[str, int]:
        self.server = await asyncio.start_server(self._handle, host, port, reuse_address=True, limit=1 << 20)
        sock = self.server.sockets[0].getsockname()
        return sock[0], sock[1]

    async def close(self) -> None:
        if self.server:
            self.server.close()
            await self.server.wait_closed()
