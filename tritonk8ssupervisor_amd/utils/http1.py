"""A small HTTP/1.1 client connection over a plain socket.

``http.client`` imports ``email.parser``, ``ssl`` and friends: ~5 ms on the MI355X host (~20 ms
on slow CPUs) in every tk8s process that talks to the control plane -- ``./setup.sh``, the node
agents, the validation payloads -- most of them on the bring-up's critical path. The control
plane and the kubelet-facing endpoints tk8s talks to are plain-HTTP, JSON, HTTP/1.1 servers;
this connection speaks exactly that: one request at a time, keep-alive, bodies delimited by
Content-Length, chunked transfer encoding or connection close. HTTPS is not handled here
(callers fall back to ``http.client`` for it).
"""
from __future__ import annotations

import _socket
import io

# ``_socket``, not ``socket``: the latter turns hundreds of constants into enums on import (~3 ms,
# ~1.5 ms on the MI355X host) in every process on the bring-up's path that only needs a TCP
# connection to the control plane.


class _SockReader(io.RawIOBase):
    """What ``socket.makefile("rb")`` wraps, for a bare ``_socket.socket``."""

    def __init__(self, sock):
        self._sock = sock

    def readable(self) -> bool:
        return True

    def readinto(self, b) -> int:
        return self._sock.recv_into(b)


def create_connection(host, port: int, timeout: float | None):
    """``socket.create_connection`` on ``_socket``: the first address of ``host`` that connects."""
    err: OSError | None = None
    for af, st, proto, _canon, addr in _socket.getaddrinfo(host, port, 0, _socket.SOCK_STREAM):
        s = _socket.socket(af, st, proto)
        try:
            s.settimeout(timeout)
            s.connect(addr)
            return s
        except OSError as e:
            err = e
            s.close()
    raise err or OSError(f"no address for {host!r}")


class ProtocolError(OSError):
    """The peer sent something that is not an HTTP/1.1 response (or closed mid-response)."""


class Response:
    __slots__ = ("status", "reason", "headers", "body")

    def __init__(self, status: int, reason: str, headers: dict[str, str], body: bytes):
        self.status, self.reason, self.headers, self.body = status, reason, headers, body

    def header(self, name: str, default: str = "") -> str:
        return self.headers.get(name.lower(), default)


class Connection:
    """One keep-alive connection to host:port. Not thread-safe (callers serialise)."""

    def __init__(self, host: str, port: int, timeout: float | None = 30.0):
        self.host, self.port, self.timeout = host, port, timeout
        self.sock = None  # a _socket.socket once connected
        self._rf = None

    def _connect(self) -> None:
        # an ASCII host goes to getaddrinfo as bytes: a str host is IDNA-encoded first, which
        # imports encodings.idna + stringprep + unicodedata (~1 ms) for a dotted-quad address
        host = self.host.encode("ascii") if self.host.isascii() else self.host
        self.sock = create_connection(host, self.port, self.timeout)
        self.sock.setsockopt(_socket.IPPROTO_TCP, _socket.TCP_NODELAY, 1)
        self._rf = io.BufferedReader(_SockReader(self.sock))

    def set_timeout(self, timeout: float | None) -> None:
        self.timeout = timeout
        if self.sock is not None:
            self.sock.settimeout(timeout)

    def close(self) -> None:
        if self._rf is not None:
            try:
                self._rf.close()
            except OSError:
                pass
        if self.sock is not None:
            try:
                self.sock.close()
            except OSError:
                pass
        self.sock = self._rf = None

    @property
    def connected(self) -> bool:
        return self.sock is not None

    def request(self, method: str, target: str, body: bytes | None = None,
                headers: dict[str, str] | None = None) -> Response:
        if self.sock is None:
            self._connect()
        hdrs = {"Host": f"{self.host}:{self.port}", **(headers or {})}
        if body is not None or method in ("POST", "PUT", "PATCH"):
            hdrs["Content-Length"] = str(len(body or b""))
        head = f"{method} {target} HTTP/1.1\r\n" + "".join(f"{k}: {v}\r\n" for k, v in hdrs.items()) + "\r\n"
        try:
            self.sock.sendall(head.encode("latin-1") + (body or b""))
            res = self._read_response(method)
        except BaseException:
            self.close()
            raise
        if res.header("connection").lower() == "close":
            self.close()
        return res

    def _line(self) -> bytes:
        line = self._rf.readline(65537)
        if not line:
            raise ProtocolError("connection closed by the server")
        if len(line) > 65536:
            raise ProtocolError("header line too long")
        return line

    def _read_response(self, method: str) -> Response:
        while True:
            status_line = self._line().decode("latin-1").rstrip("\r\n")
            parts = status_line.split(" ", 2)
            if len(parts) < 2 or not parts[0].startswith("HTTP/1."):
                raise ProtocolError(f"bad status line {status_line!r}")
            try:
                status = int(parts[1])
            except ValueError as e:
                raise ProtocolError(f"bad status line {status_line!r}") from e
            headers: dict[str, str] = {}
            while True:
                line = self._line()
                if line in (b"\r\n", b"\n"):
                    break
                k, sep, v = line.decode("latin-1").partition(":")
                if not sep:
                    raise ProtocolError(f"bad header line {line!r}")
                k = k.strip().lower()
                v = v.strip()
                headers[k] = f"{headers[k]}, {v}" if k in headers else v
            if 100 <= status < 200 and status != 101:
                continue  # an interim response (100 Continue): the real one follows
            break
        reason = parts[2] if len(parts) > 2 else ""
        if method == "HEAD" or status in (204, 304):
            return Response(status, reason, headers, b"")
        if "chunked" in headers.get("transfer-encoding", "").lower():
            chunks = []
            while True:
                size_line = self._line().split(b";", 1)[0].strip()
                try:
                    n = int(size_line, 16)
                except ValueError as e:
                    raise ProtocolError(f"bad chunk size {size_line!r}") from e
                if n == 0:
                    while self._line() not in (b"\r\n", b"\n"):
                        pass  # trailers
                    break
                chunks.append(self._exact(n))
                self._exact(2)
            return Response(status, reason, headers, b"".join(chunks))
        if "content-length" in headers:
            try:
                n = int(headers["content-length"])
            except ValueError as e:
                raise ProtocolError("bad Content-Length") from e
            return Response(status, reason, headers, self._exact(n))
        body = self._rf.read()  # delimited by the connection closing
        headers["connection"] = "close"
        return Response(status, reason, headers, body)

    def _exact(self, n: int) -> bytes:
        data = self._rf.read(n)
        if len(data) != n:
            raise ProtocolError(f"connection closed after {len(data)} of {n} body bytes")
        return data
