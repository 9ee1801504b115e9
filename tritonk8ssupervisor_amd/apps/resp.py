"""RESP2 (the Redis protocol): encoding and a small synchronous client."""
from __future__ import annotations

import socket


class RespError(Exception):
    """A ``-ERR ...`` reply (or one to send)."""


class Status(str):
    """A ``+OK``-style simple string."""


def encode(v) -> bytes:
    if v is None:
        return b"$-1\r\n"
    if isinstance(v, RespError):
        return b"-" + str(v).encode() + b"\r\n"
    if isinstance(v, Status):
        return b"+" + v.encode() + b"\r\n"
    if isinstance(v, bool):
        v = int(v)
    if isinstance(v, int):
        return b":%d\r\n" % v
    if isinstance(v, str):
        v = v.encode()
    if isinstance(v, (bytes, bytearray)):
        return b"$%d\r\n%s\r\n" % (len(v), bytes(v))
    if isinstance(v, (list, tuple)):
        return b"*%d\r\n" % len(v) + b"".join(encode(x) for x in v)
    raise TypeError(f"cannot encode {type(v).__name__} as RESP")


def command(*args) -> bytes:
    return encode([a if isinstance(a, (bytes, bytearray)) else str(a).encode() for a in args])


def read_reply(f):
    """One reply from a binary file-like object (socket.makefile('rb'))."""
    line = f.readline()
    if not line:
        raise ConnectionError("connection closed")
    t, rest = line[:1], line[1:].rstrip(b"\r\n")
    if t == b"+":
        return Status(rest.decode())
    if t == b"-":
        raise RespError(rest.decode(errors="replace"))
    if t == b":":
        return int(rest)
    if t == b"$":
        n = int(rest)
        return None if n < 0 else f.read(n + 2)[:-2]
    if t == b"*":
        n = int(rest)
        return None if n < 0 else [read_reply(f) for _ in range(n)]
    raise RespError(f"protocol error: {line[:40]!r}")


def call(host: str, port: int, *args, timeout: float = 5.0):
    """Send one command, return its reply (RespError for an error reply)."""
    with socket.create_connection((host, port), timeout=timeout) as s:
        s.sendall(command(*args))
        with s.makefile("rb") as f:
            return read_reply(f)
