"""Name-based UUIDs (RFC 4122 version 5) without importing ``uuid``.

``uuid`` imports ``platform`` and friends (~1.5 ms on the MI355X host) just to hash a name; the
providers derive every machine / network / package id this way on the bring-up path. The
result is identical to ``str(uuid.uuid5(uuid.UUID(namespace), name))`` (pinned by
tests/test_runtime_utils.py).
"""
from __future__ import annotations

try:
    from _sha1 import sha1
except ImportError:  # an interpreter without the builtin module
    from hashlib import sha1


def _fmt(h: bytearray) -> str:
    x = h.hex()
    return f"{x[:8]}-{x[8:12]}-{x[12:16]}-{x[16:20]}-{x[20:]}"


def uuid4() -> str:
    """``str(uuid.uuid4())``: 122 random bits from os.urandom, version 4, RFC 4122 variant."""
    import os

    h = bytearray(os.urandom(16))
    h[6] = (h[6] & 0x0F) | 0x40
    h[8] = (h[8] & 0x3F) | 0x80
    return _fmt(h)


def token_hex(nbytes: int) -> str:
    """``secrets.token_hex(nbytes)`` (which is ``os.urandom(nbytes).hex()``) without importing
    secrets -> random, hmac, hashlib, base64 (~1.5 ms in the control plane's start)."""
    import os

    return os.urandom(nbytes).hex()


def uuid5(namespace: str, name: str) -> str:
    ns = bytes.fromhex(namespace.replace("-", ""))
    h = bytearray(sha1(ns + name.encode("utf-8")).digest()[:16])
    h[6] = (h[6] & 0x0F) | 0x50  # version 5
    h[8] = (h[8] & 0x3F) | 0x80  # RFC 4122 variant
    return _fmt(h)
