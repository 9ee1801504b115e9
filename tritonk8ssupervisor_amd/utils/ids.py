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


def uuid5(namespace: str, name: str) -> str:
    ns = bytes.fromhex(namespace.replace("-", ""))
    h = bytearray(sha1(ns + name.encode("utf-8")).digest()[:16])
    h[6] = (h[6] & 0x0F) | 0x50  # version 5
    h[8] = (h[8] & 0x3F) | 0x80  # RFC 4122 variant
    x = h.hex()
    return f"{x[:8]}-{x[8:12]}-{x[12:16]}-{x[16:20]}-{x[20:]}"
