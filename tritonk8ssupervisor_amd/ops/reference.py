"""Exact host oracles for the tk8s HIP kernels (numpy / hashlib; no GPU).

* :func:`philox4x32_10` / :func:`philox_bytes` — bit-exact model of ``philox_fill``
  (native/src/stream_kernels.hip): Random123 Philox4x32-10, counter = (block index lo, hi, 0, 0),
  key = (seed lo, seed hi).
* :func:`md5_tree` — the chunked, fan-in-4 MD5 tree of ``md5_tree`` (native/src/md5_kernels.hip), built
  from :mod:`hashlib` MD5 so the GPU digest can be checked against an independent implementation.
* :func:`allreduce_expected` — value of the N6 pattern after a sum all-reduce.

Reference anchor: docs/benchmarks.md:11-12 (the /cpu benchmark md5-hashes random numbers).
"""
from __future__ import annotations

import hashlib

import numpy as np

_M0 = np.uint64(0xD2511F53)
_M1 = np.uint64(0xCD9E8D57)
_W0 = 0x9E3779B9
_W1 = 0xBB67AE85
_MASK = np.uint64(0xFFFFFFFF)


def philox4x32_10(ctr: np.ndarray, key: tuple[int, int]) -> np.ndarray:
    """Philox4x32-10 over counters ``ctr`` (shape [n, 4], uint32) with key (k0, k1)."""
    c = ctr.astype(np.uint64)
    c0, c1, c2, c3 = c[:, 0], c[:, 1], c[:, 2], c[:, 3]
    k0, k1 = int(key[0]) & 0xFFFFFFFF, int(key[1]) & 0xFFFFFFFF
    for r in range(10):
        if r:
            k0 = (k0 + _W0) & 0xFFFFFFFF
            k1 = (k1 + _W1) & 0xFFFFFFFF
        p0 = _M0 * c0
        p1 = _M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & _MASK
        hi1, lo1 = p1 >> np.uint64(32), p1 & _MASK
        c0, c1, c2, c3 = hi1 ^ c1 ^ np.uint64(k0), lo1, hi0 ^ c3 ^ np.uint64(k1), lo0
    return np.stack([c0, c1, c2, c3], axis=1).astype(np.uint32)


def philox_bytes(nbytes: int, seed: int) -> bytes:
    """Bytes written by ``philox_fill(dst, nbytes, seed)`` (nbytes multiple of 16)."""
    if nbytes % 16:
        raise ValueError("nbytes must be a multiple of 16")
    n = nbytes // 16
    idx = np.arange(n, dtype=np.uint64)
    ctr = np.zeros((n, 4), dtype=np.uint32)
    ctr[:, 0] = (idx & _MASK).astype(np.uint32)
    ctr[:, 1] = (idx >> np.uint64(32)).astype(np.uint32)
    out = philox4x32_10(ctr, (seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF))
    return out.astype("<u4").tobytes()


def md5_tree(data: bytes, chunk_bytes: int = 1024, fan_in: int = 4) -> bytes:
    """MD5 tree: hash each ``chunk_bytes`` chunk (one chunk: its plain MD5), then fold the
    digests ``fan_in`` at a time -- a parent is the MD5 of its children's concatenated digests --
    until one remains."""
    if chunk_bytes <= 0 or chunk_bytes % 64:
        raise ValueError("chunk_bytes must be a positive multiple of 64")
    data = bytes(data)
    if len(data) <= chunk_bytes:
        return hashlib.md5(data).digest()
    level = [hashlib.md5(data[i : i + chunk_bytes]).digest() for i in range(0, len(data), chunk_bytes)]
    while len(level) > 1:
        level = [hashlib.md5(b"".join(level[i : i + fan_in])).digest() for i in range(0, len(level), fan_in)]
    return level[0]


def allreduce_expected(count: int, nranks: int) -> np.ndarray:
    """fp32 reference of the N6 pattern: sum over ranks r of (r + 1) + (i % 7)."""
    i = np.arange(count)
    per_rank = np.stack([(r + 1) + (i % 7) for r in range(nranks)]).astype(np.float32)
    return per_rank.sum(axis=0, dtype=np.float32)
