"""Cluster key material and fingerprint discovery (setup.sh:209-239 analogue).

The reference finds the private key in ~/.ssh whose MD5 fingerprint equals SDC_KEY_ID. The local
provider owns a per-cluster key pair instead; the fingerprint has the same `aa:bb:..` MD5 format
so SDC_KEY_ID keeps its meaning, and the PUBLIC key is what machines authorise (the reference
passes the private key path as root_authorized_keys, SURVEY.md §2.2 quirk — not replicated).
"""
from __future__ import annotations

import binascii
import os
from pathlib import Path

try:  # the builtin hash modules: hashlib (OpenSSL) costs more to import than the bring-up hashes
    from _md5 import md5
    from _sha256 import sha256
except ImportError:
    from hashlib import md5, sha256

from ..utils.fsutil import atomic_write

KEY_NAME = "tk8s_cluster_key"


def fingerprint_md5(public_blob: bytes) -> str:
    h = md5(public_blob).hexdigest()
    return ":".join(h[i : i + 2] for i in range(0, 32, 2))


def public_line(private: bytes) -> str:
    pub = sha256(b"tk8s-public:" + private).digest()
    return f"tk8s-key {binascii.b2a_base64(pub, newline=False).decode()} tk8s"


def ensure_cluster_key(key_dir: str | os.PathLike) -> tuple[Path, Path, str]:
    """Create (once) the cluster key; returns (private_path, public_path, fingerprint)."""
    d = Path(key_dir)
    d.mkdir(parents=True, exist_ok=True)
    priv, pub = d / KEY_NAME, d / f"{KEY_NAME}.pub"
    if not priv.exists():
        atomic_write(priv, os.urandom(32).hex() + "\n", mode=0o600)
    line = public_line(priv.read_bytes().strip())
    if not pub.exists() or pub.read_text().strip() != line:
        atomic_write(pub, line + "\n", mode=0o644)
    return priv, pub, fingerprint_md5(binascii.a2b_base64(line.split()[1]))


def key_fingerprint(pub_path: str | os.PathLike) -> str | None:
    try:
        parts = Path(pub_path).read_text().split()
        return fingerprint_md5(binascii.a2b_base64(parts[1]))
    except (OSError, IndexError, ValueError):
        return None


def find_key(key_id: str, search_dirs: list[str | os.PathLike]) -> str | None:
    """Private key path whose public half has MD5 fingerprint `key_id` (W4 scan)."""
    want = key_id.lower().removeprefix("md5:")
    for d in search_dirs:
        d = Path(d).expanduser()
        if not d.is_dir():
            continue
        for pub in sorted(d.glob("*.pub")):
            if key_fingerprint(pub) == want and pub.with_suffix("").exists():
                return str(pub.with_suffix(""))
    return None
