"""YAML loading through libyaml when the C extension is present (5-10x faster than the pure
Python loader; the playbook engine parses every role file on each bring-up), behind a parse
cache.

Importing PyYAML costs more than parsing every file of a bring-up (its resolver and reader
compile dozens of regexes at import: ~10 ms on the MI355X host, on the critical path of
``./setup.sh``). The playbooks, roles, group_vars and manifests are the same text on every
bring-up, so -- like Python's own .pyc cache -- a parse result is kept in
``$XDG_STATE_HOME/tk8s/yaml`` (``TK8S_YAML_CACHE=<dir>`` or ``off``), keyed by the text's
length and checksums and stored WITH the text, which must match exactly before the cached
data is used: a hit returns exactly what the parser would. The entries are ``marshal`` data this
module wrote itself (plain dicts, lists and scalars; a document with types marshal cannot hold,
e.g. timestamps, is simply not cached).
"""
from __future__ import annotations

import marshal
import os
import zlib

_VERSION = "1"
_yaml_mod = None


def _parser():
    global _yaml_mod
    if _yaml_mod is None:
        import yaml

        _yaml_mod = (yaml, getattr(yaml, "CSafeLoader", yaml.SafeLoader))
    return _yaml_mod


def _cache_path(raw: bytes, kind: str) -> str | None:
    d = os.environ.get("TK8S_YAML_CACHE", "")
    if d == "off":
        return None
    if not d:
        from .pcache import state_home

        d = os.path.join(state_home(), "yaml")
    return os.path.join(d, f"{len(raw)}-{zlib.crc32(raw):08x}-{zlib.adler32(raw):08x}-{kind}{_VERSION}.marshal")


def _cached(text: str, kind: str, parse):
    raw = text.encode("utf-8", "surrogatepass")
    path = _cache_path(raw, kind)
    if path is not None:
        try:
            with open(path, "rb") as f:
                stored, data = marshal.load(f)
            if stored == text:
                return data
        except (OSError, ValueError, EOFError, TypeError):
            pass
    data = parse(text)
    if path is not None:
        try:
            blob = marshal.dumps((text, data))
        except ValueError:  # a type marshal cannot hold (e.g. a YAML timestamp): not cached
            return data
        try:
            d = os.path.dirname(path)
            os.makedirs(d, exist_ok=True)
            tmp = f"{path}.{os.getpid()}.tmp"
            with open(tmp, "wb") as f:
                f.write(blob)
            os.replace(tmp, path)
            _prune(d)
        except OSError:
            pass
    return data


def _prune(d: str, keep: int = 2048) -> None:
    """Generated YAML (per-cluster vars files, user manifests) adds entries: keep the cache
    bounded by dropping the least recently written half once it outgrows ``keep``."""
    names = os.listdir(d)
    if len(names) <= keep:
        return
    def mtime(q: str) -> int:
        try:
            return os.stat(q).st_mtime_ns
        except OSError:
            return 0

    paths = sorted((os.path.join(d, n) for n in names), key=mtime)
    for q in paths[: len(paths) // 2]:
        try:
            os.unlink(q)
        except OSError:
            pass


def _load(text: str):
    yaml, loader = _parser()
    return yaml.load(text, Loader=loader)  # noqa: S506 - CSafeLoader/SafeLoader only


def _load_all(text: str):
    yaml, loader = _parser()
    return list(yaml.load_all(text, Loader=loader))  # noqa: S506


def load(text: str):
    return _cached(text, "doc", _load)


def flat_mapping(data: dict) -> str:
    """A flat ``key: value`` YAML mapping whose values are JSON scalars (a JSON string is a YAML
    double-quoted scalar with the same escapes), seeded into the parse cache: a file the
    orchestrator generates per bring-up (the role vars) then never needs the parser."""
    if not all(isinstance(k, str) and k.isidentifier() for k in data) or not all(
            v is None or isinstance(v, (str, int, bool)) for v in data.values()):
        raise ValueError("flat_mapping takes identifier keys and str/int/bool/None values")
    import json

    text = "".join(f"{k}: {json.dumps(v, ensure_ascii=True)}\n" for k, v in data.items())
    _cached(text, "doc", lambda _t: dict(data))
    return text


def load_all(text: str) -> list:
    return _cached(text, "all", _load_all)
