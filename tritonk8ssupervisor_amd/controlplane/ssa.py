"""Managed fields and server-side apply (``kubectl apply --server-side``): who set which field of
an object, and an apply that merges a manager's configuration into the live object, reports
conflicts with other managers, and removes the fields the manager stopped applying.

The model, kept to what the kinds served here need:

* A *field path* is a tuple of FieldsV1 segments: ``f:<field>`` for a map key, ``k:{"name":"x"}``
  for an element of a list with a merge key (``k8s_wire.MERGE_KEYS``), and ``.`` for such an
  element itself. Lists without a merge key are atomic (one leaf), as in Kubernetes.
  ``apiVersion``, ``kind``, ``status`` and the identity fields of ``metadata`` are nobody's;
  ``metadata.labels`` and ``metadata.annotations`` are managed per key.
* ``metadata.managedFields`` holds one entry per (manager, operation, subresource) with its set
  encoded as FieldsV1 -- the format stock kubectl shows with ``--show-managed-fields``.
* **Apply** (``PATCH`` with ``application/apply-patch+yaml``): a field the manager applies with a
  value different from the live one, owned by another manager, is a conflict (409 with one cause
  per field) unless ``force=true`` moves it to the applier; applied with the same value, it is
  shared. Fields the manager applied last time and no longer applies are removed unless another
  manager still owns them. The object is created when it does not exist.
* **Update** (create, PUT, merge/JSON/strategic patch, the scale subresource): the manager takes
  the fields whose value it changed; other managers lose them.

Not modelled: set-type lists (``v:`` segments), multi-key merge keys (container ports key on
``containerPort`` alone), per-version field sets, and the conversion of managed fields between
API versions (one version per kind here).
"""
from __future__ import annotations

import copy
import json
import time

from . import k8s_wire

_MISSING = object()
_IDENTITY = {"name", "generateName", "namespace", "uid", "resourceVersion", "generation", "creationTimestamp",
             "deletionTimestamp", "deletionGracePeriodSeconds", "managedFields", "selfLink", "ownerReferences",
             "finalizers"}

Path = tuple


class Conflict(Exception):
    def __init__(self, conflicts: list[tuple[str, str, str]]):  # (manager, apiVersion, dotted field)
        super().__init__(f"Apply failed with {len(conflicts)} conflict(s)")
        self.conflicts = conflicts

    def status(self) -> dict:
        causes = [{"type": "FieldManagerConflict", "message": f'conflict with "{m}" using {v}', "field": f}
                  for m, v, f in self.conflicts]
        lines = "\n".join(f'- conflict with "{m}" using {v}: {f}' for m, v, f in self.conflicts)
        return {"kind": "Status", "apiVersion": "v1", "metadata": {}, "status": "Failure", "reason": "Conflict",
                "code": 409, "message": f"Apply failed with {len(self.conflicts)} conflict(s):\n{lines}",
                "details": {"causes": causes}}


def _merge_key(field: str | None, items: list) -> str | None:
    if field not in k8s_wire.MERGE_KEYS or not items:
        return None
    key = k8s_wire.MERGE_KEYS[field] or (k8s_wire._ports_key(items) if field == "ports" else None)
    if key and all(isinstance(i, dict) and key in i for i in items):
        return key
    return None


def _kseg(item: dict, key: str) -> str:
    return "k:" + json.dumps({key: item[key]}, separators=(",", ":"), sort_keys=True)


def field_paths(obj: dict) -> set[Path]:
    """The leaf field paths an object (or an applied configuration) sets."""
    out: set[Path] = set()

    def walk(node, path: Path, field: str | None):
        if isinstance(node, dict) and node:
            for k, v in node.items():
                walk(v, path + (f"f:{k}",), k)
        elif isinstance(node, list) and (key := _merge_key(field, node)):
            for it in node:
                p = path + (_kseg(it, key),)
                out.add(p + (".",))
                for k, v in it.items():
                    walk(v, p + (f"f:{k}",), k)
        else:
            out.add(path)

    for k, v in (obj or {}).items():
        if k in ("apiVersion", "kind", "status") or k.startswith("_"):
            continue
        if k == "metadata":
            for mk, mv in (v or {}).items():
                if mk in ("labels", "annotations") and isinstance(mv, dict):
                    for lk, lv in mv.items():
                        out.add(("f:metadata", f"f:{mk}", f"f:{lk}"))
                elif mk not in _IDENTITY:
                    walk(mv, ("f:metadata", f"f:{mk}"), mk)
            continue
        walk(v, (f"f:{k}",), k)
    return out


def _find(lst: list, seg: str):
    want = json.loads(seg[2:])
    for i, it in enumerate(lst):
        if isinstance(it, dict) and all(it.get(k) == v for k, v in want.items()):
            return i
    return None


def get(obj, path: Path):
    cur = obj
    for seg in path:
        if seg == ".":
            return cur
        if seg.startswith("f:"):
            if not isinstance(cur, dict) or seg[2:] not in cur:
                return _MISSING
            cur = cur[seg[2:]]
        else:
            if not isinstance(cur, list):
                return _MISSING
            i = _find(cur, seg)
            if i is None:
                return _MISSING
            cur = cur[i]
    return cur


def remove(obj, path: Path) -> None:
    """Delete the field (or, for a path ending in ``.``, the list element) at ``path``."""
    if not path:
        return
    if path[-1] == ".":
        lst = get(obj, path[:-2])
        if isinstance(lst, list) and (i := _find(lst, path[-2])) is not None:
            lst.pop(i)
        return
    parent = get(obj, path[:-1])
    last = path[-1]
    if isinstance(parent, dict) and last.startswith("f:"):
        parent.pop(last[2:], None)


def dotted(path: Path) -> str:
    out = ""
    for seg in path:
        if seg == ".":
            continue
        out += "." + seg[2:] if seg.startswith("f:") else f"[{seg[2:]}]"
    return out or "."


def to_fieldsv1(paths: set[Path]) -> dict:
    root: dict = {}
    for p in sorted(paths):
        node = root
        for seg in p:
            node = node.setdefault(seg, {})
    return root


def from_fieldsv1(tree: dict) -> set[Path]:
    out: set[Path] = set()

    def walk(node: dict, path: Path):
        if not node:
            if path:
                out.add(path)
            return
        for k, v in node.items():
            walk(v if isinstance(v, dict) else {}, path + (k,))

    walk(tree or {}, ())
    return out


def _now() -> str:
    return time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())


class Managed:
    """``metadata.managedFields`` as {(manager, operation, subresource): set of paths}."""

    def __init__(self, entries: list | None, api_version: str):
        self.api_version = api_version
        self.sets: dict[tuple[str, str, str], set[Path]] = {}
        for e in entries or []:
            if isinstance(e, dict) and e.get("manager") is not None:
                k = (e["manager"], e.get("operation", "Update"), e.get("subresource", ""))
                self.sets[k] = from_fieldsv1(e.get("fieldsV1") or {})

    def entries(self) -> list[dict]:
        out = []
        for (m, op, sub), s in self.sets.items():
            if not s:
                continue
            e = {"manager": m, "operation": op, "apiVersion": self.api_version, "time": _now(),
                 "fieldsType": "FieldsV1", "fieldsV1": to_fieldsv1(s)}
            if sub:
                e["subresource"] = sub
            out.append(e)
        return out

    def others(self, key) -> set[Path]:
        return set().union(*(s for k, s in self.sets.items() if k != key)) if len(self.sets) > 1 else set()

    def update(self, old: dict | None, new: dict, manager: str, subresource: str = "") -> None:
        """An Update by ``manager``: it takes every field whose value it set or changed; fields that
        disappeared are nobody's any more."""
        new_paths = field_paths(new)
        changed = {p for p in new_paths if old is None or get(old, p) != get(new, p)}
        for s in self.sets.values():
            s -= changed
            s &= new_paths
        key = (manager, "Update", subresource)
        self.sets.setdefault(key, set()).update(changed)
        self.sets = {k: s for k, s in self.sets.items() if s}


def apply(live: dict | None, applied: dict, manager: str, force: bool, api_version: str) -> dict:
    """Server-side apply of ``applied`` by ``manager`` onto ``live`` (None: create). Returns the
    new object with its ``metadata.managedFields``; raises Conflict."""
    cur = copy.deepcopy(live) if live is not None else {}
    managed = Managed((cur.get("metadata") or {}).get("managedFields"), api_version)
    key = (manager, "Apply", "")
    new_set = field_paths(applied)
    conflicts = []
    for k, owned in managed.sets.items():
        if k == key:
            continue
        for p in sorted(owned & new_set):
            if p[-1] == ".":
                continue
            have = get(cur, p)
            if have is not _MISSING and have != get(applied, p):
                conflicts.append((k, p))
    if conflicts and not force:
        raise Conflict([(k[0], api_version, dotted(p)) for k, p in conflicts])
    for k, p in conflicts:  # force: the applier takes them
        managed.sets[k].discard(p)
    # what this manager applied before and no longer applies goes, unless someone else owns it
    others = managed.others(key)
    dropped = managed.sets.get(key, set()) - new_set
    # whole list elements first (outermost first), then leaves: removing a leaf of an element
    # could remove its merge key, after which the element could no longer be found
    for p in sorted(dropped, key=lambda p: (p[-1] != ".", len(p) if p[-1] == "." else -len(p))):
        if p in others:
            continue
        if p[-1] == "." and any(o[:len(p) - 1] == p[:-1] for o in others):
            continue  # another manager still owns a field of this element
        remove(cur, p)
    body = copy.deepcopy(applied)
    md_in = body.get("metadata") or {}
    out = k8s_wire.strategic_merge(cur, {k: v for k, v in body.items() if k != "metadata"})
    md = out.setdefault("metadata", {})
    for mk in ("labels", "annotations"):
        if isinstance(md_in.get(mk), dict):
            md.setdefault(mk, {}).update(md_in[mk])
    for mk, mv in md_in.items():
        if mk not in ("labels", "annotations") and mk not in _IDENTITY:
            md[mk] = mv
    for mk in ("name", "namespace", "generateName"):
        if mk in md_in and mk not in md:
            md[mk] = md_in[mk]
    out.setdefault("apiVersion", applied.get("apiVersion"))
    out.setdefault("kind", applied.get("kind"))
    managed.sets[key] = new_set
    managed.sets = {k: s for k, s in managed.sets.items() if s}
    md["managedFields"] = managed.entries()
    return out
