"""Placement rules the scheduler applies on top of GPU counts and nodeSelector (scheduler.py):

* **taints and tolerations** -- a node's ``NoSchedule``/``NoExecute`` taints keep pods off it
  unless they tolerate them (``Equal``/``Exists``, an empty key with ``Exists`` tolerates
  everything); ``PreferNoSchedule`` only lowers the node's score.
* **node affinity** -- ``requiredDuringSchedulingIgnoredDuringExecution.nodeSelectorTerms``
  (terms OR'ed, ``matchExpressions`` with In/NotIn/Exists/DoesNotExist/Gt/Lt and
  ``matchFields`` on ``metadata.name`` AND'ed) filters; ``preferred...`` terms add their weight.
* **inter-pod (anti-)affinity** -- required terms (``labelSelector`` + ``topologyKey``, the pod's
  namespace or ``namespaces``) filter nodes by the pods already bound in the same topology
  domain; preferred terms add or subtract their weight. Anti-affinity on
  ``kubernetes.io/hostname`` is how a job spreads one rank per MI355X node.

* **topology spread** -- ``topologySpreadConstraints`` (``maxSkew``, ``topologyKey``,
  ``labelSelector``, ``whenUnsatisfiable``): ``DoNotSchedule`` keeps a pod out of a domain that
  would then hold more than ``maxSkew`` matching pods above the emptiest eligible domain;
  ``ScheduleAnyway`` prefers the domains with fewer matching pods.

The scheduler keeps its GPU-packing order and uses these scores first (higher is better).
"""
from __future__ import annotations

from .objects import labels_match


def _expr_ok(expr: dict, value: str | None) -> bool:
    op, vals = expr.get("operator"), [str(v) for v in expr.get("values") or []]
    if op == "In":
        return value is not None and value in vals
    if op == "NotIn":
        return value is None or value not in vals
    if op == "Exists":
        return value is not None
    if op == "DoesNotExist":
        return value is None
    if op in ("Gt", "Lt") and value is not None and vals:
        try:
            return int(value) > int(vals[0]) if op == "Gt" else int(value) < int(vals[0])
        except ValueError:
            return False
    return False


def selector_matches(sel: dict | None, labels: dict | None) -> bool:
    """A LabelSelector (matchLabels + matchExpressions)."""
    if not sel:
        return True
    labels = labels or {}
    if not labels_match(sel.get("matchLabels") or {}, labels):
        return False
    return all(_expr_ok(e, labels.get(e.get("key"))) for e in sel.get("matchExpressions") or [])


def _term_ok(term: dict, node: dict) -> bool:
    labels = node["metadata"].get("labels") or {}
    if not all(_expr_ok(e, labels.get(e.get("key"))) for e in term.get("matchExpressions") or []):
        return False
    fields = {"metadata.name": node["metadata"]["name"]}
    return all(_expr_ok(e, fields.get(e.get("key"))) for e in term.get("matchFields") or [])


def tolerates(pod: dict, node: dict) -> bool:
    tols = pod["spec"].get("tolerations") or []
    for t in (node.get("spec") or {}).get("taints") or []:
        if t.get("effect") not in ("NoSchedule", "NoExecute"):
            continue
        if not any(_tolerates(x, t) for x in tols):
            return False
    return True


def _tolerates(tol: dict, taint: dict) -> bool:
    if tol.get("effect") and tol["effect"] != taint.get("effect"):
        return False
    if tol.get("operator") == "Exists":
        return not tol.get("key") or tol["key"] == taint.get("key")
    return tol.get("key") == taint.get("key") and str(tol.get("value", "")) == str(taint.get("value", ""))


def _pod_terms(pod: dict, kind: str, hard: bool) -> list[tuple[int, dict]]:
    aff = ((pod["spec"].get("affinity") or {}).get(kind)) or {}
    if hard:
        return [(0, t) for t in aff.get("requiredDuringSchedulingIgnoredDuringExecution") or []]
    return [(int(w.get("weight", 1)), w.get("podAffinityTerm") or {})
            for w in aff.get("preferredDuringSchedulingIgnoredDuringExecution") or []]


def _domain_has(term: dict, pod: dict, node: dict, nodes_by_name: dict, bound: list[dict]) -> bool:
    """Does a pod matching ``term`` run in ``node``'s topology domain?"""
    key = term.get("topologyKey") or "kubernetes.io/hostname"
    value = (node["metadata"].get("labels") or {}).get(key, node["metadata"]["name"] if key == "kubernetes.io/hostname" else None)
    if value is None:
        return False
    spaces = set(term.get("namespaces") or [pod["metadata"].get("namespace", "default")])
    for o in bound:
        if o["metadata"].get("namespace", "default") not in spaces or o is pod:
            continue
        if not selector_matches(term.get("labelSelector"), o["metadata"].get("labels")):
            continue
        other = nodes_by_name.get(o["spec"].get("nodeName"))
        if other is None:
            continue
        ov = (other["metadata"].get("labels") or {}).get(key, other["metadata"]["name"] if key == "kubernetes.io/hostname" else None)
        if ov == value:
            return True
    return False


def _domain(node: dict, key: str) -> str | None:
    labels = node["metadata"].get("labels") or {}
    return labels.get(key, node["metadata"]["name"] if key == "kubernetes.io/hostname" else None)


def _spread_counts(pod: dict, c: dict, nodes_by_name: dict, bound: list[dict]) -> dict[str, int]:
    """Matching pods per topology domain of the eligible nodes (every domain listed, 0 if empty)."""
    key = c.get("topologyKey") or "kubernetes.io/hostname"
    ns = pod["metadata"].get("namespace", "default")
    counts = {d: 0 for d in (_domain(n, key) for n in nodes_by_name.values()) if d is not None}
    for o in bound:
        if o is pod or o["metadata"].get("namespace", "default") != ns:
            continue
        if not selector_matches(c.get("labelSelector"), o["metadata"].get("labels")):
            continue
        n = nodes_by_name.get(o["spec"].get("nodeName"))
        d = _domain(n, key) if n is not None else None
        if d is not None:
            counts[d] = counts.get(d, 0) + 1
    return counts


def _spread_ok(pod: dict, node: dict, nodes_by_name: dict, bound: list[dict]) -> bool:
    for c in pod["spec"].get("topologySpreadConstraints") or []:
        if c.get("whenUnsatisfiable", "DoNotSchedule") != "DoNotSchedule":
            continue
        counts = _spread_counts(pod, c, nodes_by_name, bound)
        d = _domain(node, c.get("topologyKey") or "kubernetes.io/hostname")
        if d is None or not counts:
            return False  # a node without the key is not a place for this pod
        if counts.get(d, 0) + 1 - min(counts.values()) > int(c.get("maxSkew", 1)):
            return False
    return True


def feasible(pod: dict, node: dict, nodes_by_name: dict, bound: list[dict]) -> str | None:
    """None if ``pod`` may go to ``node``, else why not."""
    if not tolerates(pod, node):
        return "untolerated taint"
    na = ((pod["spec"].get("affinity") or {}).get("nodeAffinity") or {}).get(
        "requiredDuringSchedulingIgnoredDuringExecution") or {}
    terms = na.get("nodeSelectorTerms") or []
    if terms and not any(_term_ok(t, node) for t in terms):
        return "node affinity"
    for _w, t in _pod_terms(pod, "podAffinity", True):
        if not _domain_has(t, pod, node, nodes_by_name, bound):
            return "pod affinity"
    for _w, t in _pod_terms(pod, "podAntiAffinity", True):
        if _domain_has(t, pod, node, nodes_by_name, bound):
            return "pod anti-affinity"
    if pod["spec"].get("topologySpreadConstraints") and not _spread_ok(pod, node, nodes_by_name, bound):
        return "topology spread constraints"
    return None


def score(pod: dict, node: dict, nodes_by_name: dict, bound: list[dict]) -> int:
    s = 0
    for w in ((pod["spec"].get("affinity") or {}).get("nodeAffinity") or {}).get(
            "preferredDuringSchedulingIgnoredDuringExecution") or []:
        if _term_ok(w.get("preference") or {}, node):
            s += int(w.get("weight", 1))
    for w, t in _pod_terms(pod, "podAffinity", False):
        s += w if _domain_has(t, pod, node, nodes_by_name, bound) else 0
    for w, t in _pod_terms(pod, "podAntiAffinity", False):
        s -= w if _domain_has(t, pod, node, nodes_by_name, bound) else 0
    if any(t.get("effect") == "PreferNoSchedule" and not any(_tolerates(x, t) for x in pod["spec"].get("tolerations") or [])
           for t in (node.get("spec") or {}).get("taints") or []):
        s -= 1000
    for c in pod["spec"].get("topologySpreadConstraints") or []:
        if c.get("whenUnsatisfiable") == "ScheduleAnyway":
            d = _domain(node, c.get("topologyKey") or "kubernetes.io/hostname")
            s -= 10 * _spread_counts(pod, c, nodes_by_name, bound).get(d, 0)
    return s
