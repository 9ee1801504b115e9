"""Kustomize: ``kubectl apply -k DIR`` / ``kubectl kustomize DIR`` for the bundled kubectl.

A kustomization (``kustomization.yaml``, ``kustomization.yml`` or ``Kustomization`` in DIR) is
built the way kustomize builds one, for the fields manifests commonly use:

* ``resources`` -- manifest files and other kustomization directories (built first, recursively);
* ``configMapGenerator`` / ``secretGenerator`` (``literals``, ``files``, ``envs``; ``behavior:
  create|merge|replace`` against a base's generator; ``options`` and ``generatorOptions``:
  ``disableNameSuffixHash``, ``labels``, ``annotations``) -- generated names get a content-hash
  suffix (``-<10 chars>``), and every reference to them in pod templates (``envFrom``,
  ``valueFrom``, ``volumes``, ``imagePullSecrets``) is rewritten to the hashed name, so a changed
  ConfigMap rolls the Deployment that uses it;
* ``namespace``, ``namePrefix``, ``nameSuffix`` (references to renamed ConfigMaps/Secrets/
  ServiceAccounts/PVCs/Services in pod templates and Ingress backends follow);
* ``commonLabels`` (also selectors and pod templates) and ``labels`` (``pairs``,
  ``includeSelectors``, ``includeTemplates``), ``commonAnnotations``;
* ``images`` (``newName``, ``newTag``, ``digest``), ``replicas``;
* ``patches`` (``path`` or inline ``patch``, strategic merge or JSON 6902, with a ``target``
  selector by group/version/kind/name/namespace/labelSelector), ``patchesStrategicMerge`` and
  ``patchesJson6902``.

The hash suffix is this module's own (sha256 of the canonical JSON), not kustomize's exact
encoding: parity of generated names with the kustomize binary is unpinned.
"""
from __future__ import annotations

import copy
import hashlib
import json
import re
from pathlib import Path

from .utils import yamlio

_FILES = ("kustomization.yaml", "kustomization.yml", "Kustomization")
_CLUSTER_KINDS = {"Namespace", "Node", "ClusterRole", "ClusterRoleBinding", "CustomResourceDefinition",
                  "PriorityClass", "MutatingWebhookConfiguration", "ValidatingWebhookConfiguration",
                  "PersistentVolume", "StorageClass"}
_WORKLOADS = {"Deployment", "StatefulSet", "DaemonSet", "ReplicaSet", "Job", "CronJob", "Pod"}


class KustomizeError(Exception):
    pass


def _read(path: Path) -> list[dict]:
    docs = [d for d in yamlio.load_all(path.read_text()) if d]
    out = []
    for d in docs:
        out += d.get("items", []) if d.get("kind") == "List" else [d]
    return out


def _kfile(d: Path) -> Path:
    for n in _FILES:
        if (d / n).is_file():
            return d / n
    raise KustomizeError(f"no kustomization file ({', '.join(_FILES)}) in {d}")


def _pod_spec(obj: dict) -> dict | None:
    kind, spec = obj.get("kind"), obj.get("spec") or {}
    if kind == "Pod":
        return spec
    if kind == "CronJob":
        return (((spec.get("jobTemplate") or {}).get("spec") or {}).get("template") or {}).get("spec")
    if kind in _WORKLOADS:
        return (spec.get("template") or {}).get("spec")
    return None


def _template_meta(obj: dict) -> dict | None:
    """The pod template's metadata of a workload (None for other kinds)."""
    spec = obj.get("spec") or {}
    if obj.get("kind") == "CronJob":
        jt = spec.get("jobTemplate")
        return jt.setdefault("spec", {}).setdefault("template", {}).setdefault("metadata", {}) if jt else None
    if obj.get("kind") in _WORKLOADS - {"Pod"} and "template" in spec:
        return spec["template"].setdefault("metadata", {})
    return None


def _containers(ps: dict) -> list[dict]:
    return (ps.get("containers") or []) + (ps.get("initContainers") or [])


# ---- name references ----------------------------------------------------------------------------
def _rename_refs(objs: list[dict], kind: str, old: str, new: str, ns: str | None) -> None:
    """Point every reference to ``kind``/``old`` (in namespace ``ns``) at ``new``."""
    for o in objs:
        if ns is not None and (o.get("metadata") or {}).get("namespace") not in (None, ns):
            continue
        ps = _pod_spec(o)
        if ps is not None:
            for c in _containers(ps):
                for ef in c.get("envFrom") or []:
                    key = "configMapRef" if kind == "ConfigMap" else "secretRef" if kind == "Secret" else None
                    if key and (ef.get(key) or {}).get("name") == old:
                        ef[key]["name"] = new
                for e in c.get("env") or []:
                    vf = e.get("valueFrom") or {}
                    key = "configMapKeyRef" if kind == "ConfigMap" else "secretKeyRef" if kind == "Secret" else None
                    if key and (vf.get(key) or {}).get("name") == old:
                        vf[key]["name"] = new
            for v in ps.get("volumes") or []:
                if kind == "ConfigMap" and (v.get("configMap") or {}).get("name") == old:
                    v["configMap"]["name"] = new
                if kind == "Secret" and (v.get("secret") or {}).get("secretName") == old:
                    v["secret"]["secretName"] = new
                if kind == "PersistentVolumeClaim" and (v.get("persistentVolumeClaim") or {}).get("claimName") == old:
                    v["persistentVolumeClaim"]["claimName"] = new
                for src in (v.get("projected") or {}).get("sources") or []:
                    for k, f in (("configMap", "ConfigMap"), ("secret", "Secret")):
                        if kind == f and (src.get(k) or {}).get("name") == old:
                            src[k]["name"] = new
            if kind == "Secret":
                for s in ps.get("imagePullSecrets") or []:
                    if s.get("name") == old:
                        s["name"] = new
            if kind == "ServiceAccount" and ps.get("serviceAccountName") == old:
                ps["serviceAccountName"] = new
        if kind == "Service" and o.get("kind") == "Ingress":
            def fix(b):
                svc = (b or {}).get("service") or {}
                if svc.get("name") == old:
                    svc["name"] = new
            spec = o.get("spec") or {}
            fix(spec.get("defaultBackend"))
            for r in spec.get("rules") or []:
                for p in ((r.get("http") or {}).get("paths")) or []:
                    fix(p.get("backend"))
        if kind == "Service" and o.get("kind") == "StatefulSet" and (o.get("spec") or {}).get("serviceName") == old:
            o["spec"]["serviceName"] = new
        if kind == "ServiceAccount" and o.get("kind") in ("RoleBinding", "ClusterRoleBinding"):
            for s in o.get("subjects") or []:
                if s.get("kind") == "ServiceAccount" and s.get("name") == old:
                    s["name"] = new


# ---- generators ---------------------------------------------------------------------------------
def _env_file(path: Path) -> dict[str, str]:
    out = {}
    for line in path.read_text().splitlines():
        line = line.strip()
        if line and not line.startswith("#"):
            k, _, v = line.partition("=")
            out[k.strip()] = v
    return out


def _gen_data(g: dict, base: Path) -> dict[str, str]:
    data: dict[str, str] = {}
    for kv in g.get("literals") or []:
        k, _, v = str(kv).partition("=")
        data[k] = v
    for f in g.get("files") or []:
        k, _, p = str(f).partition("=") if "=" in str(f) else (Path(str(f)).name, "", str(f))
        data[k] = (base / p).read_text()
    for e in g.get("envs") or ([g["env"]] if g.get("env") else []):
        data.update(_env_file(base / e))
    return data


def _hash(obj: dict) -> str:
    canon = json.dumps({k: obj.get(k) for k in ("kind", "data", "type")}, sort_keys=True, separators=(",", ":"))
    h = hashlib.sha256(canon.encode()).hexdigest()
    return "".join(c if c not in "aeiou013" else "bcdfghjk"[int(c, 16) % 8] for c in h[:10])


def _generate(kdoc: dict, base: Path, objs: list[dict]) -> None:
    import base64

    gopts = kdoc.get("generatorOptions") or {}
    for kind, key in (("ConfigMap", "configMapGenerator"), ("Secret", "secretGenerator")):
        for g in kdoc.get(key) or []:
            data = _gen_data(g, base)
            opts = {**gopts, **(g.get("options") or {})}
            ns = g.get("namespace")
            behavior = g.get("behavior", "create")
            existing = next((o for o in objs if o.get("kind") == kind and o.get("_kgen") == g["name"]
                             and (o["metadata"].get("namespace") == ns or ns is None)), None)
            if behavior in ("merge", "replace"):
                if existing is None:
                    raise KustomizeError(f"{key} {g['name']}: behavior {behavior} but no base generator to {behavior}")
                old = existing.get("_kraw") or {}
                if kind == "Secret":
                    old = {k: base64.b64decode(v).decode() for k, v in old.items()}
                data = {**old, **data} if behavior == "merge" else data
                objs.remove(existing)
                prev = existing["metadata"]["name"]  # what the base's references point at
            elif existing is not None:
                raise KustomizeError(f"{key} {g['name']}: already generated by a base (use behavior: merge|replace)")
            else:
                prev = None
            md = {"name": g["name"], **({"namespace": ns} if ns else {})}
            if opts.get("labels"):
                md["labels"] = dict(opts["labels"])
            if opts.get("annotations"):
                md["annotations"] = dict(opts["annotations"])
            o = {"apiVersion": "v1", "kind": kind, "metadata": md}
            if kind == "Secret":
                o["type"] = g.get("type", "Opaque")
                o["data"] = {k: base64.b64encode(v.encode()).decode() for k, v in data.items()}
            else:
                o["data"] = data
            o["_kgen"] = g["name"]
            o["_kraw"] = o["data"]
            o["_khash"] = not opts.get("disableNameSuffixHash")
            if prev and prev != g["name"]:
                o["_kprev"] = prev
            objs.append(o)


# ---- transformers -------------------------------------------------------------------------------
def _match_target(o: dict, t: dict | None) -> bool:
    if not t:
        return True
    gv = o.get("apiVersion", "")
    group, _, version = gv.rpartition("/")
    for f, v in (("kind", o.get("kind")), ("name", (o.get("metadata") or {}).get("name")),
                 ("namespace", (o.get("metadata") or {}).get("namespace")), ("group", group), ("version", version)):
        want = t.get(f)
        if want is not None and not re.fullmatch(str(want), str(v or "")):
            return False
    if t.get("labelSelector"):
        labels = (o.get("metadata") or {}).get("labels") or {}
        for term in str(t["labelSelector"]).split(","):
            k, _, v = term.partition("=")
            if labels.get(k.strip()) != v.strip():
                return False
    return True


def _apply_patch(objs: list[dict], patch, target: dict | None) -> None:
    from .controlplane import k8s_wire

    if isinstance(patch, list):  # JSON 6902
        if not target:
            raise KustomizeError("a JSON 6902 patch needs a target")
        hit = False
        for i, o in enumerate(objs):
            if _match_target(o, target):
                keep = {k: v for k, v in o.items() if k.startswith("_")}
                objs[i] = {**k8s_wire.json_patch({k: v for k, v in o.items() if not k.startswith("_")}, patch), **keep}
                hit = True
        if not hit:
            raise KustomizeError(f"patch target {target} matches no resource")
        return
    tgt = target or {"kind": patch.get("kind"), "name": (patch.get("metadata") or {}).get("name")}
    hit = False
    for i, o in enumerate(objs):
        if _match_target(o, tgt):
            keep = {k: v for k, v in o.items() if k.startswith("_")}
            body = copy.deepcopy(patch)
            if target:  # a patch with a target applies whatever its own name says
                body.setdefault("metadata", {}).pop("name", None)
            objs[i] = {**k8s_wire.strategic_merge({k: v for k, v in o.items() if not k.startswith("_")}, body), **keep}
            hit = True
    if not hit:
        raise KustomizeError(f"patch target {tgt} matches no resource")


def _load_patch(p: dict | str, base: Path):
    text = (base / p["path"]).read_text() if isinstance(p, dict) and p.get("path") else (
        p.get("patch") if isinstance(p, dict) else (base / p).read_text())
    docs = [d for d in yamlio.load_all(text) if d is not None]
    if len(docs) == 1:
        return docs[0]
    if not docs:
        raise KustomizeError("an empty patch")
    return docs


def _add_labels(o: dict, labels: dict, selectors: bool, templates: bool) -> None:
    o.setdefault("metadata", {}).setdefault("labels", {}).update(labels)
    kind = o.get("kind")
    if selectors and "spec" in o:
        spec = o["spec"]
        if kind == "Service":
            spec.setdefault("selector", {}).update(labels)
        elif kind in ("Deployment", "StatefulSet", "DaemonSet", "ReplicaSet", "PodDisruptionBudget"):
            spec.setdefault("selector", {}).setdefault("matchLabels", {}).update(labels)
    if templates:
        tm = _template_meta(o)
        if tm is not None:
            tm.setdefault("labels", {}).update(labels)


def build(directory: str | Path) -> list[dict]:
    """The objects of the kustomization in ``directory``, ready to apply."""
    objs = _build(Path(directory), set())
    out = []
    for o in objs:
        out.append({k: v for k, v in o.items() if not k.startswith("_")})
    return out


def _build(d: Path, seen: set) -> list[dict]:
    d = d.resolve()
    if d in seen:
        raise KustomizeError(f"cycle: {d} includes itself")
    seen = seen | {d}
    kdoc = yamlio.load(_kfile(d).read_text()) or {}
    objs: list[dict] = []
    for r in kdoc.get("resources") or kdoc.get("bases") or []:
        p = (d / r)
        if p.is_dir():
            objs += _build(p, seen)
        elif p.is_file():
            objs += [copy.deepcopy(x) for x in _read(p)]
        else:
            raise KustomizeError(f"resource {r!r} not found in {d} (remote resources are not fetched)")
    _generate(kdoc, d, objs)
    for p in kdoc.get("patchesStrategicMerge") or []:
        _apply_patch(objs, _load_patch(p, d), None)
    for p in kdoc.get("patchesJson6902") or []:
        _apply_patch(objs, _load_patch(p, d), p.get("target"))
    for p in kdoc.get("patches") or []:
        _apply_patch(objs, _load_patch(p, d), p.get("target"))
    # names: generated objects get their hash, then prefix/suffix; references follow
    prefix, suffix = kdoc.get("namePrefix", ""), kdoc.get("nameSuffix", "")
    renames = []
    for o in objs:
        md = o.setdefault("metadata", {})
        old = md.get("name", "")
        new = old
        if o.get("kind") not in ("Namespace", "CustomResourceDefinition"):
            new = f"{prefix}{old}{suffix}" if (prefix or suffix) else old
        if o.pop("_khash", False):
            new = f"{new}-{_hash(o)}"
        if new != old:
            md["name"] = new
            renames.append((o.get("kind"), old, new, md.get("namespace")))
        prev = o.pop("_kprev", None)
        if prev and prev != new:  # a merged/replaced base generator: the base's references move too
            renames.append((o.get("kind"), prev, new, md.get("namespace")))
    for kind, old, new, ns in renames:
        _rename_refs(objs, kind, old, new, ns)
    ns = kdoc.get("namespace")
    if ns:
        for o in objs:
            if o.get("kind") not in _CLUSTER_KINDS:
                o.setdefault("metadata", {})["namespace"] = ns
            if o.get("kind") in ("RoleBinding", "ClusterRoleBinding"):
                for s in o.get("subjects") or []:
                    if s.get("kind") == "ServiceAccount":
                        s["namespace"] = ns
    if kdoc.get("commonLabels"):
        for o in objs:
            _add_labels(o, {k: str(v) for k, v in kdoc["commonLabels"].items()}, True, True)
    for spec in kdoc.get("labels") or []:
        for o in objs:
            _add_labels(o, {k: str(v) for k, v in (spec.get("pairs") or {}).items()}, bool(spec.get("includeSelectors")),
                        bool(spec.get("includeTemplates") or spec.get("includeSelectors")))
    if kdoc.get("commonAnnotations"):
        ann = {k: str(v) for k, v in kdoc["commonAnnotations"].items()}
        for o in objs:
            o.setdefault("metadata", {}).setdefault("annotations", {}).update(ann)
            tm = _template_meta(o)
            if tm is not None:
                tm.setdefault("annotations", {}).update(ann)
    for img in kdoc.get("images") or []:
        for o in objs:
            ps = _pod_spec(o)
            for c in _containers(ps or {}):
                ref = c.get("image", "")
                name = re.split(r"[@]", ref)[0]
                name = name.rsplit(":", 1)[0] if ":" in name.rsplit("/", 1)[-1] else name
                if name != img.get("name"):
                    continue
                new = img.get("newName", name)
                if img.get("digest"):
                    new += "@" + img["digest"]
                elif img.get("newTag"):
                    new += ":" + str(img["newTag"])
                elif ref != name:
                    new += ref[len(name):]
                c["image"] = new
    for rep in kdoc.get("replicas") or []:
        for o in objs:
            if (o.get("metadata") or {}).get("name") in (rep.get("name"), f"{prefix}{rep.get('name')}{suffix}") \
                    and o.get("kind") in ("Deployment", "StatefulSet", "ReplicaSet"):
                o.setdefault("spec", {})["replicas"] = int(rep["count"])
    return objs
