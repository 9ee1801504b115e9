"""Pod volumes on a node (the kubelet's volume manager, for the volume types served here):

* ``emptyDir``        -- a directory of the pod's own (``<pod dir>/volumes/<name>``), gone with it
* ``configMap``       -- the ConfigMap's keys as files (``data`` and ``binaryData``; ``items``
                         picks and renames keys; ``defaultMode``/item ``mode``; ``optional``)
* ``secret``          -- the same for a Secret (``secretName``), decoded, mode 0644 by default
* ``downwardAPI``     -- ``fieldRef`` items as files (metadata.name, labels, annotations, ...)
* ``hostPath``        -- a node path (``DirectoryOrCreate``/``FileOrCreate`` create it)
* ``persistentVolumeClaim`` -- a node-local directory per claim (``<node dir>/volumes/<ns>_<claim>``),
                         on the node the scheduler bound the claim to (``volume.kubernetes.io/
                         selected-node``); it outlives pods, so a StatefulSet's ordinal finds its
                         data again

``materialize`` returns the mounts of one container: (source path, mountPath, read-only), with
``subPath`` applied. Image pods get them bind-mounted at ``mountPath`` (tk8s-container
``--bind``/``--bind-ro``); process pods share the host's file system, so they get each volume's
directory in ``TK8S_VOLUME_<NAME>`` instead.
"""
from __future__ import annotations

import base64
import os
import re
from pathlib import Path
from typing import Callable

from ..utils.k8senv import field_path


class VolumeError(Exception):
    """A volume cannot be set up yet (a missing ConfigMap/Secret/claim): the pod waits."""


def _safe_rel(p: str) -> str:
    parts = [x for x in Path(p).parts if x not in ("", ".")]
    if not parts or ".." in parts or Path(p).is_absolute():
        raise VolumeError(f"path {p!r} must be relative and stay inside the volume")
    return str(Path(*parts))


def _write_files(root: Path, files: dict[str, bytes], modes: dict[str, int]) -> None:
    root.mkdir(parents=True, exist_ok=True)
    for rel, data in files.items():
        dst = root / _safe_rel(rel)
        dst.parent.mkdir(parents=True, exist_ok=True)
        tmp = dst.with_name(f".{dst.name}.tmp")
        tmp.write_bytes(data)
        os.chmod(tmp, modes.get(rel, 0o644))
        os.replace(tmp, dst)


def _key_files(vol: dict, data: dict[str, bytes], what: str) -> tuple[dict[str, bytes], dict[str, int]]:
    default = int(vol.get("defaultMode", 0o644))
    files, modes = {}, {}
    if vol.get("items"):
        for it in vol["items"]:
            if it["key"] not in data:
                if vol.get("optional"):
                    continue
                raise VolumeError(f"{what}: no key {it['key']!r}")
            files[it.get("path") or it["key"]] = data[it["key"]]
            modes[it.get("path") or it["key"]] = int(it.get("mode", default))
    else:
        for k, v in data.items():
            files[k], modes[k] = v, default
    return files, modes


def env_name(volume: str) -> str:
    return "TK8S_VOLUME_" + re.sub(r"[^A-Z0-9_]", "_", volume.upper())


def volume_dirs(pod: dict, pod_dir: Path, node_dir: Path, fetch: Callable[[str, str, str], dict | None],
                pod_ip: str = "", host_ip: str = "") -> dict[str, tuple[Path, bool]]:
    """Set up every volume of the pod: name -> (path on the node, read-only by nature)."""
    ns = pod["metadata"]["namespace"]
    out: dict[str, tuple[Path, bool]] = {}
    for vol in pod["spec"].get("volumes") or []:
        name = vol.get("name", "")
        own = pod_dir / "volumes" / name
        if "emptyDir" in vol:
            own.mkdir(parents=True, exist_ok=True)
            out[name] = (own, False)
        elif "hostPath" in vol:
            hp = vol["hostPath"]
            p = Path(hp.get("path", ""))
            kind = hp.get("type", "")
            if kind == "DirectoryOrCreate":
                p.mkdir(parents=True, exist_ok=True)
            elif kind == "FileOrCreate" and not p.exists():
                p.parent.mkdir(parents=True, exist_ok=True)
                p.touch()
            elif kind in ("Directory", "File") and not p.exists():
                raise VolumeError(f"hostPath {p} does not exist")
            out[name] = (p, False)
        elif "configMap" in vol or "secret" in vol:
            is_secret = "secret" in vol
            src = vol["secret"] if is_secret else vol["configMap"]
            obj_name = src.get("secretName") if is_secret else src.get("name")
            kind = "secrets" if is_secret else "configmaps"
            o = fetch(kind, ns, obj_name)
            if o is None:
                if not src.get("optional"):
                    raise VolumeError(f'{kind[:-1]} "{obj_name}" not found')
                o = {}
            if is_secret:
                data = {k: base64.b64decode(v) for k, v in (o.get("data") or {}).items()}
            else:
                data = {k: str(v).encode() for k, v in (o.get("data") or {}).items()}
                data.update({k: base64.b64decode(v) for k, v in (o.get("binaryData") or {}).items()})
            files, modes = _key_files(src, data, f"{kind[:-1]} {obj_name}")
            _write_files(own, files, modes)
            out[name] = (own, True)
        elif "downwardAPI" in vol:
            files, modes = {}, {}
            for it in vol["downwardAPI"].get("items") or []:
                ref = (it.get("fieldRef") or {}).get("fieldPath", "")
                md = pod["metadata"]
                if ref in ("metadata.labels", "metadata.annotations"):
                    d = md.get(ref.split(".")[1]) or {}
                    text = "".join(f'{k}="{v}"\n' for k, v in sorted(d.items()))
                else:
                    try:
                        text = field_path(pod, ref, pod_ip, host_ip)
                    except ValueError as e:
                        raise VolumeError(str(e)) from e
                files[it["path"]] = text.encode()
                modes[it["path"]] = int(it.get("mode", vol["downwardAPI"].get("defaultMode", 0o644)))
            _write_files(own, files, modes)
            out[name] = (own, True)
        elif "persistentVolumeClaim" in vol:
            claim = vol["persistentVolumeClaim"].get("claimName", "")
            pvc = fetch("persistentvolumeclaims", ns, claim)
            if pvc is None:
                raise VolumeError(f'persistentvolumeclaim "{claim}" not found')
            uid = (pvc.get("metadata") or {}).get("uid", "")[:8]
            d = node_dir / "volumes" / f"{ns}_{claim}-{uid}"
            d.mkdir(parents=True, exist_ok=True)
            out[name] = (d, bool(vol["persistentVolumeClaim"].get("readOnly")))
        else:
            kinds = [k for k in vol if k != "name"]
            raise VolumeError(f"volume {name!r}: type {kinds} is not supported on this node "
                              "(emptyDir, configMap, secret, downwardAPI, hostPath, persistentVolumeClaim)")
    return out


def mounts(container: dict, dirs: dict[str, tuple[Path, bool]]) -> list[tuple[str, str, bool]]:
    """The container's volumeMounts as (source, mountPath, read-only)."""
    out = []
    for m in container.get("volumeMounts") or []:
        name, dst = m.get("name"), m.get("mountPath")
        if name not in dirs:
            raise VolumeError(f"volumeMount {name!r}: no such volume in the pod")
        if not dst or not dst.startswith("/"):
            raise VolumeError(f"volumeMount {name!r}: mountPath must be absolute")
        src, ro = dirs[name]
        if m.get("subPath"):
            src = src / _safe_rel(m["subPath"])
            if not src.exists():
                src.mkdir(parents=True, exist_ok=True)
        out.append((str(src), dst, bool(m.get("readOnly")) or ro))
    return out
