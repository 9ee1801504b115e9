"""Pod volumes on a node (the kubelet's volume manager, for the volume types served here):

* ``emptyDir``        -- a directory of the pod's own (``<pod dir>/volumes/<name>``), gone with it
* ``configMap``       -- the ConfigMap's keys as files (``data`` and ``binaryData``; ``items``
                         picks and renames keys; ``defaultMode``/item ``mode``; ``optional``)
* ``secret``          -- the same for a Secret (``secretName``), decoded, mode 0644 by default
* ``downwardAPI``     -- ``fieldRef`` items as files (metadata.name, labels, annotations, ...)
* ``projected``       -- configMap, secret, downwardAPI and serviceAccountToken sources in one
                         directory
* ``hostPath``        -- a node path (``DirectoryOrCreate``/``FileOrCreate`` create it)
* ``persistentVolumeClaim`` -- a node-local directory per claim (``<node dir>/volumes/<ns>_<claim>``),
                         on the node the scheduler bound the claim to (``volume.kubernetes.io/
                         selected-node``); it outlives pods, so a StatefulSet's ordinal finds its
                         data again

ConfigMap, Secret, downwardAPI and projected volumes are published as the kubelet's atomic writer
does: the files live in a timestamped ``..<time>`` directory, ``..data`` links to the current one
and every top-level entry links through ``..data``, so ``refresh`` (the agent calls it every
``TK8S_VOLUME_SYNC_PERIOD`` s) swaps a changed ConfigMap in with one rename -- a running pod
sees the old set of files or the new one, never a mix. ``subPath`` mounts keep what they got.

``mounts`` returns the mounts of one container: (source path, mountPath, read-only), with
``subPath`` applied. Image pods get them bind-mounted at ``mountPath`` (tk8s-container
``--bind``/``--bind-ro``); process pods share the host's file system, so they get each volume's
directory in ``TK8S_VOLUME_<NAME>`` instead.
"""
from __future__ import annotations

import base64
import os
import re
import time
from pathlib import Path
from collections.abc import Callable  # (not typing: ~1.5-4 ms of every agent zygote's imports)

from ..utils.k8senv import field_path


class VolumeError(Exception):
    """A volume cannot be set up yet (a missing ConfigMap/Secret/claim): the pod waits."""


def _safe_rel(p: str) -> str:
    parts = [x for x in Path(p).parts if x not in ("", ".")]
    if not parts or ".." in parts or Path(p).is_absolute():
        raise VolumeError(f"path {p!r} must be relative and stay inside the volume")
    return str(Path(*parts))


def _current(root: Path) -> dict[str, tuple[bytes, int]]:
    """What ``root/..data`` holds now: relative path -> (bytes, mode)."""
    data = root / "..data"
    out = {}
    if data.is_dir():
        for p in data.resolve().rglob("*"):
            if p.is_file():
                out[str(p.relative_to(data.resolve()))] = (p.read_bytes(), p.stat().st_mode & 0o777)
    return out


def _write_files(root: Path, files: dict[str, bytes], modes: dict[str, int]) -> bool:
    """Publish ``files`` under ``root`` atomically (see the module doc); False if nothing changed."""
    want = {_safe_rel(rel): (data, modes.get(rel, 0o644)) for rel, data in files.items()}
    root.mkdir(parents=True, exist_ok=True)
    if (root / "..data").exists() and _current(root) == want:
        return False
    ts = root / f"..{time.strftime('%Y_%m_%d_%H_%M_%S', time.gmtime())}.{time.time_ns() % 10**9:09d}"
    ts.mkdir()
    for rel, (data, mode) in want.items():
        dst = ts / rel
        dst.parent.mkdir(parents=True, exist_ok=True)
        dst.write_bytes(data)
        os.chmod(dst, mode)
    tmp = root / "..data_tmp"
    tmp.unlink(missing_ok=True)
    os.symlink(ts.name, tmp)
    os.replace(tmp, root / "..data")  # the switch: one rename
    tops = {rel.split("/", 1)[0] for rel in want}
    for top in tops:
        link = root / top
        if not link.is_symlink():
            if link.is_file():  # a plain file from before (an older agent): replace it
                link.unlink()
            os.symlink(f"..data/{top}", link)
    for p in root.iterdir():
        if p.name.startswith(".."):
            if p.name not in ("..data", ts.name) and p.is_dir() and not p.is_symlink():
                import shutil  # (lazy: shutil pulls in bz2/lzma, ~4 ms of the agent's start)

                shutil.rmtree(p, ignore_errors=True)
        elif p.is_symlink() and p.name not in tops:
            p.unlink()  # a key that is gone
    return True


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


def _config_files(src: dict, is_secret: bool, ns: str, fetch) -> tuple[dict[str, bytes], dict[str, int]]:
    obj_name = src.get("secretName") if is_secret and "secretName" in src else src.get("name")
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
    return _key_files(src, data, f"{kind[:-1]} {obj_name}")


def _downward_files(pod: dict, src: dict, pod_ip: str, host_ip: str,
                    default: int = 0o644) -> tuple[dict[str, bytes], dict[str, int]]:
    files, modes = {}, {}
    for it in src.get("items") or []:
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
        modes[it["path"]] = int(it.get("mode", src.get("defaultMode", default)))
    return files, modes


def _projected_files(pod: dict, vol: dict, ns: str, fetch, pod_ip: str, host_ip: str):
    """A projected volume's sources merged into one directory (later sources win a clash)."""
    default = int(vol.get("defaultMode", 0o644))
    files, modes = {}, {}
    for s in vol.get("sources") or []:
        if "configMap" in s or "secret" in s:
            sec = "secret" in s
            f, m = _config_files({"defaultMode": default, **(s["secret"] if sec else s["configMap"])}, sec, ns, fetch)
        elif "downwardAPI" in s:
            f, m = _downward_files(pod, s["downwardAPI"], pod_ip, host_ip, default)
        elif "serviceAccountToken" in s:
            sa = pod["spec"].get("serviceAccountName") or pod["spec"].get("serviceAccount") or "default"
            tok = fetch("secrets", ns, f"{sa}-token")
            if tok is None:
                raise VolumeError(f'serviceaccount "{sa}" has no token yet')
            path = s["serviceAccountToken"].get("path", "token")
            f, m = {path: base64.b64decode((tok.get("data") or {}).get("token", ""))}, {path: 0o600}
        else:
            raise VolumeError(f"projected source {sorted(s)} is not supported")
        files.update(f)
        modes.update(m)
    return files, modes


_DYNAMIC = ("configMap", "secret", "downwardAPI", "projected")


def _render(pod: dict, vol: dict, fetch, pod_ip: str, host_ip: str) -> tuple[dict[str, bytes], dict[str, int]]:
    ns = pod["metadata"]["namespace"]
    if "configMap" in vol or "secret" in vol:
        return _config_files(vol["secret"] if "secret" in vol else vol["configMap"], "secret" in vol, ns, fetch)
    if "downwardAPI" in vol:
        return _downward_files(pod, vol["downwardAPI"], pod_ip, host_ip)
    return _projected_files(pod, vol["projected"], ns, fetch, pod_ip, host_ip)


def refresh(pod: dict, pod_dir: Path, fetch: Callable[[str, str, str], dict | None], pod_ip: str = "",
            host_ip: str = "") -> list[str]:
    """Re-publish the pod's ConfigMap/Secret/downwardAPI/projected volumes; the names that changed.
    A source that is gone (or unreachable) leaves the volume as it is, as the kubelet does."""
    changed = []
    for vol in pod["spec"].get("volumes") or []:
        if not any(k in vol for k in _DYNAMIC):
            continue
        try:
            name = _vol_name(vol)
            files, modes = _render(pod, vol, fetch, pod_ip, host_ip)
        except VolumeError:
            continue
        if _write_files(pod_dir / "volumes" / name, files, modes):
            changed.append(name)
    return changed


def has_dynamic(pod: dict) -> bool:
    return any(any(k in v for k in _DYNAMIC) for v in pod["spec"].get("volumes") or [])


def _vol_name(vol: dict) -> str:
    """A volume's name, refused unless it is one path component (the API admits DNS labels only;
    this holds even against an object that reached the node some other way)."""
    name = str(vol.get("name", ""))
    if not name or "/" in name or name in (".", "..") or "\0" in name:
        raise VolumeError(f"volume name {name!r} is not a DNS label")
    return name


def volume_dirs(pod: dict, pod_dir: Path, node_dir: Path, fetch: Callable[[str, str, str], dict | None],
                pod_ip: str = "", host_ip: str = "") -> dict[str, tuple[Path, bool]]:
    """Set up every volume of the pod: name -> (path on the node, read-only by nature)."""
    ns = pod["metadata"]["namespace"]
    out: dict[str, tuple[Path, bool]] = {}
    for vol in pod["spec"].get("volumes") or []:
        name = _vol_name(vol)
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
        elif any(k in vol for k in _DYNAMIC):
            files, modes = _render(pod, vol, fetch, pod_ip, host_ip)
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
                              "(emptyDir, configMap, secret, downwardAPI, projected, hostPath, persistentVolumeClaim)")
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
