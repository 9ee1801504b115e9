"""The node's image store: container images loaded from files, unpacked once, run by
``tk8s-container`` (native/tools/tk8s_container.cpp).

The reference's nodes pulled Docker images (rancher/server, rancher/agent, the Kubernetes
stack, the demo apps; ansible/roles/*/tasks/main.yml, docs/detailed.md:261-370). A tk8s node has
no registry to pull from (the GPU hosts are offline), so images come from files, the way an
air-gapped node is fed: ``./tk8s image load FILE`` takes a ``docker save`` tarball or an OCI image
layout (directory or tar), checks every blob against its sha256, and keeps them in a
content-addressed store (``$TK8S_IMAGE_STORE``, default ``$XDG_STATE_HOME/tk8s/images``):

    blobs/sha256/<hex>         layers (tar, tar+gzip), configs, manifests
    refs.json                  {"docker.io/library/nginx:1.27": {"manifest": <digest>, ...}}
    rootfs/<manifest hex>/     the layers applied in order (whiteouts honoured), built once

A pod whose container names a loaded image runs in that image's root file system: the image's
ENTRYPOINT/CMD/Env/WorkingDir, with Kubernetes' rules (``command`` replaces the entrypoint,
``args`` the cmd). Images the store does not hold fall back to the built-in apps
(tritonk8ssupervisor_amd/apps) for the reference's demo names, else the pod fails with
ErrImageNeverPull.
"""
from __future__ import annotations

import gzip
import hashlib
import io
import json
import os
import shutil
import tarfile
import tempfile
from pathlib import Path

from ..utils.fsutil import atomic_write_json, file_lock, read_json

DEFAULT_REGISTRY = "docker.io"
OCI_MANIFEST = "application/vnd.oci.image.manifest.v1+json"
OCI_INDEX = "application/vnd.oci.image.index.v1+json"
REF_ANNOTATION = "org.opencontainers.image.ref.name"


class ImageError(RuntimeError):
    pass


def store_dir() -> Path:
    d = os.environ.get("TK8S_IMAGE_STORE")
    if d:
        return Path(d)
    from ..utils.pcache import state_home  # (not ~/.cache: pods write there, agent._jail_layers)

    return Path(state_home()) / "images"


def normalize(ref: str) -> str:
    """Docker's reference rules: ``nginx`` -> ``docker.io/library/nginx:latest``, ``me/app:1`` ->
    ``docker.io/me/app:1``; a first component with a dot, a colon or ``localhost`` is a registry."""
    ref = ref.strip()
    digest = ""
    if "@" in ref:
        ref, digest = ref.split("@", 1)
        digest = "@" + digest
    first, _, rest = ref.partition("/")
    if not rest or not ("." in first or ":" in first or first == "localhost"):
        name = ref if rest else f"library/{ref}"
        registry = DEFAULT_REGISTRY
    else:
        registry, name = first, rest
    if ":" not in name.rsplit("/", 1)[-1] and not digest:
        name += ":latest"
    return f"{registry}/{name}{digest}"


def _sha256_file(path: Path) -> str:
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


class ImageStore:
    def __init__(self, root: str | os.PathLike | None = None):
        self.root = Path(root) if root else store_dir()
        self.blobs = self.root / "blobs" / "sha256"
        self.refs_file = self.root / "refs.json"
        self.lock = self.root / "store.lock"

    # ---- reading ----------------------------------------------------------------------------
    def refs(self) -> dict:
        return read_json(self.refs_file, {}) or {}

    def get(self, ref: str) -> dict | None:
        """The image record of ``ref`` (its normal form or a short alias), or None."""
        refs = self.refs()
        if ref in refs:
            return refs[ref]
        try:
            return refs.get(normalize(ref))
        except Exception:  # noqa: BLE001 - not a reference at all
            return None

    def blob(self, digest: str) -> bytes:
        return (self.blobs / digest.split(":", 1)[-1]).read_bytes()

    def config(self, ref: str) -> dict:
        rec = self.get(ref)
        if rec is None:
            raise ImageError(f"image {ref!r} is not in the store")
        return (json.loads(self.blob(rec["config"])).get("config") or {})

    def list(self) -> list[dict]:
        out = []
        for ref, rec in sorted(self.refs().items()):
            size = sum((self.blobs / d.split(":", 1)[-1]).stat().st_size for d in rec["layers"]
                       if (self.blobs / d.split(":", 1)[-1]).exists())
            out.append({"ref": ref, "manifest": rec["manifest"], "layers": len(rec["layers"]), "size": size})
        return out

    # ---- loading ----------------------------------------------------------------------------
    def _put_blob(self, data_path: Path, want: str | None = None) -> str:
        hexd = _sha256_file(data_path)
        if want and want.split(":", 1)[-1] != hexd:
            raise ImageError(f"blob {want} does not match its content (sha256:{hexd})")
        self.blobs.mkdir(parents=True, exist_ok=True)
        dst = self.blobs / hexd
        if not dst.exists():
            tmp = dst.with_suffix(".tmp")
            shutil.copyfile(data_path, tmp)
            os.replace(tmp, dst)
        return f"sha256:{hexd}"

    def _put_bytes(self, data: bytes) -> str:
        with tempfile.NamedTemporaryFile(dir=self.root, delete=False) as f:
            f.write(data)
        try:
            return self._put_blob(Path(f.name))
        finally:
            os.unlink(f.name)

    def load(self, source: str | os.PathLike, tag: str | None = None) -> list[str]:
        """Load a ``docker save`` tarball or an OCI image layout (directory or tar); returns the
        references it now holds. ``tag`` names an image the file does not name itself."""
        src = Path(source)
        self.root.mkdir(parents=True, exist_ok=True)
        with tempfile.TemporaryDirectory(dir=self.root) as tmp:
            if src.is_dir():
                d = src
            else:
                d = Path(tmp) / "x"
                d.mkdir()
                with tarfile.open(src) as tf:
                    _safe_extract(tf, d)
            with file_lock(self.lock):
                if (d / "index.json").exists() and (d / "oci-layout").exists():
                    loaded = self._load_oci(d, tag)
                elif (d / "manifest.json").exists():
                    loaded = self._load_docker(d, tag)
                else:
                    raise ImageError(f"{source}: neither an OCI image layout nor a docker save archive")
        if not loaded:
            raise ImageError(f"{source}: no image with a name in it (give one with --tag)")
        return loaded

    def _record(self, ref: str, manifest_digest: str, config_digest: str, layers: list[str]) -> None:
        refs = self.refs()
        refs[normalize(ref)] = {"manifest": manifest_digest, "config": config_digest, "layers": layers}
        atomic_write_json(self.refs_file, refs)

    def _load_oci(self, d: Path, tag: str | None) -> list[str]:
        index = json.loads((d / "index.json").read_text())
        out = []

        def blob_path(desc):
            return d / "blobs" / desc["digest"].replace(":", "/", 1)

        def manifests(idx):
            for m in idx.get("manifests", []):
                if m.get("mediaType") == OCI_INDEX:  # nested index: its first linux/amd64 (or only) image
                    sub = json.loads(blob_path(m).read_text())
                    for x in sub.get("manifests", []):
                        plat = x.get("platform") or {}
                        if plat.get("architecture", "amd64") == "amd64" and plat.get("os", "linux") == "linux":
                            yield {**x, "annotations": {**(x.get("annotations") or {}), **(m.get("annotations") or {})}}
                            break
                else:
                    yield m

        for m in manifests(index):
            ref = (m.get("annotations") or {}).get(REF_ANNOTATION) or tag
            if not ref:
                continue
            mdig = self._put_blob(blob_path(m), m["digest"])
            man = json.loads(blob_path(m).read_text())
            cdig = self._put_blob(blob_path(man["config"]), man["config"]["digest"])
            layers = [self._put_blob(blob_path(x), x["digest"]) for x in man.get("layers", [])]
            self._record(ref, mdig, cdig, layers)
            out.append(normalize(ref))
        return out

    def _load_docker(self, d: Path, tag: str | None) -> list[str]:
        out = []
        for ent in json.loads((d / "manifest.json").read_text()):
            cdig = self._put_blob(d / ent["Config"])
            layers = [self._put_blob(d / lp) for lp in ent.get("Layers", [])]
            man = {"schemaVersion": 2, "mediaType": OCI_MANIFEST,
                   "config": {"digest": cdig, "mediaType": "application/vnd.oci.image.config.v1+json"},
                   "layers": [{"digest": x, "mediaType": "application/vnd.oci.image.layer.v1.tar"} for x in layers]}
            mdig = self._put_bytes(json.dumps(man, sort_keys=True).encode())
            for ref in (ent.get("RepoTags") or ([tag] if tag else [])):
                self._record(ref, mdig, cdig, layers)
                out.append(normalize(ref))
        return out

    def remove(self, ref: str) -> bool:
        with file_lock(self.lock):
            refs = self.refs()
            key = ref if ref in refs else normalize(ref)
            if key not in refs:
                return False
            rec = refs.pop(key)
            atomic_write_json(self.refs_file, refs)
            if not any(r["manifest"] == rec["manifest"] for r in refs.values()):
                shutil.rmtree(self.root / "rootfs" / rec["manifest"].split(":", 1)[-1], ignore_errors=True)
        return True

    # ---- running ----------------------------------------------------------------------------
    def rootfs(self, ref: str) -> Path:
        """The image's root file system: its layers applied in order, once per manifest."""
        rec = self.get(ref)
        if rec is None:
            raise ImageError(f"image {ref!r} is not in the store")
        dst = self.root / "rootfs" / rec["manifest"].split(":", 1)[-1]
        if (dst / ".tk8s-complete").exists():
            return dst
        with file_lock(self.lock):
            if (dst / ".tk8s-complete").exists():
                return dst
            tmp = dst.with_name(dst.name + ".partial")
            shutil.rmtree(tmp, ignore_errors=True)
            tmp.mkdir(parents=True)
            for layer in rec["layers"]:
                apply_layer(self.blobs / layer.split(":", 1)[-1], tmp)
            (tmp / ".tk8s-complete").write_text(rec["manifest"] + "\n")
            shutil.rmtree(dst, ignore_errors=True)
            os.replace(tmp, dst)
        return dst

    def container_argv(self, ref: str, command: list[str] | None, args: list[str] | None) -> tuple[list[str], dict, str]:
        """(argv, image env, working dir) by Kubernetes' rules: ``command`` replaces ENTRYPOINT
        (and drops CMD), ``args`` replaces CMD."""
        cfg = self.config(ref)
        entry, cmd = list(cfg.get("Entrypoint") or []), list(cfg.get("Cmd") or [])
        if command:
            argv = list(command) + list(args or [])
        else:
            argv = entry + (list(args) if args else cmd)
        env = dict(e.split("=", 1) for e in cfg.get("Env") or [] if "=" in e)
        return argv, env, cfg.get("WorkingDir") or "/"


def _open_layer(path: Path):
    with open(path, "rb") as f:
        magic = f.read(4)
    if magic[:2] == b"\x1f\x8b":
        return tarfile.open(fileobj=gzip.open(path), mode="r|")
    if magic == b"\x28\xb5\x2f\xfd":
        raise ImageError(f"layer {path.name}: zstd-compressed layers are not supported (re-save the image with gzip)")
    return tarfile.open(path, mode="r|")


def _safe_name(name: str) -> str | None:
    parts = [p for p in name.split("/") if p not in ("", ".")]
    if any(p == ".." for p in parts):
        return None
    return "/".join(parts)


def apply_layer(layer: Path, root: Path) -> None:
    """Apply one image layer onto ``root``: OCI whiteouts (``.wh.<name>`` deletes a lower entry,
    ``.wh..wh..opq`` empties the directory), no path may leave ``root`` (``..`` entries, links
    through a symlink), device nodes are skipped (they come from the host's /dev at run time),
    set-id bits are dropped."""
    root = root.resolve()
    with _open_layer(layer) as tf:
        for m in tf:
            name = _safe_name(m.name)
            if not name:
                continue
            base = os.path.basename(name)
            parent = root / os.path.dirname(name)
            if not _inside(root, parent):
                continue
            if base == ".wh..wh..opq":
                if parent.is_dir():
                    for child in parent.iterdir():
                        _remove(child)
                continue
            if base.startswith(".wh."):
                _remove(parent / base[4:])
                continue
            if m.ischr() or m.isblk() or m.isfifo():
                continue
            target = root / name
            if not _inside(root, target.parent):
                continue
            parent.mkdir(parents=True, exist_ok=True)
            if target.is_symlink() or (target.exists() and not (m.isdir() and target.is_dir())):
                _remove(target)
            if m.isdir():
                target.mkdir(exist_ok=True)
                os.chmod(target, (m.mode & 0o777) | 0o700)
            elif m.issym():
                os.symlink(m.linkname, target)
            elif m.islnk():
                # a hard link names a file of the image: never a symlink (os.link would follow it out
                # of the root -- ADVICE r3: `s -> /etc/shadow` then `h` hardlinked to `s`), and the
                # link itself must resolve inside the root
                src = _safe_name(m.linkname)
                sp = root / src if src else None
                if (sp is not None and not sp.is_symlink() and sp.is_file() and _inside(root, sp)
                        and _inside(root, sp.parent)):
                    os.link(sp, target, follow_symlinks=False)
            elif m.isreg():
                f = tf.extractfile(m)
                with open(target, "wb") as out:
                    shutil.copyfileobj(f, out)
                os.chmod(target, m.mode & 0o777)


def _inside(root: Path, p: Path) -> bool:
    try:
        return os.path.realpath(p) == str(root) or os.path.realpath(p).startswith(str(root) + os.sep)
    except OSError:
        return False


def _remove(p: Path) -> None:
    if p.is_symlink() or p.is_file():
        p.unlink(missing_ok=True)
    elif p.is_dir():
        shutil.rmtree(p, ignore_errors=True)


def _safe_extract(tf: tarfile.TarFile, dest: Path) -> None:
    """Extract an image archive (not a layer) refusing anything outside ``dest``."""
    for m in tf.getmembers():
        name = _safe_name(m.name)
        if name is None or m.issym() or m.islnk() or m.isdev():
            continue
        m.name = name
        tf.extract(m, dest)


def write_docker_archive(path: str | os.PathLike, ref: str, layers: list[dict[str, bytes]], config: dict) -> None:
    """A ``docker save`` archive of one image from in-memory layers ({path in image: content};
    a path ending in ``/`` is a directory, ``.wh.`` names are whiteouts, a ("symlink"|"hardlink",
    target) tuple a link). Tests and air-gapped
    hand-offs build images with it; content is stored uncompressed."""
    with tarfile.open(path, "w") as out:
        names = []
        for i, files in enumerate(layers):
            buf = io.BytesIO()
            with tarfile.open(fileobj=buf, mode="w") as lt:
                for p, data in files.items():
                    ti = tarfile.TarInfo(p.rstrip("/"))
                    if isinstance(data, tuple):  # ("symlink" | "hardlink", target)
                        ti.type = tarfile.SYMTYPE if data[0] == "symlink" else tarfile.LNKTYPE
                        ti.linkname = data[1]
                        lt.addfile(ti)
                    elif p.endswith("/"):
                        ti.type, ti.mode = tarfile.DIRTYPE, 0o755
                        lt.addfile(ti)
                    else:
                        ti.size, ti.mode = len(data), (0o755 if data.startswith(b"#!") or data[:4] == b"\x7fELF" else 0o644)
                        lt.addfile(ti, io.BytesIO(data))
            raw = buf.getvalue()
            name = f"layer{i}/layer.tar"
            ti = tarfile.TarInfo(name)
            ti.size = len(raw)
            out.addfile(ti, io.BytesIO(raw))
            names.append(name)
        cfg = json.dumps({"architecture": "amd64", "os": "linux", "config": config,
                          "rootfs": {"type": "layers", "diff_ids": []}}).encode()
        ti = tarfile.TarInfo("config.json")
        ti.size = len(cfg)
        out.addfile(ti, io.BytesIO(cfg))
        man = json.dumps([{"Config": "config.json", "RepoTags": [ref], "Layers": names}]).encode()
        ti = tarfile.TarInfo("manifest.json")
        ti.size = len(man)
        out.addfile(ti, io.BytesIO(man))
