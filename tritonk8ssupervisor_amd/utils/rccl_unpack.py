"""RCCL's device code, unpacked once per host for gfx950.

ROCm ships ``librccl.so`` with its device code as ONE compressed offload bundle (``CCOB``,
zstd) for 12 GPU targets: 570 MB that the HIP runtime inflates to 5.3 GB in every process that
first launches an RCCL kernel, to take the gfx950 code object out of it. That inflation is
~1.7 s of every ``ncclCommInit*`` on the MI355X (docs/benchmarks-history.md), i.e. nearly all
of the fabric check (BASELINE configs 4-5), and it is the same work every time.

Done once per host instead, the way a node runtime install prepares its libraries (the
reference's dockersetup role, ansible/roles/dockersetup/tasks/main.yml:42-46): the gfx950 code
object is taken out of the bundle (``clang-offload-bundler``), re-bundled UNcompressed with
only that target, and written over the ``.hip_fatbin`` section of a copy of the library -- at
the same file offset, zero-padded to the same size, so every address, relocation and the
fatbin wrapper stay exactly as they were (569 MB of gfx950 code fits the 570 MB section). The
host code is byte-for-byte the installed RCCL; only its device code is stored unpacked -- and
without its DWARF (460 of the 569 MB; ``TK8S_RCCL_KEEP_DEBUG=1`` keeps it for rocgdb) -- and HIP
then loads the 108 MB code object straight from the mapped library.

The copy lives in the tk8s tree (``build/rccl-<arch>/librccl.so.1``: read-only to pods, like
the rest of the install), is keyed to the installed library (path, size, mtime) and rebuilt when
that changes; the fabric check's ranks load it through ``LD_LIBRARY_PATH``
(``fabric.FabricCheck``), and use the installed library whenever it is missing or stale.
``TK8S_RCCL_UNPACKED=0`` turns it off.
"""
from __future__ import annotations

import json
import os
import struct
import subprocess
import tempfile
from pathlib import Path

from .build_native import ARCH, REPO, ROCM

OUT = REPO / "build" / f"rccl-{ARCH}"
LIB_NAME = "librccl.so.1"
TRIPLE = f"hipv4-amdgcn-amd-amdhsa--{ARCH}"
HOST_TRIPLE = "host-x86_64-unknown-linux-gnu-"


def installed_library() -> Path | None:
    for p in (ROCM / "lib" / LIB_NAME, ROCM / "lib" / "librccl.so"):
        if p.exists():
            return p.resolve()
    return None


def elf_section(path: Path, name: str) -> tuple[int, int] | None:
    """(file offset, size) of section ``name`` of a 64-bit little-endian ELF file; None for a file
    that is not one, or is truncated or malformed (an optional speed-up must never
    abort the native build)."""
    try:
        return _elf_section(path, name)
    except (struct.error, IndexError, ValueError, UnicodeDecodeError):
        return None


def _elf_section(path: Path, name: str) -> tuple[int, int] | None:
    with open(path, "rb") as f:
        eh = f.read(64)
        if eh[:4] != b"\x7fELF" or eh[4] != 2 or eh[5] != 1:
            return None
        shoff, = struct.unpack_from("<Q", eh, 0x28)
        shentsize, shnum, shstrndx = struct.unpack_from("<HHH", eh, 0x3A)
        f.seek(shoff)
        table = f.read(shentsize * shnum)
        sh = [struct.unpack_from("<IIQQQQIIQQ", table, i * shentsize) for i in range(shnum)]
        stroff, strsize = sh[shstrndx][4], sh[shstrndx][5]
        f.seek(stroff)
        names = f.read(strsize)
    for s in sh:
        end = names.index(b"\0", s[0])
        if names[s[0]:end].decode() == name:
            return s[4], s[5]
    return None


def _stamp(src: Path) -> dict:
    st = src.stat()
    return {"source": str(src), "size": st.st_size, "mtime_ns": st.st_mtime_ns, "arch": ARCH,
            "debug": os.environ.get("TK8S_RCCL_KEEP_DEBUG", "0") == "1"}


def library_dir() -> Path | None:
    """The directory of the unpacked copy when it is current for the installed RCCL, else None."""
    if os.environ.get("TK8S_RCCL_UNPACKED", "1") == "0":
        return None
    src = installed_library()
    try:
        stamp = json.loads((OUT / "stamp.json").read_text())
    except (OSError, ValueError):
        return None
    if src is None or stamp != _stamp(src) or not (OUT / LIB_NAME).is_file():
        return None
    return OUT


def _bundler() -> str:
    for p in (ROCM / "lib" / "llvm" / "bin" / "clang-offload-bundler", ROCM / "llvm" / "bin" / "clang-offload-bundler"):
        if p.exists():
            return str(p)
    raise FileNotFoundError("clang-offload-bundler not found under ROCm")


def unpack(force: bool = False, verbose: bool = False) -> dict:
    """Make (or confirm) the unpacked copy. Returns what was done; never raises for a library it
    cannot unpack (not compressed, no gfx950 entry, the code object does not fit): the installed
    one is then used as it is. One process at a time makes it (a lock beside it): inflating the
    bundle takes ~5 GB of memory, and concurrent builds (test workers) wait for the first."""
    import fcntl

    src = installed_library()
    if src is None:
        return {"ok": False, "why": "no librccl under ROCm"}
    if not force and library_dir() is not None:
        return {"ok": True, "path": str(OUT / LIB_NAME), "changed": False}
    OUT.mkdir(parents=True, exist_ok=True)
    with open(OUT / ".lock", "w") as lock:
        fcntl.flock(lock, fcntl.LOCK_EX)
        if not force and library_dir() is not None:  # made by another process meanwhile
            return {"ok": True, "path": str(OUT / LIB_NAME), "changed": False}
        return _unpack(src, verbose)


def _unpack(src: Path, verbose: bool) -> dict:
    sec = elf_section(src, ".hip_fatbin")
    if sec is None:
        return {"ok": False, "why": f"{src}: no .hip_fatbin section"}
    off, size = sec
    with open(src, "rb") as f:
        f.seek(off)
        magic = f.read(4)
    if magic != b"CCOB":
        return {"ok": False, "why": f"{src}: device code is not a compressed bundle (nothing to unpack)"}
    OUT.mkdir(parents=True, exist_ok=True)
    with tempfile.TemporaryDirectory(dir=OUT) as tmp:
        t = Path(tmp)
        with open(src, "rb") as f, open(t / "fatbin", "wb") as g:
            f.seek(off)
            left = size
            while left:
                chunk = f.read(min(left, 64 << 20))
                if not chunk:
                    break
                g.write(chunk)
                left -= len(chunk)
        bundler = _bundler()
        (t / "host.o").write_bytes(b"")
        r = subprocess.run([bundler, "--unbundle", "--type=o", f"--input={t / 'fatbin'}", f"--targets={TRIPLE}",
                            f"--output={t / 'dev.co'}"], capture_output=True, text=True)
        (t / "fatbin").unlink()
        if r.returncode != 0 or not (t / "dev.co").exists() or (t / "dev.co").stat().st_size == 0:
            return {"ok": False, "why": f"no {TRIPLE} entry: {r.stderr[-300:]}"}
        full = (t / "dev.co").stat().st_size
        if os.environ.get("TK8S_RCCL_KEEP_DEBUG", "0") != "1":
            # 460 of its 569 MB are DWARF for rocgdb: the loader would read and copy them into
            # every rank for nothing (the kernels, their metadata and symbols stay)
            r = subprocess.run([str(Path(bundler).parent / "llvm-objcopy"), "--strip-debug", str(t / "dev.co")],
                               capture_output=True, text=True)
            if r.returncode != 0:
                return {"ok": False, "why": f"strip-debug failed: {r.stderr[-300:]}"}
        r = subprocess.run([bundler, "--type=o", "--bundle-align=4096", f"--targets={HOST_TRIPLE},{TRIPLE}",
                            f"--input={t / 'host.o'}", f"--input={t / 'dev.co'}", f"--output={t / 'bundle'}"],
                           capture_output=True, text=True)
        (t / "dev.co").unlink()
        if r.returncode != 0:
            return {"ok": False, "why": f"re-bundling failed: {r.stderr[-300:]}"}
        new = (t / "bundle").stat().st_size
        if new > size:
            return {"ok": False, "why": f"the unpacked {ARCH} code ({new} B) does not fit the section ({size} B)"}
        lib = t / LIB_NAME
        with open(src, "rb") as f, open(lib, "wb") as g:  # a byte copy of the installed library ...
            while True:
                chunk = f.read(64 << 20)
                if not chunk:
                    break
                g.write(chunk)
        with open(t / "bundle", "rb") as b, open(lib, "r+b") as g:  # ... with its fatbin section replaced
            g.seek(off)
            while True:
                chunk = b.read(64 << 20)
                if not chunk:
                    break
                g.write(chunk)
            left, zero = size - new, bytes(16 << 20)
            while left:
                g.write(zero[:min(left, len(zero))])
                left -= min(left, len(zero))
        lib.chmod(0o755)
        os.replace(lib, OUT / LIB_NAME)
        (OUT / "stamp.json").write_text(json.dumps(_stamp(src)))
    if verbose:
        print(f"unpacked {src} -> {OUT / LIB_NAME} ({new} B of {ARCH} code in a {size} B section)", flush=True)
    return {"ok": True, "path": str(OUT / LIB_NAME), "changed": True, "code_object_bytes": full, "bundle_bytes": new,
            "section_bytes": size}


if __name__ == "__main__":
    import sys

    print(json.dumps(unpack(force="--force" in sys.argv, verbose=True)))
