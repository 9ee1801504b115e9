"""RCCL's gfx950 device code unpacked once per host (utils/rccl_unpack.py).

The copy must be the installed library byte for byte outside its .hip_fatbin section, and that
section must hold an uncompressed offload bundle with exactly the host and gfx950 entries, the
gfx950 entry an AMDGPU code object without DWARF. A copy that is missing or keyed to another
library is not used (the installed one is). On the MI355X the ranks load it and pass
(tests/test_kernels_gpu.py::test_unpacked_rccl_starts_faster_on_a_real_gpu)."""
from __future__ import annotations

import json
import struct
from pathlib import Path

import pytest

from tritonk8ssupervisor_amd.utils import rccl_unpack as ru

pytestmark = pytest.mark.skipif(ru.installed_library() is None, reason="no librccl under ROCm")


def _bundle_entries(f, off: int) -> list[tuple[int, int, str]]:
    f.seek(off)
    head = f.read(32)
    assert head[:24] == b"__CLANG_OFFLOAD_BUNDLE__", head[:24]
    n, = struct.unpack("<Q", head[24:32])
    out = []
    for _ in range(n):
        o, s, tl = struct.unpack("<QQQ", f.read(24))
        out.append((o, s, f.read(tl).decode()))
    return out


def _section_names(f, base: int) -> list[str]:
    f.seek(base)
    eh = f.read(64)
    assert eh[:4] == b"\x7fELF" and struct.unpack_from("<H", eh, 0x12)[0] == 0xE0  # EM_AMDGPU
    shoff, = struct.unpack_from("<Q", eh, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", eh, 0x3A)
    f.seek(base + shoff)
    table = f.read(shentsize * shnum)
    sh = [struct.unpack_from("<IIQQQQIIQQ", table, i * shentsize) for i in range(shnum)]
    f.seek(base + sh[shstrndx][4])
    names = f.read(sh[shstrndx][5])
    return [names[s[0]:names.index(b"\0", s[0])].decode() for s in sh]


@pytest.mark.timeout(600)
def test_the_unpacked_copy_differs_only_in_its_device_code():
    res = ru.unpack()
    if not res["ok"]:
        pytest.skip(res["why"])
    src, dst = ru.installed_library(), ru.OUT / ru.LIB_NAME
    assert ru.library_dir() == ru.OUT
    off, size = ru.elf_section(src, ".hip_fatbin")
    assert ru.elf_section(dst, ".hip_fatbin") == (off, size)
    assert dst.stat().st_size == src.stat().st_size
    with open(src, "rb") as a, open(dst, "rb") as b:
        assert a.read(off) == b.read(off)  # headers, tables, host code before the section
        for pos in range(off + size, src.stat().st_size, 8 << 20):  # everything after it
            a.seek(pos)
            b.seek(pos)
            assert a.read(8 << 20) == b.read(8 << 20), pos
        a.seek(off)
        assert a.read(4) == b"CCOB"  # the installed one: compressed, every target
        entries = _bundle_entries(b, off)
        assert sorted(t for _, _, t in entries) == sorted([ru.HOST_TRIPLE, ru.TRIPLE])
        o, s, _ = next(e for e in entries if e[2] == ru.TRIPLE)
        assert o % 4096 == 0 and 0 < o + s <= size and s > (16 << 20)
        names = _section_names(b, off + o)
        assert ".text" in names and not any(n.startswith(".debug") for n in names)
        b.seek(off + o + s)  # zero padding to the end of the section
        assert b.read(min(1 << 20, size - o - s)).count(0) == min(1 << 20, size - o - s)
    assert json.loads((ru.OUT / "stamp.json").read_text())["source"] == str(src)
    assert ru.unpack()["changed"] is False  # current: nothing to redo


def test_a_stale_or_disabled_copy_is_not_used(monkeypatch, tmp_path):
    monkeypatch.setattr(ru, "OUT", tmp_path)
    assert ru.library_dir() is None  # none made here
    (tmp_path / ru.LIB_NAME).write_bytes(b"x")
    src = ru.installed_library()
    stamp = ru._stamp(src)
    (tmp_path / "stamp.json").write_text(json.dumps(stamp))
    assert ru.library_dir() == tmp_path
    (tmp_path / "stamp.json").write_text(json.dumps({**stamp, "size": stamp["size"] + 1}))  # RCCL was upgraded
    assert ru.library_dir() is None
    (tmp_path / "stamp.json").write_text(json.dumps(stamp))
    monkeypatch.setenv("TK8S_RCCL_UNPACKED", "0")
    assert ru.library_dir() is None


def test_elf_section_reader(tmp_path):
    assert ru.elf_section(Path("/bin/sh").resolve(), ".text") is not None
    (tmp_path / "x").write_bytes(b"not an elf" * 10)
    assert ru.elf_section(tmp_path / "x", ".text") is None


def test_transport_report_of_a_one_rank_log(tmp_path):
    """a 1-rank communicator connects no channel, but its INFO log is there
    -- the report says it was logged, that init completed, and which library the rank loaded."""
    from tritonk8ssupervisor_amd.fabric import rccl_transports

    one = tmp_path / "rank0.log"
    one.write_text("host:1:1 [0] NCCL INFO ROCr version 1.18\nLibrccl path : /x/build/rccl-gfx950/librccl.so.1\n"
                   "host:1:1 [0] NCCL INFO comm 0x1 rank 0 nranks 1 cudaDev 0 busId 5000 - Init COMPLETE\n")
    r = rccl_transports([str(one)])
    assert r["logged"] and r["init_complete"] and r["p2p"] == 0 and r["library"].endswith("rccl-gfx950/librccl.so.1")
    two = tmp_path / "rank1.log"
    two.write_text("host:1:1 [0] NCCL INFO Channel 00/0 : 0[0] -> 1[1] via P2P/IPC\n")
    r = rccl_transports([str(one), str(two), None])
    assert r["p2p"] == 1 and r["logged"]
    assert rccl_transports([str(tmp_path / "none.log")]) == {"p2p": 0, "shm": 0, "net": 0, "collnet": 0,
                                                              "logged": False, "init_complete": False, "library": None}


def test_the_fabric_rank_env_carries_the_unpacked_library_and_huge_page_malloc(monkeypatch, tmp_path):
    """fabric.rccl_rank_env: the unpacked copy asked for (the node's agent prepends ITS copy to the
    rank's LD_LIBRARY_PATH) and glibc's malloc on huge pages (profiles/r5_thp: 318 -> 202 ms
    communicator start), each with its own off-switch; fake GPUs get neither. A GLIBC_TUNABLES
    already set is kept."""
    from tritonk8ssupervisor_amd import fabric
    from tritonk8ssupervisor_amd.utils import rccl_unpack

    monkeypatch.setattr(rccl_unpack, "library_dir", lambda: tmp_path)
    for var in ("TK8S_RCCL_THP", "GLIBC_TUNABLES", "NCCL_DEBUG", "NCCL_DEBUG_SUBSYS", "TK8S_SHORTCUTS", "TK8S_FAULTS",
                "TK8S_GPU_SYNC_TIMEOUT_S", "TK8S_RCCL_BLOCKING", "TK8S_RCCL_PREWARM"):
        monkeypatch.delenv(var, raising=False)
    env, lib = fabric.rccl_rank_env()
    assert lib == tmp_path
    assert {e["name"]: e["value"] for e in env} == {"TK8S_RCCL_UNPACKED": "1",
                                                     "GLIBC_TUNABLES": "glibc.malloc.hugetlb=1"}
    monkeypatch.setenv("GLIBC_TUNABLES", "glibc.malloc.arena_max=2")
    monkeypatch.setenv("NCCL_DEBUG", "INFO")
    env, _ = fabric.rccl_rank_env()
    got = {e["name"]: e["value"] for e in env}
    assert got["GLIBC_TUNABLES"] == "glibc.malloc.arena_max=2:glibc.malloc.hugetlb=1" and got["NCCL_DEBUG"] == "INFO"
    monkeypatch.setenv("TK8S_RCCL_THP", "0")
    assert "GLIBC_TUNABLES" not in {e["name"] for e in fabric.rccl_rank_env()[0]}
    monkeypatch.setenv("TK8S_RCCL_PREWARM", "0")  # the rank's code load on threads: off in the rank too
    assert {"name": "TK8S_RCCL_PREWARM", "value": "0"} in fabric.rccl_rank_env()[0]
    env, lib = fabric.rccl_rank_env(fake=True)
    assert lib is None and [e["name"] for e in env] == ["NCCL_DEBUG"]


def test_the_agent_prepends_its_own_unpacked_copy(tmp_path):
    """the rank's LD_LIBRARY_PATH is the node's copy IN FRONT of the path the node's
    runtime passes on (not replacing it); no request, or no current copy on that node: unchanged."""
    from tritonk8ssupervisor_amd.agent.agent import unpacked_rccl_env

    ask = {"TK8S_RCCL_UNPACKED": "1"}
    assert unpacked_rccl_env(ask, {"LD_LIBRARY_PATH": "/opt/x/lib"}, lambda: tmp_path) == {
        "LD_LIBRARY_PATH": f"{tmp_path}:/opt/x/lib"}
    assert unpacked_rccl_env(ask, {}, lambda: tmp_path) == {"LD_LIBRARY_PATH": str(tmp_path)}
    assert unpacked_rccl_env(ask, {"LD_LIBRARY_PATH": "/opt/x/lib"}, lambda: None) == {}
    assert unpacked_rccl_env({}, {"LD_LIBRARY_PATH": "/opt/x/lib"}, lambda: tmp_path) == {}


def test_the_fabric_rank_env_passes_the_fail_fast_knobs_and_rccl_faults(monkeypatch):
    from tritonk8ssupervisor_amd import fabric

    monkeypatch.setenv("TK8S_FAULTS", "agent.crash@kubenode1, rccl.hang@sweep:1,xgmi.degrade@0-1:0.1,rccl.exit@uid")
    monkeypatch.setenv("TK8S_GPU_SYNC_TIMEOUT_S", "3")
    env, _ = fabric.rccl_rank_env(fake=True)
    got = {e["name"]: e["value"] for e in env}
    assert got["TK8S_FAULTS"] == "rccl.hang@sweep:1,rccl.exit@uid" and got["TK8S_GPU_SYNC_TIMEOUT_S"] == "3"


def test_elf_section_survives_truncated_and_odd_files(tmp_path):
    """a truncated or malformed library must not raise out of the optional unpack."""
    sh = Path("/bin/sh").resolve().read_bytes()
    for n in (0, 10, 64, 200, len(sh) // 2):
        f = tmp_path / f"t{n}"
        f.write_bytes(sh[:n])
        ru.elf_section(f, ".hip_fatbin")  # None or a tuple; never struct.error / IndexError
    odd = bytearray(sh[:64]) + bytes(64)
    odd[0x3C:0x3E] = (0xFFFF).to_bytes(2, "little")  # e_shnum far beyond the file
    (tmp_path / "odd").write_bytes(bytes(odd))
    assert ru.elf_section(tmp_path / "odd", ".text") is None


def test_doctor_reports_the_huge_page_mode(tmp_path):
    from tritonk8ssupervisor_amd.doctor import transparent_huge_pages

    f = tmp_path / "enabled"
    f.write_text("always [madvise] never\n")
    assert transparent_huge_pages(str(f))["status"] == "OK" and "madvise" in transparent_huge_pages(str(f))["detail"]
    f.write_text("always madvise [never]\n")
    assert transparent_huge_pages(str(f))["status"] == "WARN"
    assert transparent_huge_pages(str(tmp_path / "missing"))["status"] == "WARN"
