"""Node runtime facts of the machine this runs on (the rocmsetup role's ``tk8s_gpu_facts``).

Replaces the reference's ``docker --version | grep 1.12.6`` idempotency probe
(ansible/roles/dockersetup/tasks/main.yml:2-4): what ROCm userspace is installed, whether the
KFD device is usable, how many GPUs the kernel exposes (sysfs only, the GPU is never
initialised), and whether the tk8s native validation tools are present. Runs in-process for the
local provider and as ``python3 -S -m tritonk8ssupervisor_amd.nodefacts`` on a remote machine
(one JSON line on stdout).
"""
from __future__ import annotations

import json
import os
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
NATIVE_TOOLS = ("tk8s-gpuinfo", "tk8s-probe", "tk8s-rccl")


def rocm_version(root: str | os.PathLike | None = None) -> str:
    """The installed ROCm version, from the install directory's name when it carries one
    (``/opt/rocm`` -> ``/opt/rocm-7.2.0``: a symlink, metadata only) and from ``.info/version``
    otherwise. On the GPU hosts the image's files are paged in on their first read: on a fresh
    box the first read of ``.info/version`` took 0.80 s of the first bring-up's critical path
    (node facts, play 1; ``profiles/r5_cold_facts/``) -- the cold first run of BENCH_r04."""
    import re

    base = Path(root or os.environ.get("ROCM_PATH", "/opt/rocm"))
    m = re.fullmatch(r"rocm-(\d+\.\d+\.\d+)", os.path.basename(os.path.realpath(base)))
    if m:
        return m.group(1)
    try:
        return (base / ".info" / "version").read_text().strip()
    except OSError:
        return ""


def node_facts(timing: dict | None = None) -> dict:
    """The facts; ``timing`` (when given) receives how long each part took, in ms: a slow
    gathering on the bring-up's critical path names its part (bench.py's cold first run)."""
    import time

    t = time.perf_counter()
    marks = []

    def mark(what: str) -> None:
        nonlocal t
        now = time.perf_counter()
        marks.append((what, round((now - t) * 1e3, 3)))
        t = now

    from .models.hostinfo import discover

    mark("import")
    rocm = rocm_version()
    mark("rocm_version")
    kfd = os.path.exists("/dev/kfd") and os.access("/dev/kfd", os.R_OK | os.W_OK)
    mark("kfd_access")
    inv = discover()
    mark("gpu_inventory")
    built = all((PKG / "bin" / t).exists() for t in NATIVE_TOOLS)
    mark("native_tools")
    if timing is not None:
        timing.update(marks)
    return {
        "tk8s_rocm_version": rocm,
        "tk8s_kfd": kfd,
        "tk8s_host_gpus": inv.count,
        "tk8s_inventory_source": inv.source,
        "tk8s_native_built": built,
        "tk8s_node_python": sys.version.split()[0],
        "tk8s_node_kernel": os.uname().release,
    }


if __name__ == "__main__":
    print(json.dumps(node_facts(), separators=(",", ":")))
