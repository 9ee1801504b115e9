"""Host GPU inventory WITHOUT initialising the GPU.

Reads the KFD topology in sysfs (``/sys/class/kfd/kfd/topology/nodes/*``): GPU nodes carry a
non-zero ``gfx_target_version`` (90500 = gfx950) and ``io_links`` whose ``type`` 11 is xGMI.
Only render nodes this process may open count (a container may see all GPUs in sysfs but be
granted a subset), and ``ROCR_VISIBLE_DEVICES`` then ``HIP_VISIBLE_DEVICES``/``CUDA_VISIBLE_DEVICES``
are honoured.
``TK8S_FAKE_GPUS=N`` replaces the inventory with N virtual fully-xGMI-connected gfx950 GPUs so
the allocation logic runs on CPU-only hosts.

Why not HIP: processes that spawn other programs (provisioner, agents) must never touch the
GPU runtime; only leaf validation pods do (tools/tk8s_gpuinfo.cpp is the authoritative view).
"""
from __future__ import annotations

import os
from pathlib import Path

from ..earlyburn import compose_visible_devices, idx_list, kfd_gpu_nodes, read_props, visible_filter  # noqa: F401
from ..utils.record import asdict, field, record as dataclass

KFD_ROOT = Path("/sys/class/kfd/kfd/topology/nodes")
IOLINK_XGMI = 11
IOLINK_PCIE = 2


@dataclass
class HostGpu:
    ordinal: int            # index in this process's visible view (what HIP calls device i)
    kfd_node: int = -1
    gfx: str = "gfx950"
    render_minor: int = -1
    simd_count: int = 0
    cu_count: int = 0
    mem_bytes: int = 0
    location_id: int = 0
    domain: int = 0
    fake: bool = False

    @property
    def pci_bus_id(self) -> str:
        """dddd:bb:dd.f from the KFD node's PCI domain and location_id (bus<<8 | dev<<3 | fn) —
        the key that joins this view to AMD SMI's and HIP's."""
        loc = self.location_id
        return f"{self.domain:04x}:{(loc >> 8) & 0xff:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 7:x}"

    def to_dict(self) -> dict:
        return {**asdict(self), "pci_bus_id": self.pci_bus_id}


@dataclass
class HostInventory:
    gpus: list[HostGpu] = field(default_factory=list)
    # links[i][j] = {"type": "xgmi"|"pcie"|"self"|"unknown", "hops": int}
    links: list[list[dict]] = field(default_factory=list)
    source: str = "none"

    @property
    def count(self) -> int:
        return len(self.gpus)

    def to_dict(self) -> dict:
        return {"gpus": [g.to_dict() for g in self.gpus], "links": self.links, "source": self.source}


def _props(path: Path) -> dict[str, int]:
    out = {}
    try:
        for line in path.read_text().splitlines():
            parts = line.split()
            if len(parts) == 2:
                try:
                    out[parts[0]] = int(parts[1])
                except ValueError:
                    pass
    except OSError:
        pass
    return out


def _gfx_name(v: int) -> str:
    major, minor, step = v // 10000, (v // 100) % 100, v % 100
    return f"gfx{major}{minor:x}{step:x}" if v else "cpu"


_idx_list = idx_list
_visible_filter = visible_filter


def fake_inventory(n: int) -> HostInventory:
    gpus = [HostGpu(ordinal=i, kfd_node=i + 1, render_minor=128 + i, simd_count=1024, cu_count=256,
                    mem_bytes=288 * 10**9, location_id=(0x10 + i) << 8, fake=True) for i in range(n)]
    links = [[{"type": "self" if i == j else "xgmi", "hops": 0 if i == j else 1} for j in range(n)] for i in range(n)]
    return HostInventory(gpus=gpus, links=links, source="fake")


_CACHE: dict[tuple, HostInventory] = {}


def discover(root: Path = KFD_ROOT, cache: bool = True) -> HostInventory:
    """Host inventory; memoised per process for the same root and visibility environment
    (provisioning asks once per machine, the playbook once per host: on an 8-GPU host each
    sysfs walk reads ~100 property files). The result is shared: treat it as read-only."""
    key = (str(root), os.environ.get("TK8S_FAKE_GPUS"), os.environ.get("ROCR_VISIBLE_DEVICES"),
           os.environ.get("HIP_VISIBLE_DEVICES"), os.environ.get("CUDA_VISIBLE_DEVICES"))
    if cache and key in _CACHE:
        return _CACHE[key]
    inv = _discover(root)
    if cache:
        _CACHE[key] = inv
    return inv


def _discover(root: Path) -> HostInventory:
    fake = os.environ.get("TK8S_FAKE_GPUS")
    if fake is not None and fake.strip() != "":
        return fake_inventory(int(fake))
    nodes = [(n, p, Path(d)) for n, p, d in kfd_gpu_nodes(str(root))]
    gpus: list[HostGpu] = []
    for kfd_node, p, _ in nodes:
        minor = p.get("drm_render_minor", -1)
        gpus.append(HostGpu(
            ordinal=len(gpus), kfd_node=kfd_node, gfx=_gfx_name(p.get("gfx_target_version", 0)),
            render_minor=minor, simd_count=p.get("simd_count", 0),
            cu_count=p.get("simd_count", 0) // max(p.get("simd_per_cu", 4), 1),
            location_id=p.get("location_id", 0), domain=p.get("domain", 0),
        ))
    vis = _visible_filter(len(gpus))
    if vis is not None:
        gpus = [gpus[i] for i in vis]
        for i, g in enumerate(gpus):
            g.ordinal = i
    by_node = {g.kfd_node: g.ordinal for g in gpus}
    n = len(gpus)
    links = [[{"type": "self" if i == j else "unknown", "hops": 0} for j in range(n)] for i in range(n)]
    for kfd_node, _, d in nodes:
        if kfd_node not in by_node:
            continue
        i = by_node[kfd_node]
        io = d / "io_links"
        if not io.is_dir():
            continue
        for link in io.iterdir():
            lp = _props(link / "properties")
            j = by_node.get(lp.get("node_to", -1))
            if j is None or j == i:
                continue
            t = lp.get("type", 0)
            links[i][j] = {"type": "xgmi" if t == IOLINK_XGMI else "pcie" if t == IOLINK_PCIE else "unknown",
                           "hops": 1}
    return HostInventory(gpus=gpus, links=links, source="kfd-sysfs" if n else "none")
