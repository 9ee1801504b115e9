"""amd.com/gpu device plugin core (N2): discovery, health, preferred allocation, Allocate.

K8s device-plugin v1beta1 semantics without a kubelet in between:
  ListAndWatch          -> ``devices()`` (+ ``refresh_health()``), pushed in node heartbeats
  GetPreferredAllocation-> ``preferred(available, must_include, size)`` — xGMI-aware, C++ core
                           (native/src/topology.cpp via ``_tk8s_topo``)
  Allocate              -> ``allocate(ids)``: env (HIP/CUDA_VISIBLE_DEVICES composed onto the
                           agent's own view), device nodes (/dev/kfd, /dev/dri/renderD*)

Discovery reads the KFD sysfs topology (models/hostinfo.py) and never initialises HIP: the
agent spawns pods, so it must stay GPU-clean. The validation pod (tk8s-probe, HIP) is the
authoritative check; its gpuinfo output refreshes PCI ids / UUIDs via ``update_from_probe``.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from pathlib import Path

from ..models.hostinfo import HostInventory, compose_visible_devices, discover

_LINK_WEIGHT = {"self": 1000, "xgmi": 100, "pcie": 10}


def link_matrix(links: list[list[dict]]) -> list[int]:
    """Flatten a links[i][j] = {type, hops} matrix into link weights (row-major)."""
    n = len(links)
    out = []
    for i in range(n):
        for j in range(n):
            lk = links[i][j] if j < len(links[i]) else {"type": "unknown", "hops": 1}
            w = _LINK_WEIGHT.get(lk.get("type", "unknown"), 1)
            hops = max(int(lk.get("hops", 1) or 1), 1)
            out.append(w if lk.get("type") == "self" else max(w // hops, 1))
    return out


@dataclass
class Device:
    id: str
    ordinal: int              # host ordinal (this agent's parent view)
    health: str = "Healthy"
    render_minor: int = -1
    gfx: str = "gfx950"
    pci_bus_id: str = ""
    uuid: str = ""
    reason: str = ""

    def to_dict(self) -> dict:
        return {"id": self.id, "ordinal": self.ordinal, "health": self.health, "gfx": self.gfx,
                "renderMinor": self.render_minor, "pciBusId": self.pci_bus_id, "uuid": self.uuid,
                "reason": self.reason}


@dataclass
class DevicePlugin:
    node_gpus: list[int]
    inventory: HostInventory = field(default_factory=discover)
    devices_: list[Device] = field(default_factory=list)

    def __post_init__(self):
        by_ord = {g.ordinal: g for g in self.inventory.gpus}
        for o in self.node_gpus:
            g = by_ord.get(o)
            if g is None:
                self.devices_.append(Device(f"gpu{o}", o, "Unhealthy", reason="not visible on this host"))
            else:
                self.devices_.append(Device(f"gpu{o}", o, "Healthy", g.render_minor, g.gfx))

    # ---- ListAndWatch -----------------------------------------------------------------
    def devices(self) -> list[dict]:
        return [d.to_dict() for d in self.devices_]

    def refresh_health(self) -> bool:
        """Cheap periodic health check (render node still present). Returns True if changed."""
        changed = False
        for d in self.devices_:
            if d.render_minor < 0 or os.environ.get("TK8S_FAKE_GPUS"):
                continue
            ok = Path(f"/dev/dri/renderD{d.render_minor}").exists()
            new = "Healthy" if ok else "Unhealthy"
            if new != d.health and d.reason != "probe failed":
                d.health, changed = new, True
        return changed

    def update_from_probe(self, result: dict) -> None:
        """Fold the validation pod's HIP gpuinfo (pod-local device i = allocated ids[i])."""
        info = result.get("gpuinfo") or {}
        ids = result.get("_allocated_ids") or [d.id for d in self.devices_]
        by_id = {d.id: d for d in self.devices_}
        for i, dev in enumerate(info.get("devices", [])):
            if i < len(ids) and ids[i] in by_id:
                d = by_id[ids[i]]
                d.pci_bus_id = dev.get("pci_bus_id", d.pci_bus_id)
                d.uuid = dev.get("uuid", d.uuid)
                d.gfx = dev.get("gfx", d.gfx)
        if result.get("ok") is False:
            for d in self.devices_:
                if d.id in ids:
                    d.health, d.reason = "Unhealthy", "probe failed"

    # ---- GetPreferredAllocation ---------------------------------------------------------
    def preferred(self, available: list[str], must_include: list[str], size: int) -> list[str]:
        by_id = {d.id: d for d in self.devices_}
        inv_n = self.inventory.count
        if size <= 0:
            return []
        if inv_n == 0 or size == 1:
            must = [i for i in must_include if i in available]
            rest = [i for i in sorted(available, key=lambda x: by_id[x].ordinal) if i not in must]
            return (must + rest)[:size]
        from ..ops import topo

        res = topo().preferred_allocation(inv_n, link_matrix(self.inventory.links),
                                          [by_id[i].ordinal for i in available],
                                          [by_id[i].ordinal for i in must_include], size)
        back = {d.ordinal: d.id for d in self.devices_}
        return [back[o] for o in res["devices"]]

    # ---- Allocate ---------------------------------------------------------------------
    def allocate(self, ids: list[str]) -> dict:
        by_id = {d.id: d for d in self.devices_}
        ords = [by_id[i].ordinal for i in ids]
        env = compose_visible_devices(ords)
        devs = ["/dev/kfd"] + [f"/dev/dri/renderD{by_id[i].render_minor}" for i in ids if by_id[i].render_minor >= 0]
        return {"env": env, "devices": devs, "annotations": {"amd.com/gpu-ids": ",".join(ids)}}
