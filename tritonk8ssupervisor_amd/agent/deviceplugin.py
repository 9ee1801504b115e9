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
Runtime health comes from AMD SMI (``tk8s-smi``, no HIP): ``update_from_smi`` marks a device
Unhealthy while it reports uncorrectable or deferred ECC errors, and keeps its telemetry.
"""
from __future__ import annotations

import os
from pathlib import Path

from ..models.hostinfo import HostInventory, compose_visible_devices, discover
from ..utils.record import field, record as dataclass

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
    telemetry: dict = field(default_factory=dict)   # last AMD SMI sample (temp, power, ECC, VRAM)

    def to_dict(self) -> dict:
        d = {"id": self.id, "ordinal": self.ordinal, "health": self.health, "gfx": self.gfx,
             "renderMinor": self.render_minor, "pciBusId": self.pci_bus_id, "uuid": self.uuid,
             "reason": self.reason}
        if self.telemetry:
            d["telemetry"] = self.telemetry
        return d


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
                self.devices_.append(Device(f"gpu{o}", o, "Healthy", g.render_minor, g.gfx,
                                            pci_bus_id=g.pci_bus_id if g.location_id else ""))

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

    def update_from_smi(self, result: dict) -> bool:
        """Fold one AMD SMI sample (tk8s-smi JSON, every GPU of the host, keyed by PCI bus id).
        Returns True if any device's health changed."""
        if not result.get("ok"):
            return False
        by_pci = {g.get("pci_bus_id", "").lower(): g for g in result.get("gpus", [])}
        changed = False
        for d in self.devices_:
            g = by_pci.get(d.pci_bus_id.lower()) if d.pci_bus_id else None
            if g is None:
                continue
            ecc = g.get("ecc") or {}
            ue, deferred = int(ecc.get("uncorrectable", 0) or 0), int(ecc.get("deferred", 0) or 0)
            d.telemetry = {k: g[k] for k in ("temp_c", "power", "vram_used_bytes", "ecc", "activity") if k in g}
            if d.reason == "probe failed":
                continue
            if ue or deferred:
                reason = f"ECC: {ue} uncorrectable, {deferred} deferred"
                if d.health != "Unhealthy" or d.reason != reason:
                    d.health, d.reason, changed = "Unhealthy", reason, True
            elif d.reason.startswith("ECC:"):
                d.health, d.reason, changed = "Healthy", "", True
        return changed

    def telemetry_annotations(self) -> dict[str, str]:
        """Node-level summary of the last AMD SMI sample (hottest GPU, total power, ECC)."""
        tel = [d.telemetry for d in self.devices_ if d.telemetry]
        if not tel:
            return {}
        hot = [t["temp_c"]["hotspot"] for t in tel if "hotspot" in t.get("temp_c", {})]
        watts = [t["power"]["current_w"] for t in tel if "current_w" in t.get("power", {})]
        ue = sum(int(t.get("ecc", {}).get("uncorrectable", 0) or 0) for t in tel)
        out = {"amd.com/gpu-health-source": "amdsmi", "amd.com/gpu-ecc-uncorrectable": str(ue)}
        if hot:
            out["amd.com/gpu-temp-hotspot-max-c"] = str(max(hot))
        if watts:
            out["amd.com/gpu-power-w"] = str(sum(watts))
        return out

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
