"""CPU stand-in for ``tk8s-smi`` (AMD SMI health) over the fake gfx950 inventory (TK8S_FAKE_GPUS).

Same JSON shape and exit codes as native/tools/tk8s_smi.cpp. Like AMD SMI it reports every GPU
of the host (it ignores ROCR/HIP visibility); callers join on ``pci_bus_id``.

Fault injection (uncorrectable ECC errors), host ordinal -> count, comma separated:
``TK8S_FAKE_SMI_UE="0:2,3:1"``, or the same text in the file named by ``TK8S_FAKE_SMI_FILE``
(read on every call, so a test can inject errors into a running cluster).
"""
from __future__ import annotations

import json
import os
import sys


def _faults() -> dict[int, int]:
    text = os.environ.get("TK8S_FAKE_SMI_UE", "")
    path = os.environ.get("TK8S_FAKE_SMI_FILE")
    if path:
        try:
            with open(path) as f:
                text = f.read()
        except OSError:
            pass
    out = {}
    for part in text.replace("\n", ",").split(","):
        if ":" in part:
            k, v = part.split(":", 1)
            if k.strip().isdigit() and v.strip().isdigit():
                out[int(k)] = int(v)
    return out


def report(n: int | None = None, with_links: bool = True) -> dict:
    if n is None:
        n = int(os.environ.get("TK8S_FAKE_GPUS", "0") or 0)
    ue = _faults()
    gpus = []
    for i in range(n):
        bad = ue.get(i, 0)
        gpus.append({
            "index": i, "pci_bus_id": f"0000:{0x10 + i:02x}:00.0", "market_name": "AMD Instinct MI355 OAM (fake)",
            "cu_count": 256, "oam_id": i, "temp_c": {"hotspot": 40 + i, "vram": 33},
            "power": {"current_w": 180 + i, "limit_w": 1400}, "vram_total_bytes": 309220868096,
            "vram_used_bytes": 297766912, "ecc": {"correctable": 0, "uncorrectable": bad, "deferred": 0},
            "activity": {"gfx_pct": 0, "umc_pct": 0}, "healthy": bad == 0, "unsupported": ["temp_edge"],
        })
    out = {"ok": n > 0, "healthy": all(g["healthy"] for g in gpus), "gpu_count": n, "amdsmi_version": "fake",
           "gpus": gpus, "ms": 0.0}
    if with_links:
        out["links"] = [[{"type": "self" if i == j else "xgmi", "hops": 0 if i == j else 1} for j in range(n)]
                        for i in range(n)]
    if not n:
        out["error"] = "AMD SMI found no GPU"
    return out


def main(argv: list[str] | None = None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    r = report(with_links="--no-links" not in argv)
    print(json.dumps(r, separators=(",", ":")))
    if not r["ok"]:
        return 3
    return 0 if r["healthy"] else 1


if __name__ == "__main__":
    sys.exit(main())
