"""CPU stand-in for tk8s-probe when ``TK8S_FAKE_GPUS`` is set (tests on hosts without a GPU).

Emits the same JSON shape as native/tools/tk8s_probe.cpp so the validation DaemonSet, the
node condition logic and the device-plugin refresh run unchanged; never used on a GPU host
(setup picks the real tool whenever TK8S_FAKE_GPUS is unset).
"""
import json
import os
import time

n = len([x for x in os.environ.get("HIP_VISIBLE_DEVICES", "").split(",") if x])
fail = os.environ.get("TK8S_FAKE_PROBE_FAIL", "") == os.environ.get("NODE_NAME", "-")
if os.environ.get("TK8S_FAKE_PROBE_HANG", "") == os.environ.get("NODE_NAME", "-"):
    time.sleep(3600)  # a wedged validation pod (the analogue of the reference's stuck dashboard)
dev = {"ok": not fail, "hbm": {"ok": True, "gbps": 4400.0}, "md5": {"ok": True, "mbps": 2.3e6}}
out = {"ok": not fail, "fake": True, "device_count": n, "devices": [dev] * n, "hbm": dev["hbm"], "md5": dev["md5"],
       "gpuinfo": {"ok": True, "device_count": n, "devices": [{"index": i, "gfx": "gfx950", "pci_bus_id": f"0000:{i:02x}:00.0",
                                                                "uuid": f"fake-{i}"} for i in range(n)]}}
print(json.dumps(out))
raise SystemExit(0 if not fail else 1)
