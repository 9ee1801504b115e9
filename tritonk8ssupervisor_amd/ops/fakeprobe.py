"""CPU stand-in for tk8s-probe when ``TK8S_FAKE_GPUS`` is set (tests on hosts without a GPU).

Emits the same JSON shape as native/tools/tk8s_probe.cpp and honours the same pipelining flags
(``--out FILE`` for the early burn-in, ``--reuse FILE [--reuse-wait S]`` for the validation
pod), so the validation DaemonSet, the node condition logic and the device-plugin refresh run
unchanged; never used on a GPU host (setup picks the real tool whenever TK8S_FAKE_GPUS is unset).
Test hooks: ``TK8S_FAKE_PROBE_FAIL=<node>`` fails, ``TK8S_FAKE_PROBE_HANG=<node>`` wedges,
``TK8S_FAKE_BURNIN_CRASH=<node>`` kills the early burn-in before it writes a result.
"""
import json
import os
import sys
import time


def _arg(name, default=None):
    a = sys.argv[1:]
    return a[a.index(name) + 1] if name in a and a.index(name) + 1 < len(a) else default


def _alive(pending):
    try:
        pid = int(open(pending).read().strip() or 0)
    except (OSError, ValueError):
        return True
    if pid <= 0:
        return True
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    except PermissionError:
        pass
    try:  # an exited burn-in its launcher has not reaped yet is a zombie: dead for our purpose
        with open(f"/proc/{pid}/stat") as f:
            return f.read().rsplit(")", 1)[1].split()[0] != "Z"
    except (OSError, IndexError):
        return True


def _reuse(path, wait):
    t = time.monotonic()
    while not os.path.exists(path) and os.path.exists(path + ".pending") and time.monotonic() - t < wait:
        if not _alive(path + ".pending") and not os.path.exists(path):
            break
        time.sleep(0.002)
    try:  # single-use (native/tools/reuse.h): take it atomically, then read it
        os.rename(path, path + ".consumed")
        with open(path + ".consumed") as f:
            text = f.read().strip()
    except OSError:
        return None
    if not text.startswith("{"):
        return None
    print(text)
    return 0 if json.loads(text).get("ok") else 1


def _emit(out, path):
    text = json.dumps(out)
    if path:
        with open(path + ".tmp", "w") as f:
            f.write(text + "\n")
        os.replace(path + ".tmp", path)
        try:
            os.remove(path + ".pending")
        except OSError:
            pass
    print(text)


def main():
    node = os.environ.get("NODE_NAME") or os.environ.get("TK8S_MACHINE", "-")
    # a failing (or wedged) node's GPU fails its own validation even when a (host-level) burn-in
    # result exists
    if os.environ.get("TK8S_FAKE_PROBE_HANG", "") == node:
        time.sleep(3600)  # a wedged validation (the analogue of the reference's stuck dashboard)
    if "--reuse" in sys.argv and os.environ.get("TK8S_FAKE_PROBE_FAIL", "") != node:
        rc = _reuse(_arg("--reuse"), float(_arg("--reuse-wait", "120")))
        if rc is not None:
            return rc
    if "--out" in sys.argv and os.environ.get("TK8S_FAKE_BURNIN_CRASH", "") == node:
        return 139  # the burn-in dies without a result; the validation pod must probe by itself
    if os.environ.get("TK8S_FAKE_PROBE_HANG", "") == node:
        time.sleep(3600)  # a wedged validation (the analogue of the reference's stuck dashboard)
    visible = [x for x in (os.environ.get("ROCR_VISIBLE_DEVICES") or os.environ.get("HIP_VISIBLE_DEVICES", "")).split(",") if x]
    n = len(visible)
    # the fake inventory's bus ids (models/hostinfo.py, ops/fakesmi.py: 0x10 + host ordinal), as
    # the real probe reports the devices' own: the agent joins probe, SMI and inventory on them
    bus = [0x10 + int(x) if x.isdigit() else i for i, x in enumerate(visible)]
    fail = os.environ.get("TK8S_FAKE_PROBE_FAIL", "") == node
    dev = {"ok": not fail, "hbm": {"ok": True, "gbps": 6200.0}, "md5": {"ok": True, "mbps": 2.3e6}}
    devices = [dict(dev, device=i) for i in range(n)]
    if "--peers" in sys.argv:  # every ordered pair, the shape of tk8s-hsaprobe --peers
        for i, d in enumerate(devices):
            d["peers"] = [{"ok": True, "probe": "xgmi_peer_pull", "src_device": j, "dst_device": i, "bytes": 32 << 20,
                           "iters": 2, "access": "allowed", "kernel_ms": 0.6, "kernel_gbps": 55.0 + 0.1 * ((i + j) % 5),
                           "bad_words": 0} for j in range(n) if j != i]
            d["peers_ok"] = True
    out = {"ok": not fail, "fake": True, "runtime": "fake", "device_count": n, "probed": n, "devices": devices,
           "hbm": dev["hbm"], "md5": dev["md5"],
           "gpuinfo": {"ok": True, "device_count": n, "devices": [{"index": i, "gfx": "gfx950", "pci_bus_id": f"0000:{bus[i]:02x}:00.0",
                                                                    "uuid": f"fake-{i}"} for i in range(n)]}}
    _emit(out, _arg("--out"))
    return 0 if not fail else 1


if __name__ == "__main__":
    sys.exit(main())
