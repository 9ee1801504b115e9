"""CPU stand-in for tk8s-rccl's multi-process rendezvous (``TK8S_FAKE_GPUS`` test mode).

Exercises exactly the control-plane path of the real job: rank 0 publishes a unique id to the
KV store (PUT), the other ranks long-poll it (GET ?wait=), then every rank reports one JSON
line. No GPU, no RCCL.
"""
import argparse
import json
import secrets
import sys
import time
import urllib.request

ap = argparse.ArgumentParser()
ap.add_argument("--rank", type=int, required=True)
ap.add_argument("--nranks", type=int, required=True)
ap.add_argument("--kv-url", required=True)
a = ap.parse_args()
if a.rank == 0:
    uid = secrets.token_hex(128)
    urllib.request.urlopen(urllib.request.Request(a.kv_url, data=uid.encode(), method="PUT"), timeout=10).read()
else:
    deadline = time.monotonic() + 60
    uid = ""
    while time.monotonic() < deadline and len(uid) != 256:
        try:
            uid = urllib.request.urlopen(a.kv_url + "?wait=10", timeout=15).read().decode().strip()
        except OSError:
            time.sleep(0.02)
    if len(uid) != 256:
        print(json.dumps({"ok": False, "error": "no unique id"}))
        sys.exit(2)
print(json.dumps({"ok": True, "fake": True, "mode": "multi_process", "nranks": a.nranks, "rank": a.rank,
                  "peak_busbw_gbps": 0.0, "uid_prefix": uid[:8]}))
