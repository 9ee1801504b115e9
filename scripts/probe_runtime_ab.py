"""The burn-in payload on its two runtimes, settled (1.5 s apart, so no process waits for the
previous one's KFD release): tk8s-hsaprobe (ROCr directly; the 1-GPU burn-in) against
tk8s-probe (HIP; the multi-GPU burn-in, for its xGMI pulls). Same checks, same sizes.
Usage: python3 scripts/probe_runtime_ab.py OUT_JSON [ROUNDS]"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main() -> int:
    from tritonk8ssupervisor_amd.earlyburn import BIN, default_validation_command

    dest = sys.argv[1]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    base = default_validation_command(peers=False)[1:]
    tools = {"hsa": os.path.join(BIN, "tk8s-hsaprobe"), "hip": os.path.join(BIN, "tk8s-probe")}
    out: dict = {"args": base, "runs": {k: [] for k in tools}}
    for r in range(rounds):
        for name, tool in tools.items():
            time.sleep(1.5)
            res = tempfile.mktemp(suffix=".json")
            t = time.perf_counter()
            p = subprocess.run([tool, *base, "--out", res], capture_output=True, text=True, timeout=60)
            wall = (time.perf_counter() - t) * 1e3
            if p.returncode != 0:
                raise SystemExit(f"{name} exit {p.returncode}: {p.stderr[-800:]}")
            with open(res) as f:
                d = json.load(f)
            os.unlink(res)
            tm = d.get("timings_ms", {})
            rec = {"wall_ms": round(wall, 2), "runtime_init_ms": tm.get("runtime_init", tm.get("hip_init")),
                   "total_ms": tm.get("total"), "device_wall_ms": [x.get("wall_ms") for x in d.get("devices", [])]}
            out["runs"][name].append(rec)
            print(name, r, rec, flush=True)
    with open(dest, "w") as f:
        json.dump(out, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
