#!/usr/bin/env python3
"""How does a GPU process's runtime start scale when k validation payloads start together?

At N workers the bring-up starts N burn-ins (tk8s-probe, one per worker GPU) at once. On the
8-GPU node each uses its own GPU; on the 1-GPU box they share one, so this measures the
host-side part of the contention (KFD open, topology, queue creation serialised in the driver)
as an upper bound. For k in 1, 2, 4, 8: launch k probes at the same instant (small buffers),
collect each one's ``timings_ms`` and the wall time until the last exits; settle 1.5 s between
rounds so no round sees the previous one's teardown. Output: one JSON document.
"""
from __future__ import annotations

import json
import statistics
import subprocess
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
PROBE = REPO / "tritonk8ssupervisor_amd" / "bin" / "tk8s-probe"
ARGS = ["--hbm-bytes", str(64 << 20), "--md5-bytes", str(16 << 20), "--copy-bytes", str(16 << 20), "--iters", "1"]


def round_(k: int) -> dict:
    t0 = time.perf_counter()
    procs = [subprocess.Popen([str(PROBE), *ARGS], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
             for _ in range(k)]
    outs = [p.communicate(timeout=60) for p in procs]
    wall = (time.perf_counter() - t0) * 1000
    res = []
    for (out, err), p in zip(outs, procs):
        try:
            res.append(json.loads(out.strip().splitlines()[-1]))
        except (ValueError, IndexError):
            res.append({"ok": False, "rc": p.returncode, "err": err[-300:]})
    inits = [r.get("timings_ms", {}).get("hip_init") for r in res if r.get("timings_ms")]
    totals = [r.get("timings_ms", {}).get("total") for r in res if r.get("timings_ms")]
    return {"k": k, "wall_ms": round(wall, 1), "ok": all(r.get("ok") for r in res),
            "hip_init_ms": inits, "total_ms": totals,
            "hip_init_median": round(statistics.median(inits), 1) if inits else None,
            "hip_init_max": round(max(inits), 1) if inits else None}


def main() -> int:
    out = {"probe": str(PROBE), "args": ARGS, "rounds": []}
    time.sleep(1.5)
    for k in (1, 2, 4, 8, 1, 2, 4, 8):
        r = round_(k)
        out["rounds"].append(r)
        print(f"k={k}: wall {r['wall_ms']} ms, hip_init median {r['hip_init_median']} max {r['hip_init_max']} ms, "
              f"ok={r['ok']}", file=sys.stderr, flush=True)
        time.sleep(1.5)
    print(json.dumps(out, indent=1))
    return 0 if all(r["ok"] for r in out["rounds"]) else 1


if __name__ == "__main__":
    sys.exit(main())
