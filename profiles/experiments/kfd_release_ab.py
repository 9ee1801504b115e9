"""Does freeing the burn-in's queues and VRAM before exit (TK8S_PROBE_RELEASE=1) shorten the next
GPU process's runtime start? A = burn-in with/without the release, then after `gap_s` B = burn-in;
B's runtime_init is the figure (see profiles/r2_gap for the KFD release window)."""
import json
import os
import subprocess
import sys
import time

P = "tritonk8ssupervisor_amd/bin/tk8s-hsaprobe"
A = ["--all-devices", "--gpuinfo", "--peers", "--hbm-bytes", "1073741824", "--md5-bytes", "268435456", "--iters", "3"]


def run(cmd, env=None):
    t = time.monotonic()
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=60, env=env)
    return p.returncode, p.stdout, (time.monotonic() - t) * 1e3


reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
for r in range(reps):
    for gap in (0.0, 0.1):
        for release in ("0", "1"):
            time.sleep(1.5)
            rc, out_a, wall_a = run([P, *A], env={**os.environ, "TK8S_PROBE_RELEASE": release})
            ta = json.loads(out_a.strip().splitlines()[-1])["timings_ms"]
            time.sleep(gap)
            rc2, out, wall_b = run([P, *A])
            if rc != 0 or rc2 != 0:
                sys.exit(f"probe failed: {out_a[-300:]} {out[-300:]}")
            t = json.loads(out.strip().splitlines()[-1])["timings_ms"]
            print(json.dumps({"rep": r, "gap_s": gap, "release": release == "1",
                              "a_total_ms": ta["total"], "a_wall_ms": round(wall_a, 2),
                              "b_runtime_init": t["runtime_init"], "b_total": t["total"],
                              "b_wall_ms": round(wall_b, 2)}), flush=True)
