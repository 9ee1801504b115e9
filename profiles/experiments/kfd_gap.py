"""Runtime start of a burn-in B as a function of the gap since a previous GPU process A exited.
A is the burn-in itself (tk8s-hsaprobe, bring-up arguments) or tk8s-smi (AMD SMI, no HSA)."""
import json
import subprocess
import sys
import time

P = "tritonk8ssupervisor_amd/bin/tk8s-hsaprobe"
S = "tritonk8ssupervisor_amd/bin/tk8s-smi"
A = ["--all-devices", "--gpuinfo", "--peers", "--hbm-bytes", "1073741824", "--md5-bytes", "268435456", "--iters", "3"]


def run(cmd):
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=60)
    return p.returncode, p.stdout


reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
for r in range(reps):
    for first, gap in [("probe", 0), ("probe", 0.05), ("probe", 0.1), ("probe", 0.2), ("probe", 0.35), ("probe", 0.6),
                       ("probe", 1.0), ("smi", 0), ("none", 0)]:
        time.sleep(1.5)
        if first == "probe":
            rc, _ = run([P, *A])
        elif first == "smi":
            rc, _ = run([S, "--no-links"])
        else:
            rc = 0
        time.sleep(gap)
        rc2, out = run([P, *A])
        if rc2 != 0:
            sys.exit(f"probe failed: {out[-300:]}")
        t = json.loads(out.strip().splitlines()[-1])["timings_ms"]
        print(json.dumps({"rep": r, "first": first, "first_rc": rc, "gap_s": gap, "runtime_init": t["runtime_init"],
                          "total": t["total"]}), flush=True)
