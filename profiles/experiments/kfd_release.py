"""How long the kernel takes to release a KFD process after it exits, and what a new runtime start
pays when it begins before that release is done.

A: the burn-in (tk8s-hsaprobe, default bring-up arguments) runs and exits; the script polls
/sys/class/kfd/kfd/proc/<pid> until it disappears (the KFD process is gone) -> release_ms.
Then B starts either immediately after A's exit ("immediate"), or after the release ("after")
and reports its runtime_init.
"""
import json
import os
import subprocess
import sys
import time

P = "tritonk8ssupervisor_amd/bin/tk8s-hsaprobe"
A = ["--all-devices", "--gpuinfo", "--peers", "--hbm-bytes", "1073741824", "--md5-bytes", "268435456", "--iters", "3"]


def probe():
    t = time.monotonic()
    p = subprocess.Popen([P, *A], stdout=subprocess.PIPE, text=True)
    out, _ = p.communicate(timeout=60)
    if p.returncode != 0:
        sys.exit(f"probe failed rc={p.returncode}")
    return p.pid, time.monotonic(), json.loads(out.strip().splitlines()[-1])["timings_ms"]["runtime_init"], t


def wait_release(pid, since):
    d = f"/sys/class/kfd/kfd/proc/{pid}"
    seen = os.path.exists(d)
    while os.path.exists(d) and time.monotonic() - since < 3:
        time.sleep(0.0005)
    return seen, round((time.monotonic() - since) * 1e3, 2)


rows = []
print("proc dir:", os.path.isdir("/sys/class/kfd/kfd/proc"), flush=True)
for i in range(int(sys.argv[1]) if len(sys.argv) > 1 else 5):
    for mode in ("immediate", "after"):
        time.sleep(1.0)
        pid, t_exit, init_a, _ = probe()
        if mode == "after":
            seen, rel = wait_release(pid, t_exit)
        else:
            seen, rel = None, None
        pid_b, t_exit_b, init_b, t_b = probe()
        seen_b, rel_b = wait_release(pid_b, t_exit_b)
        rows.append({"mode": mode, "init_a": init_a, "release_a_ms": rel, "proc_dir_seen": seen,
                     "gap_ms": round((t_b - t_exit) * 1e3, 2), "init_b": init_b, "release_b_ms": rel_b})
        print(json.dumps(rows[-1]), flush=True)
print(json.dumps({"rows": rows}))
