"""Why a rebuild right after a teardown starts its GPU runtime slowly (bench.py back_to_back).

bench.py's back-to-back steps showed the new burn-in's runtime start at 80-150 ms instead of
~15 ms, ending exactly when the previous bring-up's KFD process (/sys/class/kfd/kfd/proc/<pid>)
went away. This measures, for the burn-in payload (tk8s-hsaprobe, the bring-up's own command):
  linger_ms    -- how long a probe's KFD process outlives the probe's exit (nothing else started);
  b2b_init_ms  -- the runtime start of a probe launched the moment the previous one exited;
  settled_ms   -- the same after a 1.5 s pause.
Variants: the shipped fast exit (_exit, no runtime teardown), TK8S_PROBE_CLEAN_EXIT=1 (return from
main), --release-after (queues and VRAM freed and hsa_shut_down after the result is written), and a
64 MiB arena instead of 1 GiB. Stops at the first failing probe.
Usage: python3 scripts/kfd_release_ab.py OUT_JSON [ROUNDS]"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
KFD = "/sys/class/kfd/kfd/proc"


def snap() -> set[str]:
    return {e for e in os.listdir(KFD) if e.isdigit()}


def run(cmd, env, watch=True):
    """Run one probe; returns (result json, new KFD entries seen while it ran, exit time)."""
    before = snap()
    out = tempfile.mktemp(suffix=".json")
    p = subprocess.Popen(cmd + ["--out", out], env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
    seen: set[str] = set()
    t_end = time.time() + 60
    while p.poll() is None:
        if watch:
            seen |= snap() - before
        if time.time() > t_end:
            p.kill()
            p.wait()
            raise SystemExit("probe timed out")
        time.sleep(0.001)
    t_exit = time.perf_counter()
    if p.returncode != 0:
        raise SystemExit(f"probe exit {p.returncode}: {p.stderr.read().decode()[-800:]}")
    with open(out) as f:
        res = json.load(f)
    os.unlink(out)
    return res, seen, t_exit


def linger(entries: set[str], t_exit: float, limit: float = 3.0) -> float | None:
    while time.perf_counter() - t_exit < limit:
        if not (entries & snap()):
            return round((time.perf_counter() - t_exit) * 1e3, 1)
        time.sleep(0.001)
    return None


def main() -> int:
    from tritonk8ssupervisor_amd.earlyburn import default_validation_command

    dest = sys.argv[1]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    base = default_validation_command(peers=False)
    small = default_validation_command(hbm_bytes=64 << 20, md5_bytes=16 << 20, peers=False)
    env0 = {k: v for k, v in os.environ.items() if k != "TK8S_PROBE_CLEAN_EXIT"}
    variants = {"fast_exit_1g": (base, env0), "clean_exit_1g": (base, dict(env0, TK8S_PROBE_CLEAN_EXIT="1")),
                "release_after_1g": (base + ["--release-after"], env0), "fast_exit_64m": (small, env0)}
    out: dict = {"command": base, "small_command": small, "rounds": rounds, "variants": {}}
    for r in range(rounds):
        for name, (cmd, env) in variants.items():
            rec = out["variants"].setdefault(name, {"linger_ms": [], "b2b_init_ms": [], "settled_init_ms": []})
            time.sleep(1.5)
            _, seen, t_exit = run(cmd, env)
            rec["linger_ms"].append(linger(seen, t_exit))
            time.sleep(1.5)
            run(cmd, env, watch=False)
            res, _, _ = run(cmd, env, watch=False)   # launched right after the previous exit
            rec["b2b_init_ms"].append(res.get("timings_ms", {}).get("runtime_init"))
            time.sleep(1.5)
            res, _, _ = run(cmd, env, watch=False)
            rec["settled_init_ms"].append(res.get("timings_ms", {}).get("runtime_init"))
            print(name, r, {k: v[-1] for k, v in rec.items()}, flush=True)
    with open(dest, "w") as f:
        json.dump(out, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
