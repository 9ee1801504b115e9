"""Does the size of the previous GPU process (the validation payload allocates ~1.3 GiB) set how
long its exit slows the next process's hsa_init? prev = tk8s-probe at validation size, at a small
size, and at validation size with an explicit free before exit; gaps 0.1-2 s."""
import json
import os
import subprocess
import sys
import time

OUT = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/init_costs4"
os.makedirs(OUT, exist_ok=True)
P = "tritonk8ssupervisor_amd/bin/tk8s-probe"
BIG = [P, "--gpuinfo", "--hbm-bytes", str(1 << 30), "--md5-bytes", str(256 << 20), "--iters", "3"]
SMALL = [P, "--hbm-bytes", str(16 << 20), "--md5-bytes", str(1 << 20), "--copy-bytes", str(1 << 20), "--iters", "1"]
PREVS = {"big": BIG, "small": SMALL, "big_release": BIG + ["--release-after"]}


def hsa_init():
    r = subprocess.run(["/tmp/hsa_init_costs"], capture_output=True, text=True, timeout=60, check=True)
    return json.loads(r.stdout)["hsa_init_ms"]


res = []
for rep in range(2):
    for name, cmd in PREVS.items():
        for gap in (0.1, 0.3, 0.6, 1.0, 2.0):
            time.sleep(2.0)
            t = time.perf_counter()
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=60)
            prev_ms = (time.perf_counter() - t) * 1000
            time.sleep(gap)
            row = {"prev": name, "gap_s": gap, "prev_rc": r.returncode, "prev_ms": round(prev_ms, 1),
                   "stderr": r.stderr.strip()[-200:], "hsa_init_ms": hsa_init()}
            res.append(row)
            print(json.dumps(row), flush=True)
json.dump(res, open(f"{OUT}/init_costs4.json", "w"), indent=1)
