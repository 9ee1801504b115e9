"""What makes hsa_init (the bulk of a HIP process's start) take 45 ms or 200 ms on this box?
Measures (1) its dependence on the gap since the previous GPU process exited, (2) how long that
process's KFD entry (/sys/class/kfd/kfd/proc/<pid>) outlives it, (3) a live GPU process held
open meanwhile, (4) 4 processes initialising at once. Writes gpurun_out/init_costs3/*.json."""
import json
import os
import subprocess
import sys
import time

OUT = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/init_costs3"
BIN = "/tmp/hsa_init_costs"
os.makedirs(OUT, exist_ok=True)
KFD = "/sys/class/kfd/kfd/proc"


def run():
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=60, check=True)
    return json.loads(r.stdout)["hsa_init_ms"]


def kfd_pids():
    try:
        return set(os.listdir(KFD))
    except OSError:
        return None


res = {"gaps": [], "kfd_linger_ms": [], "with_holder": [], "concurrent4": []}
time.sleep(3)
for gap in (0.0, 0.1, 0.25, 0.5, 0.75, 1.0, 1.5, 0.0, 0.1, 0.25, 0.5, 0.75, 1.0, 1.5):
    run()                       # the "previous" GPU process
    time.sleep(gap)
    res["gaps"].append({"gap_s": gap, "hsa_init_ms": run()})
    print(res["gaps"][-1], flush=True)

# how long does a finished process's KFD entry linger?
for _ in range(3):
    time.sleep(2)
    p = subprocess.Popen([BIN], stdout=subprocess.DEVNULL)
    pid = str(p.pid)
    p.wait()
    t = time.perf_counter()
    seen = kfd_pids()
    while seen is not None and pid in seen and time.perf_counter() - t < 5:
        time.sleep(0.002)
        seen = kfd_pids()
    res["kfd_linger_ms"].append(None if seen is None else round((time.perf_counter() - t) * 1000, 1))
    print("linger", res["kfd_linger_ms"][-1], flush=True)

# a live GPU process alongside
time.sleep(2)
h = subprocess.Popen([BIN, "hold", "8"], stdout=subprocess.PIPE, text=True)
h.stdout.readline()
time.sleep(2.5)
for _ in range(2):
    res["with_holder"].append(run())
    time.sleep(2)
h.wait()
print("holder", res["with_holder"], flush=True)

# four at once (each with a quiet KFD)
for _ in range(2):
    time.sleep(2.5)
    ps = [subprocess.Popen([BIN], stdout=subprocess.PIPE, text=True) for _ in range(4)]
    res["concurrent4"].append([json.loads(p.communicate(timeout=60)[0])["hsa_init_ms"] for p in ps])
    print("conc", res["concurrent4"][-1], flush=True)
json.dump(res, open(f"{OUT}/init_costs3.json", "w"), indent=1)
