"""Why is the burn-in's HIP start fast in the bench's first step and slower afterwards? Times
hsa_init of a fresh process (1 s apart) (a) alone, (b) while this process holds a torch/HIP
context and synchronises before each spawn (what bench.py does), (c) same but right after
a torch process exits."""
import json
import os
import subprocess
import sys
import time

OUT = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/init_costs5"
os.makedirs(OUT, exist_ok=True)


def hsa_init():
    r = subprocess.run(["/tmp/hsa_init_costs"], capture_output=True, text=True, timeout=60, check=True)
    return json.loads(r.stdout)["hsa_init_ms"]


res = {"alone": [], "with_torch": [], "probe_alone": [], "probe_with_torch": []}
PROBE = ["tritonk8ssupervisor_amd/bin/tk8s-probe", "--gpuinfo", "--iters", "3"]


def probe_init():
    r = subprocess.run(PROBE, capture_output=True, text=True, timeout=60)
    return json.loads(r.stdout)["timings_ms"]["hip_init"]


time.sleep(2)
for _ in range(5):
    res["alone"].append(hsa_init())
    time.sleep(1)
for _ in range(4):
    res["probe_alone"].append(probe_init())
    time.sleep(1)
print("alone", res["alone"], res["probe_alone"], flush=True)
import torch  # noqa: E402

x = torch.ones(1 << 20, device="cuda")
torch.cuda.synchronize()
time.sleep(2)
for _ in range(5):
    torch.cuda.synchronize()
    res["with_torch"].append(hsa_init())
    time.sleep(1)
for _ in range(4):
    torch.cuda.synchronize()
    res["probe_with_torch"].append(probe_init())
    time.sleep(1)
print("with torch", res["with_torch"], res["probe_with_torch"], flush=True)
json.dump(res, open(f"{OUT}/init_costs5.json", "w"), indent=1)
