#!/usr/bin/env bash
# What does mapping a shared library cost a payload process? Times the exec -> exit of
# empty programs linked against libamdhip64 only vs libamdhip64 + librccl (which the probe used
# to pull in through libtk8s.so), then the real tk8s-probe with and without a HIP runtime start.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${1:-loadcost}
mkdir -p "$out"
printf 'int main(){return 0;}\n' > /tmp/empty.cpp
printf '#include <hip/hip_runtime.h>\nint main(){int n=0; return hipGetDeviceCount(&n)!=hipSuccess;}\n' > /tmp/count.cpp
H=/opt/rocm/bin/hipcc
$H -O2 /tmp/empty.cpp -o /tmp/empty_hip -Wl,--no-as-needed -L/opt/rocm/lib -lamdhip64
$H -O2 /tmp/empty.cpp -o /tmp/empty_hip_rccl -Wl,--no-as-needed -L/opt/rocm/lib -lamdhip64 -lrccl
$H -O2 /tmp/count.cpp -o /tmp/count_hip -Wl,--no-as-needed -L/opt/rocm/lib -lamdhip64
$H -O2 /tmp/count.cpp -o /tmp/count_hip_rccl -Wl,--no-as-needed -L/opt/rocm/lib -lamdhip64 -lrccl
timeout -k 10 300 python3 - "$out" <<'PY'
import json, subprocess, sys, time
out = sys.argv[1]
res = {}
def t(cmd, n=6):
    ms = []
    for _ in range(n):
        s = time.perf_counter()
        subprocess.run(cmd, check=True, stdout=subprocess.DEVNULL)
        ms.append(round((time.perf_counter() - s) * 1000, 2))
    return ms
# interleave so page-cache warmth is shared fairly; the first entry of each is the cold one
for name in ("empty_hip_rccl", "empty_hip", "count_hip_rccl", "count_hip"):
    res[name] = t([f"/tmp/{name}"])
res["tk8s-probe(gpuinfo)"] = t(["tritonk8ssupervisor_amd/bin/tk8s-gpuinfo"], 4)
print(json.dumps(res, indent=1))
json.dump(res, open(f"{out}/loadcost.json", "w"), indent=1)
PY
