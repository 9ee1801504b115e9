"""exec -> main cost of the burn-in payload and of minimal programs linking the same runtime,
spawned the way earlyburn spawns the burn-in (posix_spawn, setsid). 10 rounds, interleaved."""
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
progs = {"plain": [os.path.join(REPO, "build/stamp_plain")], "hsa_linked": [os.path.join(REPO, "build/stamp_hsa")],
         "hsa_linked_static_cxx": [os.path.join(REPO, "build/stamp_hsa_static")]}
for lib in ("rocprofiler-register", "drm", "drm_amdgpu", "numa", "elf"):
    if os.path.exists(os.path.join(REPO, f"build/stamp_{lib}")):
        progs[lib] = [os.path.join(REPO, f"build/stamp_{lib}")]
ENVS = {"hsa_linked_register_off": {"ROCPROFILER_REGISTER_ENABLED": "0"}}
for name, extra in ENVS.items():
    progs[name] = [os.path.join(REPO, "build/stamp_hsa")]
out = {k: [] for k in progs}
for r in range(10):
    for name, cmd in progs.items():
        rd, wr = os.pipe()
        t = time.time()
        pid = os.posix_spawn(cmd[0], cmd, {**os.environ, **ENVS.get(name, {})}, setsid=True,
                             file_actions=[(os.POSIX_SPAWN_DUP2, wr, 1)])
        os.close(wr)
        data = os.read(rd, 100)
        os.close(rd)
        os.waitpid(pid, 0)
        out[name].append(round(float(data.decode().strip()) - t * 1e3, 3))
        time.sleep(0.05)
summary = {k: {"median_ms": sorted(v)[len(v) // 2], "all": v} for k, v in out.items()}
json.dump(summary, open(sys.argv[1], "w"), indent=1)
print(json.dumps({k: v["median_ms"] for k, v in summary.items()}))
