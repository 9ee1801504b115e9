"""Which HIP runtime allocation makes the first stream cost ~20 ms (queue ~10 ms + a 16 MiB pinned
host buffer ~10 ms)? Runs native/bench/init_costs with one runtime knob at a time; records the
stream timings and the sizes of the runtime's own allocations (AMD_LOG_LEVEL=4)."""
import json
import os
import re
import subprocess
import sys
import time

OUT = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/stream_knobs"
os.makedirs(OUT, exist_ok=True)
VARIANTS = {
    "base": {},
    "staging1": {"GPU_STAGING_BUFFER_SIZE": "1"},
    "xfer1": {"GPU_XFER_BUFFER_SIZE": "1"},
    "pinned_xfer1": {"GPU_PINNED_XFER_SIZE": "1"},
    "kernarg_pool64k": {"HSA_KERNARG_POOL_SIZE": "65536"},
    "signal_pool64": {"ROC_SIGNAL_POOL_SIZE": "64"},
    "sysmem_pool0": {"DEBUG_CLR_SYSMEM_POOL": "0"},
    "aql1024": {"ROC_AQL_QUEUE_SIZE": "1024"},
    "dev_kernarg0": {"HIP_FORCE_DEV_KERNARG": "0"},
}
ALLOC = re.compile(r"Allocate hsa (host|device) memory \S+, size (0x[0-9a-f]+)")
res = {}
for name, env in VARIANTS.items():
    e = dict(os.environ, **env)
    runs = []
    for _ in range(2):
        time.sleep(0.5)
        r = subprocess.run(["/tmp/init_costs"], env=e, capture_output=True, text=True, timeout=60)
        runs.append(json.loads(r.stdout) if r.returncode == 0 else {"rc": r.returncode, "err": r.stderr[-300:]})
    time.sleep(0.5)
    log = subprocess.run(["/tmp/init_costs"], env=dict(e, AMD_LOG_LEVEL="4"), capture_output=True, text=True,
                         timeout=60)
    allocs = [(k, int(s, 16)) for k, s in ALLOC.findall(log.stdout + log.stderr)]
    res[name] = {"env": env, "runs": runs, "allocs": allocs}
    print(name, [(r.get("set_device_stream_ms"), r.get("second_stream_ms")) for r in runs],
          [(k, s >> 10) for k, s in allocs if s < (1 << 30)], flush=True)
json.dump(res, open(f"{OUT}/stream_knobs.json", "w"), indent=1)
