#!/usr/bin/env bash
# First light / A-B of tk8s-hsaprobe (ROCr direct) against tk8s-probe (HIP) on the GPU box:
# a small run whose MD5 tree digest is checked against the host oracle, then full-size runs of
# both tools alternating, each under its own time limit. Output: gpurun_out/hsaprobe/.
set -euo pipefail
cd "$(dirname "$0")/.."
out=gpurun_out/hsaprobe
mkdir -p "$out"
B=tritonk8ssupervisor_amd/bin
timeout -k 10 60 "$B/tk8s-hsaprobe" --hbm-bytes 16777216 --md5-bytes 1048576 --copy-bytes 1048576 --iters 1 > "$out/small.json"
python3 - "$out/small.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
assert d["ok"], d
assert d["md5"]["digest"] == "7d164cf2f6284ee704cb26209536fcb8", d["md5"]
print("small ok", d["timings_ms"], file=sys.stderr)
PY
for i in 1 2 3; do
  timeout -k 10 60 "$B/tk8s-hsaprobe" --all-devices --gpuinfo --hbm-bytes 1073741824 --md5-bytes 268435456 --iters 3 > "$out/hsa_$i.json"
  sleep 1
  timeout -k 10 60 "$B/tk8s-probe" --all-devices --gpuinfo --hbm-bytes 1073741824 --md5-bytes 268435456 --iters 3 > "$out/hip_$i.json"
  sleep 1
done
python3 - "$out" <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/h*_*.json")):
    d = json.load(open(f))
    dev = d["devices"][0]
    print(f.rsplit("/", 1)[1], "ok", d["ok"], "total_ms", round(d["timings_ms"]["total"], 1), "init_ms", round(d["timings_ms"]["hip_init"], 1),
          "hbm", round(d["hbm"]["gbps"]), "read", round(d["hbm"].get("read_gbps", 0)), "md5", round(d["md5"]["mbps"]),
          "copy", round(d["copy"]["kernel_gbps"]), "digest", d["md5"]["digest"] == d["md5_expected"],
          "host_ms", d["hbm"].get("host_ms"))
PY
