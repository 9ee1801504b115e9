set -euo pipefail
cd "$GRAFT_REPO_ROOT"
B=tritonk8ssupervisor_amd/bin
mkdir -p gpurun_out/hsaiters
for it in 3 30; do
  timeout -k 10 60 $B/tk8s-hsaprobe --hbm-bytes 1073741824 --md5-bytes 268435456 --iters $it > gpurun_out/hsaiters/hsa_$it.json
  sleep 1
  timeout -k 10 60 $B/tk8s-probe --hbm-bytes 1073741824 --md5-bytes 268435456 --iters $it > gpurun_out/hsaiters/hip_$it.json
  sleep 1
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/hsaiters/*.json")):
    d = json.load(open(f))
    print(f.rsplit("/",1)[1], "cold_ms", round(d["hbm"]["cold_ms"],3), "hbm", round(d["hbm"]["gbps"]), "read", round(d["hbm"]["read_gbps"]), "md5", round(d["md5"]["mbps"]), "fill", round(d["md5"]["fill_gbps"]), "copy", round(d["copy"]["kernel_gbps"]), "total", round(d["timings_ms"]["total"],1))
PY
