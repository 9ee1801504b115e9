#!/usr/bin/env bash
# Per-kernel durations of tk8s-hsaprobe (ROCr dispatch) and tk8s-probe (HIP) as rocprofv3 sees
# them: the same kernels, timed the same way, whatever runtime launched them.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
export TK8S_PROBE_CLEAN_EXIT=1
B=$GRAFT_REPO_ROOT/tritonk8ssupervisor_amd/bin
O=$GRAFT_REPO_ROOT/gpurun_out/hsaprof
mkdir -p "$O"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/hsa" -o run -- "$B/tk8s-hsaprobe" --hbm-bytes 1073741824 --md5-bytes 268435456 --iters 10 > "$O/hsa.json"
sleep 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/hip" -o run -- "$B/tk8s-probe" --hbm-bytes 1073741824 --md5-bytes 268435456 --iters 10 > "$O/hip.json"
for r in hsa hip; do
  f=$(find "$O/$r" -name '*kernel_stats.csv' | head -1)
  echo "== $r"; cut -d, -f1-4 "$f" | head -12
done
