#!/usr/bin/env bash
# Round-3 feasibility probe on the 1-GPU box (one gpurun call):
#  1. can an unprivileged user + mount namespace re-shape the KFD topology and /dev/dri view
#     (the GPU isolation of tk8s pods)?  -> gpurun_out/r3probe/userns.log
#  2. where does tk8s-rccl's 1.8 s communicator start go at n=1?  NCCL_DEBUG=INFO lines stamped
#     on arrival + a rocprofv3 HIP API trace.  -> gpurun_out/r3probe/rccl_*.{log,json}, prof_rccl/
#  3. is /sys/class/kfd/kfd/proc readable (per-step KFD process census of bench.py)?
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${1:-r3probe}"
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
BIN="$ROOT/tritonk8ssupervisor_amd/bin"
{
  id; uname -r
  echo "--- sysctls"; for f in /proc/sys/kernel/unprivileged_userns_clone /proc/sys/user/max_user_namespaces \
    /proc/sys/kernel/apparmor_restrict_unprivileged_userns; do echo "$f=$(cat $f 2>&1)"; done
  echo "--- kfd"; ls -la /dev/kfd /dev/dri; readlink -f /sys/class/kfd/kfd; ls /sys/class/kfd/kfd/topology/nodes
  ls -la /sys/class/kfd/kfd/proc 2>&1 | head -20
  for n in /sys/class/kfd/kfd/topology/nodes/*; do echo "node $n gpu_id=$(cat $n/gpu_id) $(grep -E 'drm_render_minor|simd_count' $n/properties | tr '\n' ' ')"; ls $n; done
  echo "--- mounts"; grep -E ' /dev| /sys' /proc/self/mountinfo
  echo "--- unshare"; timeout -k 5 20 unshare -Urm sh -c 'id; mount -t tmpfs none /tmp && echo tmpfs-on-tmp-ok'; echo "rc=$?"
} > "$OUT/userns.log" 2>&1
timeout -k 5 30 python3 "$ROOT/profiles/experiments/r3_isolation_try.py" >> "$OUT/userns.log" 2>&1; echo "isolation try rc=$?" >> "$OUT/userns.log"
echo "[r3probe] userns done"
# RCCL start-up, stamped line by line
timeout -k 10 120 python3 "$ROOT/profiles/experiments/r3_stamp.py" "$OUT/rccl_info.log" NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=ALL -- \
  "$BIN/tk8s-rccl" --ngpus 1 --max-bytes 1048576 --factor 4 > "$OUT/rccl_info.json" &&
echo "[r3probe] rccl stamped done" &&
timeout -k 10 120 python3 "$ROOT/profiles/experiments/r3_stamp.py" "$OUT/rccl_plain.log" -- "$BIN/tk8s-rccl" --ngpus 1 --max-bytes 1048576 --factor 4 > "$OUT/rccl_plain.json" &&
cd /tmp && timeout -k 10 180 rocprofv3 --hip-trace --kernel-trace --stats -d "$OUT/prof_rccl" -o rccl --output-format csv -- \
  "$BIN/tk8s-rccl" --ngpus 1 --max-bytes 1048576 --factor 4 > "$OUT/rocprof_rccl.log" 2>&1 &&
echo "[r3probe] done"
