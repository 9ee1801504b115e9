#!/usr/bin/env bash
# Round-3 probe 2 of the GPU jail: which denial makes ROCr's thunk give up on the allowed GPU?
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${1:-r3jail2}"
mkdir -p "$OUT"
cd "$ROOT"
BIN="$ROOT/tritonk8ssupervisor_amd/bin"
J="$BIN/tk8s-gpujail"
NODE=""; MINOR=""
for n in /sys/class/kfd/kfd/topology/nodes/*; do
  s=$(awk '$1=="simd_count"{print $2}' "$n/properties" 2>/dev/null)
  if [[ -n "$s" && "$s" != 0 ]]; then NODE=${n##*/}; MINOR=$(awk '$1=="drm_render_minor"{print $2}' "$n/properties"); fi
done
run() {  # title, jail args...
  local title="$1"; shift
  echo "=== $title"
  HSAKMT_DEBUG_LEVEL=7 timeout -k 5 60 "$J" "$@" -- "$BIN/tk8s-gpuinfo" --no-links 2>&1 | tail -25; echo "rc=$?"
}
{
  echo "gpu node=$NODE render=$MINOR"; ls -la /dev/dri /dev/kfd
  run "V0 no jail denials at all (roots that do not exist)" --kfd-root /nonexistent --dri-root /nonexistent
  run "V1 render nodes only, its GPU allowed" --kfd-root /nonexistent --allow-render "$MINOR"
  run "V2 topology only, its GPU allowed" --dri-root /nonexistent --allow-node "$NODE"
  run "V3 both, its GPU allowed" --allow-node "$NODE" --allow-render "$MINOR"
  run "V4 render nodes only, no GPU" --kfd-root /nonexistent
  echo "=== rocminfo under V3"; timeout -k 5 60 "$J" --allow-node "$NODE" --allow-render "$MINOR" -- /opt/rocm/bin/rocminfo 2>&1 | head -30
  echo "=== strace-free: what the thunk opens (ltrace unavailable): list of /sys/devices/virtual/kfd/kfd"
  ls -la /sys/devices/virtual/kfd/kfd /sys/devices/virtual/kfd/kfd/topology
} > "$OUT/jail2.log" 2>&1
echo "[r3jail2] done"
