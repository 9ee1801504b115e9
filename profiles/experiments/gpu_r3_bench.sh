#!/usr/bin/env bash
# One gpurun call: the driver's headline command (20 steps after 5 warm-up steps, per-step event
# logs), then rocprofv3 kernel stats of the burn-in payload (tk8s-hsaprobe, what N=1 runs).
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${1:-r3bench}"
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
BIN="$ROOT/tritonk8ssupervisor_amd/bin"
echo "[r3bench] bench" &&
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --keep-events "$OUT/events" --log "$OUT/bench_setup.log" \
  > "$OUT/bench.json" 2> "$OUT/bench.err" &&
echo "[r3bench] rocprofv3 hsaprobe" && cd /tmp && export TK8S_PROBE_CLEAN_EXIT=1 &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/prof_hsaprobe" -o hsaprobe --output-format csv -- \
  "$BIN/tk8s-hsaprobe" --all-devices --gpuinfo --hbm-bytes 1073741824 --md5-bytes 268435456 --iters 3 \
  > "$OUT/rocprof_hsaprobe.log" 2>&1 &&
echo "[r3bench] done"
