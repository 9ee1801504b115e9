#!/usr/bin/env bash
# One gpurun call: build, smoke, GPU tests, headline bench (1 GPU, per-step event logs), the
# validation payload's own timings, and rocprofv3 kernel stats of that payload.
# Every GPU step has its own time limit; steps are chained with && so a failure stops the call.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${1:-bench}"
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
BIN="$ROOT/tritonk8ssupervisor_amd/bin"
PROBE_ARGS=(--all-devices --gpuinfo --peers --hbm-bytes 1073741824 --md5-bytes 268435456 --iters 3)
echo "[gpu_bench] build" && timeout -k 10 300 python3 __graft_entry__.py build > "$OUT/build.log" 2>&1 &&
echo "[gpu_bench] smoke" && timeout -k 10 120 python3 __graft_entry__.py smoke > "$OUT/smoke.log" 2>&1 &&
echo "[gpu_bench] pytest -m gpu" && timeout -k 10 500 python3 -m pytest tests -m gpu -x -q > "$OUT/pytest_gpu.log" 2>&1 &&
echo "[gpu_bench] bench" && timeout -k 10 400 python3 bench.py --gpus 1 --steps "${STEPS:-5}" --warmup 1 --keep-events "$OUT/events" --log "$OUT/bench_setup.log" > "$OUT/bench.json" 2> "$OUT/bench.err" &&
echo "[gpu_bench] host profile" && timeout -k 10 120 python3 scripts/profile_setup.py > "$OUT/setup_profile.txt" 2>&1 &&
echo "[gpu_bench] probe" && timeout -k 10 60 "$BIN/tk8s-probe" "${PROBE_ARGS[@]}" > "$OUT/probe.json" &&
echo "[gpu_bench] rocprofv3 probe" && cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/prof_probe" -o probe --output-format csv -- "$BIN/tk8s-probe" "${PROBE_ARGS[@]}" > "$OUT/rocprof_probe.log" 2>&1 &&
echo "[gpu_bench] done"
