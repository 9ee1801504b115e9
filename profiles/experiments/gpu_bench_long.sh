#!/usr/bin/env bash
# One gpurun call: the headline bench with more timed steps (steadier mean), then the default
# driver invocation (no flags) to confirm it finishes in bounds.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${1:-bench_long}"
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
echo "[gpu_bench_long] bench 20 steps" && timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 2 --keep-events "$OUT/events" --log "$OUT/bench_setup.log" > "$OUT/bench.json" 2> "$OUT/bench.err" &&
echo "[gpu_bench_long] bench defaults" && timeout -k 10 300 python3 bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" &&
echo "[gpu_bench_long] done"
