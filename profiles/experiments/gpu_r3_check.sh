#!/usr/bin/env bash
# One gpurun call: GPU test suite, smoke, and a short headline bench on the current tree.
# Each GPU step has its own time limit; steps are chained with && so a failure stops the call.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${1:-r3check}"
STEPS="${2:-10}"
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
echo "[r3check] pytest -m gpu" &&
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest_gpu.log" 2>&1 &&
echo "[r3check] smoke" &&
timeout -k 10 300 python3 -c 'import __graft_entry__ as g; g.smoke()' > "$OUT/smoke.log" 2>&1 &&
echo "[r3check] bench" &&
timeout -k 10 600 python3 bench.py --gpus 1 --steps "$STEPS" --warmup 3 --log "$OUT/bench_setup.log" \
  > "$OUT/bench.json" 2> "$OUT/bench.err" &&
echo "[r3check] done"
