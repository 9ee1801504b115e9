#!/usr/bin/env bash
# One gpurun call: GPU test suite, smoke, a short headline bench, and a rocprofv3 kernel-stats
# pass over the validation probe, all on the current tree.
# Each GPU step has its own time limit; steps are chained with && so a failure stops the call.
#   scripts/gpu_round_check.sh <out-name> [bench-steps]
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${1:-check}"
STEPS="${2:-10}"
BIN="$ROOT/tritonk8ssupervisor_amd/bin"
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
echo "[check] pytest -m gpu" &&
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest_gpu.log" 2>&1 &&
echo "[check] smoke" &&
timeout -k 10 300 python3 -c 'import __graft_entry__ as g; g.smoke()' > "$OUT/smoke.log" 2>&1 &&
echo "[check] bench" &&
timeout -k 10 900 python3 bench.py --gpus 1 --steps "$STEPS" --warmup 3 --log "$OUT/bench_setup.log" \
  > "$OUT/bench.json" 2> "$OUT/bench.err" &&
echo "[check] rocprofv3 probe" &&
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/prof_probe" -o probe --output-format csv \
  -- "$BIN/tk8s-probe" --iters 10 > "$OUT/rocprof_probe.log" 2>&1 &&
echo "[check] done"
