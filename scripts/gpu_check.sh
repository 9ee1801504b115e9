#!/usr/bin/env bash
# One gpurun call: build, GPU tests, native probes, RCCL n=1, rocprofv3 kernel stats.
# Every GPU step has its own time limit; steps are chained with && so a failure stops the call.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${1:-check}"
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
BIN="$ROOT/tritonk8ssupervisor_amd/bin"
echo "[gpu_check] build" && timeout -k 10 300 python3 __graft_entry__.py build > "$OUT/build.log" 2>&1 &&
echo "[gpu_check] gpuinfo" && timeout -k 10 60 "$BIN/tk8s-gpuinfo" > "$OUT/gpuinfo.json" &&
echo "[gpu_check] pytest -m gpu" && timeout -k 10 400 python3 -m pytest tests -m gpu -x -q > "$OUT/pytest_gpu.log" 2>&1 &&
echo "[gpu_check] probe" && timeout -k 10 120 "$BIN/tk8s-probe" --iters 10 > "$OUT/probe.json" &&
echo "[gpu_check] probe plain" && timeout -k 10 120 "$BIN/tk8s-probe" --iters 10 --mode plain --skip-md5 > "$OUT/probe_plain.json" &&
echo "[gpu_check] rccl n=1" && timeout -k 10 120 "$BIN/tk8s-rccl" --ngpus 1 --max-bytes 268435456 --factor 4 > "$OUT/rccl1.json" &&
echo "[gpu_check] rocprofv3" && cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/prof_probe" -o probe --output-format csv -- "$BIN/tk8s-probe" --iters 10 > "$OUT/rocprof_probe.log" 2>&1 &&
echo "[gpu_check] done"
