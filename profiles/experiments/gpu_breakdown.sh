#!/usr/bin/env bash
# One gpurun call: where does bring-up time go on a real MI355X, and how fast are the streaming
# kernel shapes? Every GPU step has its own time limit; steps chained with &&.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${1:-breakdown}"
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
BIN="$ROOT/tritonk8ssupervisor_amd/bin"
echo "[bd] build" && timeout -k 10 300 python3 __graft_entry__.py build > "$OUT/build.log" 2>&1 &&
echo "[bd] variants" && /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -o /tmp/stream_variants native/bench/stream_variants.hip &&
timeout -k 10 120 /tmp/stream_variants 1024 256 20 > "$OUT/stream_variants.jsonl" 2> "$OUT/stream_variants.err" &&
echo "[bd] tool timings" && TIMEFORMAT="%R s" && { for i in 1 2 3; do echo -n "gpuinfo "; { time timeout -k 10 60 "$BIN/tk8s-gpuinfo" > /dev/null; } 2>&1; done; } > "$OUT/tool_times.txt" &&
{ for i in 1 2 3; do echo -n "probe "; { time timeout -k 10 60 "$BIN/tk8s-probe" --all-devices --gpuinfo --hbm-bytes 1073741824 --md5-bytes 268435456 --iters 3 > "$OUT/probe_$i.json"; } 2>&1; done; } >> "$OUT/tool_times.txt" &&
{ for i in 1 2 3; do echo -n "py-import-agent "; { time python3 -c "import tritonk8ssupervisor_amd.agent.agent"; } 2>&1; done; } >> "$OUT/tool_times.txt" &&
echo "[bd] bench" && timeout -k 10 400 python3 bench.py --gpus 1 --steps 3 --warmup 1 --keep-events "$OUT/events" --log "$OUT/bench_setup.log" > "$OUT/bench.json" 2> "$OUT/bench.err" &&
echo "[bd] done"
