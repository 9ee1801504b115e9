#!/usr/bin/env bash
# BASELINE.json config 5: hardware counters captured from the RCCL all-reduce pod, plus one
# counter pass over the validation payload's kernels. Counter passes carry --kernel-trace/--stats
# only, every step has its own hard time limit, and the steps are chained with &&.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/pmc"
mkdir -p "$OUT"
export TMPDIR=/tmp
COUNTERS="SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_VMEM_RD,SQ_INSTS_LDS,SQ_BUSY_CYCLES,GRBM_GUI_ACTIVE"
WS=$(mktemp -d /tmp/tk8s-pmc-XXXX)
python3 -c "import sys; sys.path.insert(0, '$ROOT'); from tritonk8ssupervisor_amd.orchestrator import init_workspace; init_workspace('$WS')"
cp "$ROOT/setup.sh" "$ROOT/tk8s" "$ROOT/kubectl" "$WS/"
cd "$WS"
echo "[pmc] RCCL pod counter pass"
PYTHONPATH="$ROOT" timeout -k 10 300 ./setup.sh --nodes 1 --yes --json --port 0 --timeout 120 --rccl on \
  --rccl-timeout 120 --rccl-max-bytes $((16 << 20)) --rocprof --rocprof-counters "$COUNTERS" > "$OUT/setup.log" 2>&1 &&
tail -1 "$OUT/setup.log" > "$OUT/setup_summary.json" &&
cp -r rocprof "$OUT/rccl_profiles" &&
PYTHONPATH="$ROOT" timeout -k 10 120 ./setup.sh -c --yes > /dev/null 2>&1 &&
cd /tmp &&
echo "[pmc] validation payload counter pass" &&
timeout -s KILL 90 rocprofv3 --pmc ${COUNTERS//,/ } --kernel-trace --stats -d "$OUT/probe" -o probe \
  --output-format csv -- "$ROOT/tritonk8ssupervisor_amd/bin/tk8s-probe" --hbm-bytes 1073741824 \
  --md5-bytes 268435456 --iters 3 > "$OUT/probe_stdout.json" 2> "$OUT/probe_rocprof.log" &&
echo "[pmc] done"
