#!/usr/bin/env bash
# Diagnostics on the GPU box: which modules does the CLI compile from source, and how long do
# the HIP-free steps take there.
set -euo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${1:-diag}"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 300 python3 __graft_entry__.py build > "$OUT/build.log" 2>&1
id > "$OUT/id.txt"; ls -la tritonk8ssupervisor_amd/__pycache__ | head -5 >> "$OUT/id.txt"
python3 -c "import sys; print(sys.flags, sys.pycache_prefix)" >> "$OUT/id.txt"
env | grep -i "^PYTHON" >> "$OUT/id.txt" || true
python3 -S -v -c "import tritonk8ssupervisor_amd.orchestrator, tritonk8ssupervisor_amd.playbook, tritonk8ssupervisor_amd.playbook_modules" > "$OUT/imports_v.txt" 2>&1
grep "code object from" "$OUT/imports_v.txt" | grep -v "\.pyc'" > "$OUT/compiled_from_source.txt" || true
wc -l "$OUT/compiled_from_source.txt"
