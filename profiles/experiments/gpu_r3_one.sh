#!/usr/bin/env bash
# One gpurun call: the named GPU tests only (pytest -k expression in $2), output under gpurun_out/$1.
set -uo pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${1:-r3one}"
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
echo "[r3one] pytest -m gpu -k $2" &&
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "$2" > "$OUT/pytest_gpu.log" 2>&1
rc=$?
echo "[r3one] rc=$rc"
exit $rc
